#!/bin/bash
# 64-row (8 x 2 x 4) vs 128-row symmetric tiles vs full storage on z slabs of
# config 2 (1/8, 1/4, 1/2) and config 2 itself, with the product library and
# with the uncapped-SGPR build (tools/libkle_nocap.so: make -C pynama_amd/csrc
# OBJDIR=build_nocap OUT=../../tools/libkle_nocap.so
# HIPFLAGS="--offload-arch=gfx950 -munsafe-fp-atomics -DSYM_XL_SGPRS=128").
# JSON lines on stdout.
set -e
V='[{},{"spmv_sym_tile64":1},{"spmv_sym":0}]'
for lib in pynama_amd/libkle.so tools/libkle_nocap.so; do
  for ne in 20,16,2 20,16,4 20,16,8 20,16,16; do
    its=100; [ $ne = 20,16,16 ] && its=40
    echo "{\"lib\": \"$lib\", \"nelem\": \"$ne\"}"
    KLE_LIBRARY=$PWD/$lib timeout -k 10 300 python -u tools/spmv_ab.py "$V" --nelem $ne --reps 4 --its $its
  done
done
# config 4 (p = 6): 8 x 8 x 2 tiles on 16 waves (one workgroup per CU) vs 64-row tiles on 8 waves (two per CU)
for lib in pynama_amd/libkle.so tools/libkle_nocap.so; do
  echo "{\"lib\": \"$lib\", \"nelem\": \"18,18,18 ngl 7\"}"
  KLE_LIBRARY=$PWD/$lib timeout -k 10 400 python -u tools/spmv_ab.py '[{},{"spmv_sym_tile64":1}]' --nelem 18,18,18 --ngl 7 --reps 3 --its 20
done
