#!/bin/bash
# Symmetric vs full storage on 1/8-size parts (the N = 8 per-rank share), one
# GPU: the unstructured mesh (graph symmetric kernel at 64 / 32-row groups vs
# the full-storage kernel the size gets by default, and with dictionaries),
# and the box slab inside the pipelined CG (64-row tiles vs full storage).
set -e
echo '{"part": "unstructured 20,16,2, default dictionaries threshold"}'
timeout -k 10 300 python -u tools/spmv_ab.py '[{},{"spmv_gsym_rows":32},{"spmv_sym":0}]' --mesh unstructured --nelem 20,16,2 --reps 4 --its 100
echo '{"part": "unstructured 20,16,2, dictionaries at every size"}'
KLE_SPMV_DICT_MIN_ROWS=0 timeout -k 10 300 python -u tools/spmv_ab.py '[{},{"spmv_sym":0}]' --mesh unstructured --nelem 20,16,2 --reps 4 --its 100
echo '{"part": "box 20,16,2 pipelined CG"}'
KLE_SPMV_SYM_MIN_ROWS=0 timeout -k 10 300 python -u tools/cg_ab.py '[{},{"spmv_sym":0}]' --nelem 20,16,2 --ksp pipecg --reps 4 --its 200
