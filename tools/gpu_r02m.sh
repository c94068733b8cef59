#!/bin/bash
# Round 2: XCD-chunked SpMV row mapping, box and unstructured 1M-DoF meshes (+ PMC fetch on unstructured)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02m
export TMPDIR=/tmp
V='[{"spmv_xcd_chunk":0},{"spmv_xcd_chunk":4},{"spmv_xcd_chunk":16},{"spmv_xcd_chunk":64}]'
step xcd_umesh 400 python tools/cg_ab.py "$V" --mesh unstructured --reps 4 --its 200 || exit 1
cp gpurun_out/xcd_umesh.log gpurun_out/r02m/xcd_chunk_umesh.jsonl
step xcd_box 400 python tools/cg_ab.py "$V" --reps 4 --its 200 || exit 1
cp gpurun_out/xcd_box.log gpurun_out/r02m/xcd_chunk_box.jsonl
step xcd_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 4 --its 1000 || exit 1
cp gpurun_out/xcd_eighth.log gpurun_out/r02m/xcd_chunk_eighth.jsonl
echo done
