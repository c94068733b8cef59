#!/bin/bash
# Round 2: split rows over 2 / 4 waves (tail of the SpMV grid) vs one wave per row, per slab size
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02y
export TMPDIR=/tmp
V='[{"spmv_split":1},{"spmv_split":2},{"spmv_split":4}]'
step split_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 5 --its 500 || exit 1
cp gpurun_out/split_eighth.log gpurun_out/r02y/split_eighth.jsonl
step split_quarter 400 python tools/cg_ab.py "$V" --nelem 20,16,4 --reps 5 --its 300 || exit 1
cp gpurun_out/split_quarter.log gpurun_out/r02y/split_quarter.jsonl
step split_half 400 python tools/cg_ab.py "$V" --nelem 20,16,8 --reps 4 --its 200 || exit 1
cp gpurun_out/split_half.log gpurun_out/r02y/split_half.jsonl
step split_full 400 python tools/cg_ab.py "$V" --reps 4 --its 200 || exit 1
cp gpurun_out/split_full.log gpurun_out/r02y/split_full.jsonl
step split_um 400 python tools/cg_ab.py "$V" --mesh unstructured --reps 4 --its 200 || exit 1
cp gpurun_out/split_um.log gpurun_out/r02y/split_umesh.jsonl
echo done
