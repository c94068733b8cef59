#!/bin/bash
# Round 2: one-rank pipecg, reduction beside (auto LDS cap) vs before the SpMV; cg reference
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02l
export TMPDIR=/tmp
V='[{"_ksp":"cg"},{"_ksp":"pipecg","pipe_side1":1},{"_ksp":"pipecg","pipe_side1":0},{"_ksp":"pipecg","pipe_side1":1,"spmv_dyn_lds":0}]'
step cgab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 5 --its 1000 || exit 1
cp gpurun_out/cgab_eighth.log gpurun_out/r02l/pipe_side_eighth.jsonl
step cgab_quarter 400 python tools/cg_ab.py "$V" --nelem 20,16,4 --reps 5 --its 500 || exit 1
cp gpurun_out/cgab_quarter.log gpurun_out/r02l/pipe_side_quarter.jsonl
step cgab_full 400 python tools/cg_ab.py "$V" --reps 4 --its 200 || exit 1
cp gpurun_out/cgab_full.log gpurun_out/r02l/pipe_side_full.jsonl
echo done
