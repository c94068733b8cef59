#!/bin/bash
# Round 2: SpMV workgroups per CU capped by unused dynamic LDS -> does the side-stream reduction co-run?
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02k
export TMPDIR=/tmp
V='[{"_ksp":"cg","spmv_dyn_lds":0},{"_ksp":"pipecg","spmv_dyn_lds":0},{"_ksp":"pipecg","spmv_dyn_lds":21504},{"_ksp":"pipecg","spmv_dyn_lds":27648},{"_ksp":"cg","spmv_dyn_lds":21504}]'
step cgab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 4 --its 1000 || exit 1
cp gpurun_out/cgab_eighth.log gpurun_out/r02k/lds_cap_eighth.jsonl
V2='[{"_ksp":"cg","spmv_dyn_lds":0},{"_ksp":"pipecg","spmv_dyn_lds":0},{"_ksp":"pipecg","spmv_dyn_lds":41984}]'
step cgab_full 400 python tools/cg_ab.py "$V2" --reps 4 --its 200 || exit 1
cp gpurun_out/cgab_full.log gpurun_out/r02k/lds_cap_full.jsonl
echo done
