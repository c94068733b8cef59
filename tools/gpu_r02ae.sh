#!/bin/bash
# Round 2: capped update / dot grids (1024 / 512) for both CG loops; KSP + multirank GPU tests; cg vs pipecg
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ae
export TMPDIR=/tmp
step gpu_ksp_tests 700 python -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
V='[{"_ksp":"cg"},{"_ksp":"pipecg"}]'
step ab_full 400 python tools/cg_ab.py "$V" --reps 5 --its 200 || exit 1
cp gpurun_out/ab_full.log gpurun_out/r02ae/cg_pipe_full.jsonl
step ab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 5 --its 500 || exit 1
cp gpurun_out/ab_eighth.log gpurun_out/r02ae/cg_pipe_eighth.jsonl
echo done
