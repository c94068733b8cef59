#!/bin/bash
# Round 2: pipelined CG with the scalar stage in the next update's prologue (two launches per iteration
# on one rank); KSP GPU tests; cg vs pipecg A/B
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02aa
export TMPDIR=/tmp
step gpu_ksp_tests 700 python -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_umesh.py -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
V='[{"_ksp":"cg"},{"_ksp":"pipecg"}]'
step ab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 6 --its 500 || exit 1
cp gpurun_out/ab_eighth.log gpurun_out/r02aa/pipe_prologue_eighth.jsonl
step ab_quarter 400 python tools/cg_ab.py "$V" --nelem 20,16,4 --reps 5 --its 300 || exit 1
cp gpurun_out/ab_quarter.log gpurun_out/r02aa/pipe_prologue_quarter.jsonl
step ab_full 400 python tools/cg_ab.py "$V" --reps 5 --its 200 || exit 1
cp gpurun_out/ab_full.log gpurun_out/r02aa/pipe_prologue_full.jsonl
step prof_eighth 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02aa/prof_eighth -o eighth --output-format csv -- python3 bench.py --nelem 20,16,2 --steps 500 --warmup 20 --no-cpu-baseline --no-aij --ksp pipecg || exit 1
echo done
