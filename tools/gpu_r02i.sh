#!/bin/bash
# Round 2: high-priority comm stream; pipecg (reduction beside the SpMV) vs cg again
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
V='[{"_ksp":"cg"},{"_ksp":"pipecg"}]'
step cgab_eighth 300 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 6 --its 1000 || exit 1
cp gpurun_out/cgab_eighth.log gpurun_out/r02i/cg_vs_pipecg_eighth.jsonl
step cgab_full 400 python tools/cg_ab.py "$V" --reps 6 --its 200 || exit 1
cp gpurun_out/cgab_full.log gpurun_out/r02i/cg_vs_pipecg_full.jsonl
step prof_eighth_pipe 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02i/prof_eighth_pipe -o eighth --output-format csv -- python3 bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline --no-aij --ksp pipecg || exit 1
step gpu_mr_tests 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
echo done
