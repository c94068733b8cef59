#!/bin/bash
# Round 2: single-reduction CG with the stage in the next update's prologue (one rank); full GPU suite;
# A/B against the k_dot_finish loop; default bench
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ab
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
V='[{"_ksp":"cg","sr_prologue":1},{"_ksp":"cg","sr_prologue":0},{"_ksp":"pipecg"}]'
step ab_full 400 python tools/cg_ab.py "$V" --reps 6 --its 200 || exit 1
cp gpurun_out/ab_full.log gpurun_out/r02ab/sr_prologue_full.jsonl
step ab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 6 --its 500 || exit 1
cp gpurun_out/ab_eighth.log gpurun_out/r02ab/sr_prologue_eighth.jsonl
step bench_default 600 python bench.py || exit 1
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02ab/bench_default.json
echo done
