#!/bin/bash
# CG update kernels: first element + stage inputs loaded before the prologue (upd_preload) vs after
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02aw
V='[{"upd_preload":0},{"upd_preload":1}]'
step ab_eighth_pipe 300 python tools/cg_ab.py "$V" --nelem 20,16,2 --ksp pipecg --reps 8 --its 1000 || exit 1
grep '^{' gpurun_out/ab_eighth_pipe.log > gpurun_out/r02aw/pre_eighth_pipe.jsonl
step ab_eighth_cg 300 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 8 --its 1000 || exit 1
grep '^{' gpurun_out/ab_eighth_cg.log > gpurun_out/r02aw/pre_eighth_cg.jsonl
step ab_full 400 python tools/cg_ab.py "$V" --reps 6 --its 200 || exit 1
grep '^{' gpurun_out/ab_full.log > gpurun_out/r02aw/pre_full.jsonl
step ab_quarter_pipe 300 python tools/cg_ab.py "$V" --nelem 20,16,4 --ksp pipecg --reps 6 --its 500 || exit 1
grep '^{' gpurun_out/ab_quarter_pipe.log > gpurun_out/r02aw/pre_quarter_pipe.jsonl
echo done
