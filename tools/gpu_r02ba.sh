#!/bin/bash
# single-reduction vs pipelined CG at one rank with the final kernels (config 2 box and 1M-DoF unstructured)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ba
V='[{"_ksp":"cg"},{"_ksp":"pipecg"}]'
step full 400 python tools/cg_ab.py "$V" --reps 6 --its 200 || exit 1
grep '^{' gpurun_out/full.log > gpurun_out/r02ba/ksp_full.jsonl
step um 400 python tools/cg_ab.py "$V" --mesh unstructured --reps 6 --its 200 || exit 1
grep '^{' gpurun_out/um.log > gpurun_out/r02ba/ksp_umesh.jsonl
echo done
