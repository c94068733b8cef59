#!/bin/bash
# Round 2: SpMV time vs slab thickness (fixed cost per launch = intercept of time vs bytes)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02x
export TMPDIR=/tmp
for nz in 1 2 3 4 6 8 16; do
  step slab_$nz 300 python bench.py --nelem 20,16,$nz --steps 400 --warmup 20 --no-solve --no-cpu-baseline --no-aij --ksp cg || exit 1
  grep '^{' gpurun_out/slab_$nz.log > gpurun_out/r02x/slab_$nz.json
done
echo done
