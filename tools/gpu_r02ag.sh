#!/bin/bash
# Fixed cost of a plain streaming read vs the SpMV's 17 us intercept
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ag
step stream_fixed 300 python tools/stream_fixed_cost.py || exit 1
grep '^{' gpurun_out/stream_fixed.log > gpurun_out/r02ag/stream_fixed_cost.jsonl
echo done
