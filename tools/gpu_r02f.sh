#!/bin/bash
# Round 2: aij SpMV unroll A/B, config-2 full-size oracle parity, default bench (aij leg, cpu_baseline)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02f
export TMPDIR=/tmp
step aij_ab 400 python tools/aij_ab.py '[{"aij_unroll":1},{"aij_unroll":2},{"aij_unroll":4},{"aij_unroll":8}]' --reps 5 --its 40 || exit 1
cp gpurun_out/aij_ab.log gpurun_out/r02f/aij_ab.jsonl
step gpu_aij_tests 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_edges.py -m gpu -x -q --timeout 150 --timeout-method thread -k "aij or convert or setvalues or SetValues" || exit 1
step fullsize 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout-method thread || exit 1
step bench_default 900 python bench.py || exit 1
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02f/bench_default.json
echo done
