#!/bin/bash
# Round 2 (re-entry): GPU suite, default bench, bench under rocprof (kernel stats)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02e
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
step bench_default 600 python bench.py || exit 1
tail -n 1 gpurun_out/bench_default.log > gpurun_out/r02e/bench_default.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02e/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/prof_bench.log > gpurun_out/r02e/bench_under_rocprof.json
step bench_eighth 300 python bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_eighth.log > gpurun_out/r02e/bench_eighth.json
echo done
