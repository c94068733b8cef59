#!/bin/bash
# Round 2 final checkpoint: full GPU suite, smoke, default bench, bench under rocprof (kernel stats)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02bh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default 600 python bench.py || exit 1
cp gpurun_out/bench_default.log gpurun_out/r02bh/bench_default.log
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02bh/bench_default.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02bh/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline || exit 1
grep '^{' gpurun_out/prof_bench.log > gpurun_out/r02bh/bench_under_rocprof.json
KLE_TRANSPORT=host KLE_DEVICE=0 step bench_gpus2 300 python bench.py --gpus 2 --steps 50 --warmup 5 --nelem 20,16,4 || exit 1
echo done
