#!/bin/bash
# Round-2 validation with the symmetric SpMV: whole GPU suite in one process, smoke,
# default bench, kernel trace of the bench command, PMC FETCH/WRITE of the SpMV kernels
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
mkdir -p gpurun_out/val3
step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log > gpurun_out/val3/pytest_gpu.txt
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default 600 python bench.py || exit 1
tail -n 1 gpurun_out/bench_default.log > gpurun_out/val3/bench_default.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/val3/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --no-aij || exit 1
B="python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij"
step pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/val3/pmc_fetch -o f --output-format csv -- $B || exit 1
step pmc_write 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/val3/pmc_write -o w --output-format csv -- $B || exit 1
echo done
