#!/bin/bash
# Round 2: GPU suite with the XCD-run SpMV mapping; aij A/B; default bench + rocprof stats;
# PMC FETCH/WRITE for config 2 (nb + aij kernels) and the 1M-DoF unstructured mesh
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02n
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
step aij_ab 300 python tools/aij_ab.py '[{"spmv_xcd_chunk":0},{"spmv_xcd_chunk":16}]' --reps 4 --its 40 || exit 1
cp gpurun_out/aij_ab.log gpurun_out/r02n/aij_ab_xcd.jsonl
step bench_default 600 python bench.py || exit 1
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02n/bench_default.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02n/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline || exit 1
grep '^{' gpurun_out/prof_bench.log > gpurun_out/r02n/bench_under_rocprof.json
step pmc_f_box 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02n/pmc_f_box -o f --output-format csv -- python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step pmc_w_box 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02n/pmc_w_box -o w --output-format csv -- python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step pmc_f_um 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02n/pmc_f_um -o f --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
step pmc_w_um 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02n/pmc_w_um -o w --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
step bench_umesh 600 python bench.py --mesh unstructured --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/bench_umesh.log > gpurun_out/r02n/bench_umesh.json
echo done
