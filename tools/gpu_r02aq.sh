#!/bin/bash
# x-in-LDS SpMV default: PMC HBM traffic of k_nb_spmv_xl, default bench with it, kernel stats
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02aq
export TMPDIR=/tmp
step pmc_f 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02aq/pmc_f -o f --output-format csv -- python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
step pmc_w 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02aq/pmc_w -o w --output-format csv -- python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
cp profiles/traffic.json gpurun_out/r02aq/traffic.json
step traffic 60 python tools/pmc_traffic.py gpurun_out/r02aq/pmc_f gpurun_out/r02aq/pmc_w k_nb_spmv_xl "[20, 16, 16]-5-1-chunk-nt-u1-struct-xl" gpurun_out/r02aq/traffic.json || exit 1
step bench_default 600 python bench.py --traffic gpurun_out/r02aq/traffic.json || exit 1
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02aq/bench_default.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02aq/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --traffic gpurun_out/r02aq/traffic.json || exit 1
grep '^{' gpurun_out/prof_bench.log > gpurun_out/r02aq/bench_under_rocprof.json
echo done
