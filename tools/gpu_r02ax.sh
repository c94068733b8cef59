#!/bin/bash
# 1/8 slab (per-rank share at N = 8): PMC HBM traffic of the SpMV and kernel stats
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ax
export TMPDIR=/tmp
A="--nelem 20,16,2 --ksp pipecg --no-cpu-baseline --no-aij"
step pmc_f 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02ax/pmc_f -o f --output-format csv -- python3 bench.py $A --steps 100 --warmup 0 --no-solve || exit 1
step pmc_w 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02ax/pmc_w -o w --output-format csv -- python3 bench.py $A --steps 100 --warmup 0 --no-solve || exit 1
cp profiles/traffic.json gpurun_out/r02ax/traffic.json
step traffic 60 python tools/pmc_traffic.py gpurun_out/r02ax/pmc_f gpurun_out/r02ax/pmc_w "k_nb_spmv<3, 3, 1, true, 4>" "[20, 16, 2]-5-1-chunk-nt-u1-struct" gpurun_out/r02ax/traffic.json || exit 1
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02ax/prof -o e --output-format csv -- python3 bench.py $A --steps 2000 --traffic gpurun_out/r02ax/traffic.json || exit 1
grep '^{' gpurun_out/prof.log > gpurun_out/r02ax/bench_eighth_under_rocprof.json
echo done
