#!/bin/bash
# column-dictionary SpMV: PMC HBM traffic (1M-DoF unstructured), bench + kernel stats, config-5 size
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02au
export TMPDIR=/tmp
step pmc_f 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02au/pmc_f -o f --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
step pmc_w 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02au/pmc_w -o w --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
cp profiles/traffic.json gpurun_out/r02au/traffic.json
step traffic 60 python tools/pmc_traffic.py gpurun_out/r02au/pmc_f gpurun_out/r02au/pmc_w k_nb_spmv_dict "[20, 16, 16]-5-1-umesh-chunk-nt-u1-dict" gpurun_out/r02au/traffic.json || exit 1
step prof_um 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02au/prof_um -o um --output-format csv -- python3 bench.py --mesh unstructured --steps 200 --no-cpu-baseline --no-aij --traffic gpurun_out/r02au/traffic.json || exit 1
grep '^{' gpurun_out/prof_um.log > gpurun_out/r02au/bench_umesh_under_rocprof.json
step bench_um 600 python bench.py --mesh unstructured --no-aij --traffic gpurun_out/r02au/traffic.json || exit 1
grep '^{' gpurun_out/bench_um.log > gpurun_out/r02au/bench_umesh.json
step bench_cfg5 700 python bench.py --mesh unstructured --nelem 40,32,32 --steps 50 --warmup 5 --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/bench_cfg5.log > gpurun_out/r02au/bench_cfg5_umesh.json
echo done
