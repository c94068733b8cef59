# Unstructured-mesh measurement pass (bench + rocprofv3 stats + PMC traffic):
#   gpurun --timeout 1800 -- 'bash tools/gpu_umesh_bench.sh'
source tools/gpu_steps.sh
step bench_umesh 600 python bench.py --mesh unstructured --ops
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_umesh 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_umesh -o u --output-format csv -- python bench.py --mesh unstructured --steps 200 --no-cpu-baseline --ops
step pmc_fetch_u 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_u -o f --output-format csv -- python bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline
step pmc_write_u 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_u -o w --output-format csv -- python bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline
tail -n 1 gpurun_out/bench_umesh.log
