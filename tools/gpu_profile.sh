# Round profiling pass (bench + rocprofv3 kernel stats + PMC FETCH/WRITE/TCC):
#   gpurun --timeout 2400 -- 'bash tools/gpu_profile.sh'
source tools/gpu_steps.sh
step bench_default 600 python bench.py --aij --ops
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_bench 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench4 -o bench --output-format csv -- python bench.py --steps 200 --no-cpu-baseline
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch4 -o f --output-format csv -- python bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write4 -o w --output-format csv -- python bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline
step pmc_tcc 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_tcc4 -o t --output-format csv -- python bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline
tail -n 1 gpurun_out/bench_default.log
