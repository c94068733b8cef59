source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_default 600 python bench.py --aij
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_bench 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench3 -o bench --output-format csv -- python bench.py --steps 200 --no-cpu-baseline
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch3 -o f --output-format csv -- python bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write3 -o w --output-format csv -- python bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline
tail -n 1 gpurun_out/bench_default.log
