source tools/gpu_steps.sh
step pytest_gpu 600 python -m pytest tests -m gpu -q
step sweep 600 python tools/spmv_sweep.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_kt 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o bench --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-solve
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o spmv --output-format csv -- python tools/spmv_only.py 10
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o spmv --output-format csv -- python tools/spmv_only.py 10
ls -R gpurun_out | head -50
