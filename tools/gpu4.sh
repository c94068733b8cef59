source tools/gpu_steps.sh
step sweep2 600 python tools/spmv_sweep.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step calib_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch -o calib --output-format csv -- python tools/stream_calib.py
step pmc_fetch_t 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_t -o spmv --output-format csv -- python tools/spmv_only.py 10 64 2 0 1 1
step pmc_fetch_n 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_n -o spmv --output-format csv -- python tools/spmv_only.py 10 64 2 0 0 0
step pmc_hit 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_hit -o spmv --output-format csv -- python tools/spmv_only.py 10 64 2 0 0 0
step pmc_hit_t 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_hit_t -o spmv --output-format csv -- python tools/spmv_only.py 10 64 2 0 1 1
cat gpurun_out/sweep2.log | head -12
