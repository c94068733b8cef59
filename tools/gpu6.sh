source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step sweepbuf 300 python tools/spmv_sweep_buf.py 30
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pmc_buf 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_buf -o spmv --output-format csv -- python tools/spmv_sweep_buf.py 3
cat gpurun_out/sweepbuf.log
