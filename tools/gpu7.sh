source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step sweeppad 400 python tools/spmv_sweep_pad.py 1,4,8,16 0,1 30 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pmc_p1 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pad -o p1 --output-format csv -- python tools/spmv_sweep_pad.py 1 0,1 5 0
step pmc_p16 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pad -o p16 --output-format csv -- python tools/spmv_sweep_pad.py 16 0,1 5 0
step pmc_p8 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pad -o p8 --output-format csv -- python tools/spmv_sweep_pad.py 8 0,1 5 0
cat gpurun_out/sweeppad.log
