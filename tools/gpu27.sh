source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
step ab 600 python tools/spmv_ab.py '[[64,1,1,1],[64,1,2,1]]' 7
step bench_default 600 python bench.py --no-cpu-baseline
tail -n 1 gpurun_out/bench_default.log
