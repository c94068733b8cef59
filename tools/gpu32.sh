source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q
step fast_ab 600 python tools/spmv_fast_ab.py 9
step bench_default 600 python bench.py --no-cpu-baseline
cat gpurun_out/fast_ab.log
