source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q
step bench_default 600 python bench.py
tail -n 1 gpurun_out/bench_default.log
