source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_cfg4 900 python bench.py --nelem 18,18,18 --ngl 7 --steps 20 --warmup 2 --no-cpu-baseline
tail -n 1 gpurun_out/bench_cfg4.log
