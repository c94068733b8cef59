source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q
step bench_pipe 300 python bench.py --ksp pipecg --no-cpu-baseline
tail -n 1 gpurun_out/bench_pipe.log
