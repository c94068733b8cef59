# Full GPU suite, then bench with setup phase timings (config 2 default, config 4)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
KLE_TIMING=1 step bench_default 600 python bench.py --ops || exit 1
tail -n 1 gpurun_out/bench_default.log | cut -c1-300
KLE_TIMING=1 step bench_cfg4 900 python bench.py --nelem 18,18,18 --ngl 7 --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log | cut -c1-300
