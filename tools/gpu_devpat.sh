# Device-built patterns: parity vs the host enumeration, full GPU suite, default + config-4 bench (assembly time)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step devpat_test 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "device_pattern" || exit 1
tail -n 3 gpurun_out/devpat_test.log
step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
step bench_default 600 python bench.py --ops || exit 1
tail -n 1 gpurun_out/bench_default.log
step bench_cfg4 900 python bench.py --nelem 18,18,18 --ngl 7 --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log
