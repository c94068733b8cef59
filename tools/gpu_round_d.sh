# Device patterns on unstructured meshes: parity, full GPU suite, config-5-size setup timing
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step devpat_u 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 150 --timeout-method thread -k "device_pattern" || exit 1
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
KLE_TIMING=1 step bench_cfg5 900 python bench.py --mesh unstructured --nelem 40,32,32 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_cfg5.log | cut -c1-200
