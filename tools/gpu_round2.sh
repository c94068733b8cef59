# LU tests, config-5-size unstructured bench, 1/8-size box (per-rank floor of the N=8 strong-scaling run)
source tools/gpu_steps.sh
step pytest_lu 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "lu or gmres" || exit 1
step bench_cfg5 900 python bench.py --mesh unstructured --nelem 40,32,32 --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
step bench_eighth 300 python bench.py --nelem 20,16,2 --steps 400 --warmup 20 --no-cpu-baseline
tail -n 1 gpurun_out/bench_cfg5.log gpurun_out/bench_eighth.log
