# GPU-box check: parity tests, smoke, default bench (run through gpurun):
#   gpurun --timeout 1800 -- 'bash tools/gpu_tests.sh'
source tools/gpu_steps.sh
step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default 600 python bench.py
tail -n 1 gpurun_out/bench_default.log
