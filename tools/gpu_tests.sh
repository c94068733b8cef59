# GPU-box check: parity tests, smoke, default bench (run through gpurun):
#   gpurun --timeout 1800 -- 'bash tools/gpu_tests.sh'
source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
tail -n 1 gpurun_out/bench_default.log
