source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_default 600 python bench.py --ops --no-cpu-baseline
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -n 1 gpurun_out/bench_default.log
