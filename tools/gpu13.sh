source tools/gpu_steps.sh
step pytest_ns 600 python -m pytest tests/test_gpu_ns.py -q -x
step pytest_gpu 900 python -m pytest tests -m gpu -q
