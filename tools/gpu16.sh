source tools/gpu_steps.sh
step pytest_mr 600 python -m pytest tests/test_gpu_multirank.py -q -x
