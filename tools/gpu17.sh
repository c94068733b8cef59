source tools/gpu_steps.sh
step pytest_mr 900 python -m pytest tests/test_gpu_multirank.py -q
