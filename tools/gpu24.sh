source tools/gpu_steps.sh
step pytest_ts 900 python -m pytest tests/test_gpu_ts.py -q
