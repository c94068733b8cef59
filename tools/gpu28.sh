source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q
