# GPU-box check of the multi-rank paths (host transport, ranks share the GPU)
source tools/gpu_steps.sh
step pytest_multirank 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_umesh.py -x -v --timeout 300 --timeout-method thread
