# GPU-box check of the unstructured-mesh row (through gpurun):
#   gpurun --timeout 1200 -- 'bash tools/gpu_umesh.sh'
source tools/gpu_steps.sh
step pytest_umesh 600 python -m pytest tests/test_gpu_umesh.py tests/test_gpu_multirank.py -q -x -k "umesh"
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
