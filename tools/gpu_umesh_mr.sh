source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step umesh_mr 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 150 --timeout-method thread -k "umesh" || exit 1
