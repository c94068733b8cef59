source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step full_size 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 280 --timeout-method thread -k full_size || exit 1
tail -n 3 gpurun_out/full_size.log
