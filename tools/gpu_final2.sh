# Round-end: full GPU suite, then the round profiling pass (default bench, rocprof stats, PMC, configs)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
bash tools/gpu_profile_final.sh
