# Full GPU parity suite on HEAD, then a kernel-trace profile of config-4 (p=6) setup + CG
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
step prof_cfg4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg4 -o run -- python3 bench.py --nelem 18,18,18 --ngl 7 --steps 20 --warmup 2 --no-cpu-baseline --no-solve || exit 1
find gpurun_out/prof_cfg4 -name '*kernel_stats.csv' | head -1 | xargs head -20
