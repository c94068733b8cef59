# Round 2, second pass (row-dot SpMV epilogue, continue): full GPU suite (incl. RCCL self-communicator, init
# deadline, 2-rank self-launch), default bench, driver-shaped bench, rocprof
# kernel stats of the bench command.
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
step bench_default 600 python bench.py || exit 1
tail -n 1 gpurun_out/bench_default.log > gpurun_out/r02c/bench_default.json
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_driver.log > gpurun_out/r02c/bench_driver.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02c/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline || exit 1
echo done
