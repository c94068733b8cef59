source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step ts_bench 600 python -u tools/ts_bench.py || exit 1
cat gpurun_out/ts_bench.log | grep "^{"
