source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step bench_contract 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread || exit 1
tail -n 4 gpurun_out/bench_contract.log
