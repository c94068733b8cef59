# Round 2: validate the pruned / fused CG path; event and hipGraph overhead A/B; default bench + rocprof
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
V='[{"_prof_spmv":0,"_graph":0},{"_prof_spmv":1,"_graph":0},{"_prof_spmv":0,"_graph":1}]'
step cgab_full 400 python tools/cg_ab.py "$V" --reps 6 --its 200 || exit 1
step cgab_eighth 300 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 6 --its 1000 || exit 1
step bench_default 600 python bench.py || exit 1
tail -n 1 gpurun_out/bench_default.log > gpurun_out/r02d/bench_default.json
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_driver.log > gpurun_out/r02d/bench_driver.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/cgab_full.log gpurun_out/cgab_eighth.log
echo done
