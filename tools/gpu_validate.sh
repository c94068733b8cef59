# Round-end validation: full GPU suite, smoke, default bench; pipecg vs single-reduction CG on the 1/8 slab
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default 600 python bench.py || exit 1
tail -n 1 gpurun_out/bench_default.log | cut -c1-400
step eighth_cg 300 python bench.py --nelem 20,16,2 --steps 1000 --no-cpu-baseline --ksp cg || exit 1
step eighth_pipecg 300 python bench.py --nelem 20,16,2 --steps 1000 --no-cpu-baseline --ksp pipecg || exit 1
grep -h "^{" gpurun_out/eighth_*.log | cut -c1-300
