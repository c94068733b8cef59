source tools/gpu_steps.sh
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1; nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -m pytest tests -m gpu -q -x
step bench1 420 python bench.py --steps 100 --warmup 10 --aij
tail -c 3000 gpurun_out/bench1.log
