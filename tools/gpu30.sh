source tools/gpu_steps.sh
step layout_ab 600 python tools/spmv_layout_ab.py 11
step bench_l0 300 python bench.py --no-cpu-baseline --no-solve
KLE_NB_LAYOUT=1 step bench_l1 300 python bench.py --no-cpu-baseline --no-solve
step bench_l0b 300 python bench.py --no-cpu-baseline --no-solve
KLE_NB_LAYOUT=1 step bench_l1b 300 python bench.py --no-cpu-baseline --no-solve
cat gpurun_out/layout_ab.log
