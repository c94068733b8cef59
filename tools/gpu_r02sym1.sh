#!/bin/bash
# Symmetric-storage SpMV: tests, in-process CG A/B against the full storage, bench
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step sym_tests 300 python -u -m pytest tests/test_gpu_sym.py -x -v --timeout 120 --timeout-method thread || exit 1
step symab_full 300 python tools/cg_ab.py '[{"spmv_sym":1},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab_full.log
step bench_sym 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_sym.log
echo done
