#!/bin/bash
# Symmetric SpMV variants (tile width, occupancy) in-process, and a kernel trace of the default bench
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step symab2 400 python tools/cg_ab.py '[{"spmv_sym_tx":8,"spmv_sym_occ":0},{"spmv_sym_tx":8,"spmv_sym_occ":8},{"spmv_sym_tx":8,"spmv_sym_occ":6},{"spmv_sym_tx":16,"spmv_sym_occ":0},{"spmv_sym_tx":16,"spmv_sym_occ":8},{"spmv_sym_tx":16,"spmv_sym_occ":6},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab2.log
step prof_sym 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sym -o b --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-aij || exit 1
echo done
