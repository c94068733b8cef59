#!/bin/bash
# Pipelined symmetric SpMV: tests, in-process A/B against the first version and the full storage
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step sym_tests 300 python -u -m pytest tests/test_gpu_sym.py -x -v --timeout 120 --timeout-method thread || exit 1
step symab3 400 python tools/cg_ab.py '[{"spmv_sym_pf":1},{"spmv_sym_pf":1,"spmv_sym_occ":6},{"spmv_sym_pf":1,"spmv_sym_tx":16},{"spmv_sym_pf":0},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab3.log
echo done
