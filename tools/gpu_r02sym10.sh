#!/bin/bash
# Symmetric SpMV: 2-plane tiles (default) and 4-wave workgroups: tests, A/B
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step sym_tests 300 python -u -m pytest tests/test_gpu_sym.py -x -q --timeout 120 --timeout-method thread || exit 1
step symab10 500 python tools/cg_ab.py '[{"spmv_sym_tz":2},{"spmv_sym_tz":2,"spmv_sym_waves":4},{"spmv_sym_tz":1},{"spmv_sym_tz":1,"spmv_sym_waves":4},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab10.log
echo done
