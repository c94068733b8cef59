#!/bin/bash
# Symmetric SpMV: two items ahead (three register sets), 8 or 4 waves per workgroup: tests, A/B
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step sym_tests 300 python -u -m pytest tests/test_gpu_sym.py -x -q --timeout 120 --timeout-method thread || exit 1
step symab13 400 python tools/cg_ab.py '[{"spmv_sym_pf":1},{"spmv_sym_pf":2},{"spmv_sym_pf":2,"spmv_sym_waves":4},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab13.log
echo done
