#!/bin/bash
# Symmetric SpMV with DPP row sums: tests, A/B, SQ counters
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step sym_tests 300 python -u -m pytest tests/test_gpu_sym.py -x -q --timeout 120 --timeout-method thread || exit 1
step symab5 400 python tools/cg_ab.py '[{"spmv_sym_pf":1},{"spmv_sym_pf":1,"spmv_sym_occ":6},{"spmv_sym_pf":1,"spmv_sym_tx":16},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab5.log
B="python3 bench.py --steps 20 --warmup 0 --no-solve --no-cpu-baseline --no-aij"
step pmc_sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_sq5 -o s --output-format csv -- $B || exit 1
echo done
