#!/bin/bash
# Symmetric SpMV: cheaper index math A/B, then PMC passes (SQ stall/LDS counters, FETCH, WRITE)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step sym_tests 300 python -u -m pytest tests/test_gpu_sym.py -x -q --timeout 120 --timeout-method thread || exit 1
step symab4 400 python tools/cg_ab.py '[{"spmv_sym_pf":1},{"spmv_sym_pf":1,"spmv_sym_occ":6},{"spmv_sym_pf":0},{"spmv_sym":0}]' --reps 4 --its 200 || exit 1
tail -n 1 gpurun_out/symab4.log
B="python3 bench.py --steps 20 --warmup 0 --no-solve --no-cpu-baseline --no-aij"
step pmc_sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_sq -o s --output-format csv -- $B || exit 1
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f --output-format csv -- $B || exit 1
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w --output-format csv -- $B || exit 1
echo done
