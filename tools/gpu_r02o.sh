#!/bin/bash
# Round 2: MatFS.Rd test; k_dot_finish grid-size A/B (1/8 slab and config 2)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02o
export TMPDIR=/tmp
step rd_test 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "rd_is_preallocated or spmv_and_solve" || exit 1
V='[{"fin_blocks":0},{"fin_blocks":64},{"fin_blocks":128},{"fin_blocks":512},{"fin_blocks":1024}]'
step fin_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 4 --its 1000 || exit 1
cp gpurun_out/fin_eighth.log gpurun_out/r02o/fin_blocks_eighth.jsonl
step fin_full 400 python tools/cg_ab.py "$V" --reps 4 --its 200 || exit 1
cp gpurun_out/fin_full.log gpurun_out/r02o/fin_blocks_full.jsonl
echo done
