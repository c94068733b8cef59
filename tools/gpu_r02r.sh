#!/bin/bash
# Round 2: k_dot_finish ticket: 8 slot words + global vs one word; cg vs pipecg (separate reduction)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02r
export TMPDIR=/tmp
step gpu_ksp_tests 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 150 --timeout-method thread -k "cg or pipe or partition or rccl or bench or continue" || exit 1
V='[{"_ksp":"cg","ticket_slots":8},{"_ksp":"cg","ticket_slots":1},{"_ksp":"pipecg"}]'
step ab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 6 --its 500 || exit 1
cp gpurun_out/ab_eighth.log gpurun_out/r02r/ticket_eighth.jsonl
step ab_full 400 python tools/cg_ab.py "$V" --reps 6 --its 200 || exit 1
cp gpurun_out/ab_full.log gpurun_out/r02r/ticket_full.jsonl
echo done
