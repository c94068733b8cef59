#!/bin/bash
# x-in-LDS SpMV as the default: GPU suite, default bench, CG A/B at config 2 and the 1/8 slab
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ap
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
tail -n 2 gpurun_out/pytest_gpu.log
step bench_default 600 python bench.py || exit 1
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02ap/bench_default.json
step cgab_full 400 python tools/cg_ab.py '[{"spmv_x_lds":0},{"spmv_x_lds":1}]' --reps 6 --its 200 || exit 1
grep '^{' gpurun_out/cgab_full.log > gpurun_out/r02ap/cg_xl_full.jsonl
step cgab_eighth 300 python tools/cg_ab.py '[{"spmv_x_lds":0},{"spmv_x_lds":1}]' --nelem 20,16,2 --ksp pipecg --reps 6 --its 1000 || exit 1
grep '^{' gpurun_out/cgab_eighth.log > gpurun_out/r02ap/cg_xl_eighth.jsonl
echo done
