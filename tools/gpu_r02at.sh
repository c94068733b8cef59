#!/bin/bash
# column-dictionary SpMV (unstructured): bitwise tests, multirank split ranges, CG A/B, bench
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02at
step t_dict 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py -x -v --timeout 150 --timeout-method thread -k "column_dictionaries or umesh_solve" || exit 1
grep -E "PASS|FAIL|passed|failed" gpurun_out/t_dict.log | tail -16 > gpurun_out/r02at/tests.txt
step cgab_um 500 python tools/cg_ab.py '[{"spmv_dict":0},{"spmv_dict":1}]' --mesh unstructured --reps 6 --its 200 || exit 1
grep '^{' gpurun_out/cgab_um.log > gpurun_out/r02at/cg_dict_umesh.jsonl
step bench_um 600 python bench.py --mesh unstructured --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/bench_um.log > gpurun_out/r02at/bench_umesh.json
echo done
