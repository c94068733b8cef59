#!/bin/bash
# x-in-LDS SpMV on split row ranges (multirank, host transport) + bitwise tests + config 4 bench
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ar
step t_xl 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu.py -x -v --timeout 150 --timeout-method thread -k "x_in_lds or partitioned_solve_matches or eight_slab" || exit 1
grep -E "PASS|FAIL|passed|failed" gpurun_out/t_xl.log | tail -30 > gpurun_out/r02ar/tests.txt
step bench_cfg4 600 python bench.py --nelem 18,18,18 --ngl 7 --steps 20 --warmup 3 --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/bench_cfg4.log > gpurun_out/r02ar/bench_cfg4.json
echo done
