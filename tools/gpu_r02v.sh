#!/bin/bash
# Round 2: unstructured node order, Morton (0) vs Hilbert (1): time (alternating processes) and PMC fetch
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02v
export TMPDIR=/tmp
for rep in 1 2; do
  for o in 0 1; do
    KLE_UMESH_ORDER=$o step um_o${o}_r$rep 400 python bench.py --mesh unstructured --steps 200 --no-cpu-baseline --no-aij || exit 1
    grep '^{' gpurun_out/um_o${o}_r$rep.log > gpurun_out/r02v/um_order${o}_rep$rep.json
  done
done
for o in 0 1; do
  KLE_UMESH_ORDER=$o step pmc_f_o$o 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02v/pmc_f_o$o -o f --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
  KLE_UMESH_ORDER=$o step pmc_w_o$o 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02v/pmc_w_o$o -o w --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
done
KLE_UMESH_ORDER=1 step um_cfg5_hilbert 600 python bench.py --mesh unstructured --nelem 40,32,32 --steps 50 --warmup 5 --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/um_cfg5_hilbert.log > gpurun_out/r02v/cfg5_hilbert.json
echo done
