#!/bin/bash
# Round 2: Hilbert default; unstructured column stream padded to 128 B per row (KLE_BCOL_PAD 32 vs 1);
# unstructured / NS / operator GPU tests
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02w
export TMPDIR=/tmp
step um_tests 600 python -u -m pytest tests/test_gpu_umesh.py tests/test_gpu_ns.py tests/test_gpu_ops.py tests/test_gpu_multirank.py tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
for rep in 1 2; do
  for p in 1 32; do
    KLE_BCOL_PAD=$p step um_p${p}_r$rep 400 python bench.py --mesh unstructured --steps 200 --no-cpu-baseline --no-aij || exit 1
    grep '^{' gpurun_out/um_p${p}_r$rep.log > gpurun_out/r02w/um_bcolpad${p}_rep$rep.json
  done
done
step pmc_f 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02w/pmc_f_um -o f --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
step pmc_w 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02w/pmc_w_um -o w --output-format csv -- python3 bench.py --mesh unstructured --steps 10 --warmup 0 --no-solve --no-cpu-baseline --no-aij || exit 1
echo done
