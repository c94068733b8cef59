#!/bin/bash
# Round 2: the other configs with the round-2 kernels: operators chain, config 4 (p=6), config-5 size
# (unstructured 8M DoF), the 1/8 slab (cg and pipecg); kernel stats of the operators run
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02t
export TMPDIR=/tmp
step bench_ops 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02t/prof_ops -o ops --output-format csv -- python3 bench.py --ops --steps 100 --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/bench_ops.log > gpurun_out/r02t/bench_ops.json
step bench_cfg4 600 python bench.py --nelem 18,18,18 --ngl 7 --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
grep '^{' gpurun_out/bench_cfg4.log > gpurun_out/r02t/bench_cfg4.json
step bench_cfg5 600 python bench.py --mesh unstructured --nelem 40,32,32 --steps 50 --warmup 5 --no-cpu-baseline --no-aij || exit 1
grep '^{' gpurun_out/bench_cfg5.log > gpurun_out/r02t/bench_cfg5_umesh.json
step eighth_cg 300 python bench.py --nelem 20,16,2 --steps 500 --warmup 20 --no-cpu-baseline --no-aij --ksp cg || exit 1
grep '^{' gpurun_out/eighth_cg.log > gpurun_out/r02t/bench_eighth_cg.json
step eighth_pipe 300 python bench.py --nelem 20,16,2 --steps 500 --warmup 20 --no-cpu-baseline --no-aij --ksp pipecg || exit 1
grep '^{' gpurun_out/eighth_pipe.log > gpurun_out/r02t/bench_eighth_pipecg.json
echo done
