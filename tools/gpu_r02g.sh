#!/bin/bash
# Round 2: aij SpMV unroll x waves A/B; 1/8-slab CG vs pipecg with kernel stats
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
step aij_ab 400 python tools/aij_ab.py '[{"aij_unroll":8,"aij_waves":4},{"aij_unroll":16,"aij_waves":4},{"aij_unroll":8,"aij_waves":8},{"aij_unroll":16,"aij_waves":8}]' --reps 5 --its 40 || exit 1
cp gpurun_out/aij_ab.log gpurun_out/r02g/aij_ab.jsonl
step prof_eighth_cg 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02g/prof_eighth_cg -o eighth --output-format csv -- python3 bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline --no-aij --ksp cg || exit 1
grep '^{' gpurun_out/prof_eighth_cg.log > gpurun_out/r02g/bench_eighth_cg_rocprof.json
step prof_eighth_pipe 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02g/prof_eighth_pipe -o eighth --output-format csv -- python3 bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline --no-aij --ksp pipecg || exit 1
grep '^{' gpurun_out/prof_eighth_pipe.log > gpurun_out/r02g/bench_eighth_pipe_rocprof.json
step eighth_pipe 300 python bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline --no-aij --ksp pipecg || exit 1
grep '^{' gpurun_out/eighth_pipe.log > gpurun_out/r02g/bench_eighth_pipe.json
step eighth_cg 300 python bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline --no-aij --ksp cg || exit 1
grep '^{' gpurun_out/eighth_cg.log > gpurun_out/r02g/bench_eighth_cg.json
echo done
