#!/bin/bash
# Round 2: hierarchical last-arriver tickets; pipecg reduction fused into its update kernel;
# KSP GPU tests; cg vs pipecg and dot-finish grid A/B
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02p
export TMPDIR=/tmp
step gpu_ksp_tests 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_edges.py tests/test_gpu_ns.py tests/test_gpu_umesh.py -m gpu -x -q --timeout 150 --timeout-method thread || exit 1
V='[{"_ksp":"cg"},{"_ksp":"cg","fin_blocks":1024},{"_ksp":"cg","fin_blocks":2048},{"_ksp":"pipecg"}]'
step ab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 4 --its 1000 || exit 1
cp gpurun_out/ab_eighth.log gpurun_out/r02p/ab_eighth.jsonl
step ab_full 400 python tools/cg_ab.py "$V" --reps 4 --its 200 || exit 1
cp gpurun_out/ab_full.log gpurun_out/r02p/ab_full.jsonl
step prof_eighth 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02p/prof_eighth -o eighth --output-format csv -- python3 bench.py --nelem 20,16,2 --steps 2000 --warmup 50 --no-cpu-baseline --no-aij --ksp pipecg || exit 1
echo done
