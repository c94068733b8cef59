# Kernel stats of the unstructured-mesh bench (1M DoF) and of the default bench with the
# operator leg, current code (device patterns, MFMA element kernel, batched scratch)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step prof_umesh 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_umesh -o u --output-format csv -- python3 bench.py --mesh unstructured --steps 200 --no-cpu-baseline --ops || exit 1
step prof_ops 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ops -o o --output-format csv -- python3 bench.py --steps 50 --no-cpu-baseline --no-solve --ops || exit 1
echo done
