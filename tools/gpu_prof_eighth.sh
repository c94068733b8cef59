source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step prof_eighth 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_eighth -o e --output-format csv -- python3 bench.py --nelem 20,16,2 --steps 400 --no-cpu-baseline --no-solve || exit 1
head -8 gpurun_out/prof_eighth/e_kernel_stats.csv | cut -c1-200
