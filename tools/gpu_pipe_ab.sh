# pipecg vs single-reduction CG at N = 1 on config 2 (alternating, 1000 steps)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
for r in 1 2; do
step full_cg_$r 300 python bench.py --steps 1000 --no-cpu-baseline --ksp cg || exit 1
step full_pipecg_$r 300 python bench.py --steps 1000 --no-cpu-baseline --ksp pipecg || exit 1
done
grep -h "^{" gpurun_out/full_*.log | cut -c1-200
