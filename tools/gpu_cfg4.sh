# Config 4 (TG-3D box [18,18,18], ngl=7 / p=6, ~3.9M DoF) on one MI355X
source tools/gpu_steps.sh
step bench_cfg4 900 python bench.py --nelem 18,18,18 --ngl 7 --steps 50 --warmup 5 --cpu-seconds 10
tail -n 1 gpurun_out/bench_cfg4.log
