source tools/gpu_steps.sh
step cg_gaps 400 python tools/cg_gaps.py 20,16,16 300
cat gpurun_out/cg_gaps.log
