source tools/gpu_steps.sh
step sweepseq 600 python tools/spmv_sweep_seq.py 20,16,16 5 30
cat gpurun_out/sweepseq.log
