source tools/gpu_steps.sh
step ab 600 python tools/spmv_ab.py '[[64,1,1,1],[64,1,2,1],[32,1,1,1],[32,1,2,1],[16,1,1,1],[16,1,2,1],[64,2,1,1]]' 9
cat gpurun_out/ab.log
