source tools/gpu_steps.sh
step ab 600 python tools/spmv_ab.py '[[1,2,1],[1,1,1],[2,1,1],[2,2,1],[4,2,1],[3,1,1]]' 9
cat gpurun_out/ab.log
