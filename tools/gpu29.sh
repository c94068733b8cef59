source tools/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
step layout_ab 600 python tools/spmv_layout_ab.py 7
cat gpurun_out/layout_ab.log
