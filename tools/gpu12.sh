source tools/gpu_steps.sh
step pytest_el 600 python -m pytest tests/test_gpu.py -q -x -k element_kernel
export KLE_DEVICE=0
step rccl2 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 2 --no-solve --no-cpu-baseline --nelem 8,8,8
tail -n 30 gpurun_out/rccl2.log
