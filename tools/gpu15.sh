source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_default 600 python bench.py
export KLE_DEVICE=0 KLE_TRANSPORT=host
step bench_host2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 50 --warmup 5 --no-solve --no-cpu-baseline
tail -n 1 gpurun_out/bench_default.log gpurun_out/bench_host2.log
