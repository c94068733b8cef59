source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_n1 420 python bench.py --steps 200 --warmup 20 --aij
export KLE_TRANSPORT=host
step bench_n2host 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --no-solve
unset KLE_TRANSPORT
tail -c 2500 gpurun_out/bench_n1.log; tail -c 1500 gpurun_out/bench_n2host.log
