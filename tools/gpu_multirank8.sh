# 8-rank rehearsal of the multi-GPU path on one GPU (host transport): the new
# 8-rank parity tests, then bench.py launched by torch.distributed.run with 8
# ranks on config 3's mesh (ranks share cuda:0; RCCL itself cannot run here)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step mr8_tests 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 400 --timeout-method thread -k "eight or 8-inertial" || exit 1
tail -n 4 gpurun_out/mr8_tests.log
export KLE_TRANSPORT=host
step bench_n8_host 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 2 || exit 1
tail -n 1 gpurun_out/bench_n8_host.log
