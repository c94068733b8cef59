#!/bin/bash
# Full-size config 2 on 2 / 4 / 8 ranks sharing one GPU (host-staged transport): the distributed
# path with the round-2 kernels (x-in-LDS SpMV on split row ranges at 2 / 4 ranks) converges as at N = 1
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02bc
export KLE_TRANSPORT=host KLE_DEVICE=0
for n in 2 4 8; do
  step bench_n$n 600 python bench.py --gpus $n --steps 20 --warmup 2 || exit 1
  grep '^{' gpurun_out/bench_n$n.log > gpurun_out/r02bc/bench_host_n$n.json
done
echo done
