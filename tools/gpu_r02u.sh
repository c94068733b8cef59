#!/bin/bash
# Round 2: resources of the RCCL kernels (one-rank communicator) from a kernel trace
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02u
export TMPDIR=/tmp
export KLE_RCCL_SELF=1 KLE_COMM_TIMEOUT_S=60
step rccl_trace 300 rocprofv3 --kernel-trace -d gpurun_out/r02u/trace -o rccl --output-format csv -- python3 tools/rccl_self_kernels.py || exit 1
echo done
