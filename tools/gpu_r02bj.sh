#!/bin/bash
# Whole GPU suite in one process (as the driver runs it), after the full-size unstructured parity test
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02bj
step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log > gpurun_out/r02bj/pytest_gpu.txt
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo done
