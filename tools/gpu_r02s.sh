#!/bin/bash
# Round 2: full GPU suite after the BoundaryConditions refactor; default bench; N=2 self-launch (host transport)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02s
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -n 3 gpurun_out/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default 600 python bench.py || exit 1
grep '^{' gpurun_out/bench_default.log > gpurun_out/r02s/bench_default.json
echo done
