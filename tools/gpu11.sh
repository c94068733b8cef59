source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_ops 600 python bench.py --ops --no-cpu-baseline --no-solve
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_ops 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ops -o ops --output-format csv -- python bench.py --ops --no-cpu-baseline --no-solve --steps 20
tail -n 1 gpurun_out/bench_ops.log
