source tools/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_sr 420 python bench.py --steps 200 --warmup 20
step bench_classic 420 python bench.py --steps 200 --warmup 20 --classic-cg --no-cpu-baseline
python - <<'PY'
import json
for f in ("bench_sr","bench_classic"):
    l=[x for x in open(f"gpurun_out/{f}.log") if x.startswith("{")]
    if l:
        d=json.loads(l[-1]); print(f, d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["breakdown_ms_per_iter"], d["solve"], d.get("cpu_baseline"))
PY
