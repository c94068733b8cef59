"""bench.py's output contract (the driver parses this line): one JSON object
on stdout with the metric / value / roofline / cpu_baseline fields, on a small
mesh so it runs in seconds."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_contract():
    d = _run("--nelem", "4,4,4", "--ngl", "4", "--steps", "20", "--warmup", "2", "--cpu-seconds", "0.5")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 2 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and d["unit"] == "CG iters/s" and d["value"] > 0
    assert abs(d["ms_per_step"] - 1e3 / d["value"]) <= 1e-6 * d["ms_per_step"]
    assert "workload" in d["config"] and "model" not in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    # a PMC figure is only quoted for the kernel it was measured on
    assert r["traffic_status"] and r["traffic_key"]
    if r["traffic"] is not None:
        assert r["traffic_status"].startswith("measured")
        assert abs(r["traffic_over_bytes"] - r["traffic"] / r["bytes_per_launch"]) < 1e-12
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0 and c["unit"] == d["unit"]
    s = d["solve"]
    assert s["reason"] > 0 and s["true_rel_residual"] <= 2e-10
    assert d["symmetric_bricks"] is None  # (below spmv_sym_min_rows: full storage)
    # the streaming ceiling the SpMV is graded against is this box's own
    # (16-B nontemporal reads), and the PMC traffic rate cannot exceed it
    assert r["achievable_gbps"] > 4000.0 and abs(r["frac_of_achievable"] - r["achieved"] / r["achievable_gbps"]) < 1e-12
    if r["traffic_frac_of_read_ceiling"] is not None:
        assert r["traffic_frac_of_read_ceiling"] <= 1.0
    # the (f)#1 operator chain is measured in the default run (N = 1)
    ops = d["operators"]
    assert ops is not None and ops["evalRHS_chain_ms"] > 0
    for nm in ("Curl", "SrT", "DivSrT"):
        assert ops[nm]["bytes"] > 0 and ops[nm]["avg_ms"] > 0 and 0 < ops[nm]["frac"] < 1
    # what RCCL itself reports, per rank (one rank: no communicator)
    cfg = d["config"]
    assert cfg["rccl_ranks"] == 0 and cfg["rccl_user_ranks"] == [-1] and len(cfg["spmv_ms_per_rank"]) == 1


def test_bench_unstructured_line():
    d = _run("--mesh", "unstructured", "--nelem", "3,3,3", "--ngl", "4", "--steps", "10", "--warmup", "1",
             "--no-cpu-baseline")
    assert d["config"]["mesh"] == "unstructured" and d["cpu_baseline"] is None and d["value"] > 0
    assert d["roofline"]["achieved"] > 0
    assert d["config"]["parallelism"].startswith("inertial recursive bisection")
