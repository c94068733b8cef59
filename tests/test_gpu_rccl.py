"""RCCL transport and the multi-rank launch, on a one-GPU box.

RCCL refuses two ranks on one device, so the real two-way exchange runs only
in the driver's 8-GPU bench.  What one GPU can run is checked here:
  * a one-rank RCCL communicator (KLE_RCCL_SELF=1): the solver's allreduce
    goes through ncclAllReduce on the compute stream (CG, single-reduction CG)
    and on the comm stream (pipelined CG), and must reproduce the fused
    single-rank path bit for bit (one rank: the sum is the identity);
  * ncclCommInitRank's deadline: rank 0 of 2 whose peer never joins returns
    KLE_ERR_COMM after KLE_COMM_TIMEOUT_S instead of hanging;
  * `python bench.py --gpus 2` launching its own ranks (host transport, both
    ranks on cuda:0) and printing one JSON line with n_gpus = 2.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SOLVE = r'''
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import pynama_amd as pa
cfg = {"domain": {"ngl": 4, "box-mesh": {"nelem": [3, 3, 4], "lower": [0, 0, 0], "upper": [1, 1, 1]}},
       "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
dom = pa.Domain(); dom.configure(cfg); dom.setUp()
mat = pa.MatFS(); mat.setDomain(dom); mat.build()
f = pa.fields.get("taylor_green3d")
out = {"rccl": pa.get_ctx().transport}
for kt, single in (("cg", True), ("cg", False), ("pipecg", True)):
    sol = pa.KleSolver(); sol.setMat(mat); sol.setUp()
    ksp = sol.getKSP(); ksp.setType(kt); ksp.setCGSingleReduction(single)
    ksp.setTolerances(rtol=1e-11)
    vort = mat.Rw.createVecRight(); vort.setArray(f.vorticity(dom.getFullCoordArray(), 1.0))
    vel = sol.getSolution(); dom.applyBoundaryConditions(vel, "velocity", 0.0, 0.02)
    sol.solve(vort)
    u = vel.getArray()
    out[f"{kt}-{int(single)}"] = [ksp.getIterationNumber(), ksp.getConvergedReason(),
                                  hashlib.sha256(u.tobytes()).hexdigest(), float(vort.dot(vort)), float(vel.norm())]
print(json.dumps(out), flush=True)
'''


def _run_solve(extra_env):
    env = dict(os.environ, **extra_env)
    out = subprocess.run([sys.executable, "-c", _SOLVE, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=180)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_one_rank_rccl_communicator_matches_fused_path():
    ref = _run_solve({"KLE_RCCL_SELF": "0"})
    got = _run_solve({"KLE_RCCL_SELF": "1", "KLE_COMM_TIMEOUT_S": "60"})
    for k in ("cg-1", "cg-0", "pipecg-1"):
        assert ref[k][1] > 0, (k, ref[k])
        assert got[k] == ref[k], (k, got[k], ref[k])


_INIT = r'''
import ctypes as C, os, sys, time
sys.path.insert(0, sys.argv[1])
from pynama_amd._lib import load
lib = load()
raw = C.create_string_buffer(128)
assert lib.kle_get_unique_id(raw) == 0
h = C.c_void_p()
t = time.time()
rc = lib.kle_ctx_create(0, 0, 2, raw, C.byref(h))
print(rc, round(time.time() - t, 1), lib.kle_last_error().decode(), flush=True)
os._exit(0)   # the init helper thread is still blocked in the bootstrap
'''


def test_comm_init_times_out_when_a_peer_never_joins():
    env = dict(os.environ, KLE_COMM_TIMEOUT_S="8")
    out = subprocess.run([sys.executable, "-c", _INIT, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-3000:]
    rc, secs, msg = out.stdout.strip().splitlines()[-1].split(" ", 2)
    assert int(rc) != 0 and "did not complete" in msg, out.stdout
    assert 7.0 <= float(secs) <= 60.0, secs


def test_bench_launches_its_own_ranks():
    env = dict(os.environ, KLE_TRANSPORT="host", KLE_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--nelem", "4,4,4",
                          "--ngl", "4", "--steps", "10", "--warmup", "2", "--no-cpu-baseline"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 10
    assert d["solve"]["reason"] > 0 and d["solve"]["true_rel_residual"] <= 2e-10
    assert d["roofline"]["peak"] == 16000.0
    assert len(d["config"]["spmv_local_ms_per_rank"]) == 2  # (null: full-storage parts at this size)
