"""In-process A/B of the scalar CSR (aij) SpMV on config 2's K (SURVEY 8(d)'s
format: 12 B per nonzero + row pointers + x + y).

K is assembled in node-block form and converted once; variants (tuning knobs)
alternate rep by rep in one process, each rep timing --its launches with HIP
events.  Prints one JSON line per (rep, variant) and a summary; also checks
that every variant's y is bitwise the first variant's.

  python tools/aij_ab.py '[{}]' [--nelem 20,16,16] [--reps 5] [--its 50]
(the unroll / waves-per-workgroup knobs of the round-2 A/B,
profiles/r02/aij_ab_*.jsonl, were removed once k_aij_spmv<8,4> won; a
variant is a dict of kle_set_tuning keys)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--nelem", default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--its", type=int, default=50)
    ap.add_argument("--format", choices=["aij", "nb"], default="aij", help="nb: the node-block K itself")
    a = ap.parse_args()
    variants = json.loads(a.variants)
    import numpy as np

    import pynama_amd as pa
    from pynama_amd.runtime import set_tuning
    ctx = pa.get_ctx()
    nelem = [int(v) for v in a.nelem.split(",")]
    cfg = {"domain": {"ngl": a.ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    A = mat.K.convert("aij") if a.format == "aij" else mat.K
    nbytes = A.spmvBytes()
    x, y = A.createVecRight(), A.createVecLeft()
    x.setArray(np.random.default_rng(0).uniform(-1, 1, x.getLocalSize()))
    res = {i: [] for i in range(len(variants))}
    ref = None
    for rep in range(a.reps):
        for vi, v in enumerate(variants):
            for k, val in v.items():
                set_tuning(k, val)
            for _ in range(3):
                A.mult(x, y)
            ctx.set_profiling(True, only="spmv")
            ctx.reset_stats()
            for _ in range(a.its):
                A.mult(x, y)
            c, ms = ctx.kernel_stats("spmv")
            ctx.set_profiling(False)
            ya = y.getArray()
            if ref is None:
                ref = ya.copy()
            bitwise = bool(np.array_equal(ya, ref))
            avg = ms / c
            res[vi].append(avg)
            print(json.dumps({"rep": rep, "variant": v, "avg_ms": avg, "gbps": nbytes / (avg * 1e-3) / 1e9,
                              "bitwise_equal_first": bitwise}), flush=True)
            for k in v:
                set_tuning(k, {"spmv_xcd_chunk": 16, "spmv_dyn_lds": -1, "spmv_x_lds": 1, "spmv_dict": 1, "upd_preload": 1}.get(k, 0))
    summ = [{"variant": v, "median_ms": statistics.median(res[i]), "min_ms": min(res[i]),
             "gbps_median": nbytes / (statistics.median(res[i]) * 1e-3) / 1e9} for i, v in enumerate(variants)]
    print(json.dumps({"summary": summ, "bytes_per_spmv": nbytes, "nnz": A.getInfo()["nz_used"],
                      "nelem": nelem, "ngl": a.ngl}), flush=True)


if __name__ == "__main__":
    main()
