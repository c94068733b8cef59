"""Does the symmetric SpMV's speed depend on where its arrays land in memory?

Probe build (tools/libkle_probe.so): times the config-2 symmetric SpMV (HIP
events, the gather included) after moving, one at a time, the tile-partial
workspace or the value array to fresh allocations (kle_probe_realloc), at
several byte offsets into them.  One JSON line per measurement.

  python tools/alloc_probe.py [--its 40] [--nelem 20,16,16]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KLE_LIBRARY"] = os.path.join(ROOT, "tools", "libkle_probe.so")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nelem", default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--its", type=int, default=40)
    ap.add_argument("--nostore", action="store_true", help="also time each placement without the partial stores")
    a = ap.parse_args()
    import numpy as np

    import pynama_amd as pa
    from pynama_amd._lib import load
    nelem = [int(v) for v in a.nelem.split(",")]
    cfg = {"domain": {"ngl": a.ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    lib = load()
    lib.kle_probe_realloc.argtypes = [C.c_void_p, C.c_int, C.c_longlong]
    ctx = pa.get_ctx()
    x = K.createVecRight()
    x.setArray(np.random.default_rng(1).uniform(-1, 1, x.getLocalSize()))
    y = K.createVecLeft()

    def timed():
        for _ in range(5):
            K.mult(x, y)
        ctx.synchronize()
        ctx.set_profiling(True, only="spmv")
        ctx.reset_stats()
        for _ in range(a.its):
            K.mult(x, y)
        ctx.synchronize()
        c, ms = ctx.kernel_stats("spmv")
        ctx.set_profiling(False)
        return ms / c * 1e3

    y0 = None
    ap_plan = os.environ.get("ALLOC_PLAN", "values")
    if ap_plan == "mix":  # each value placement with four partial-workspace placements
        plan = [("none", 0)] * 2
        for _ in range(6):
            plan += [("values", 0)] + [("ws", 0)] * 4
    elif ap_plan == "full":  # the full-storage SpMV (spmv_sym 0) with its value array moved
        from pynama_amd.runtime import set_tuning
        set_tuning("spmv_sym", 0)
        plan = [("none", 0)] * 2 + [("full", 0)] * 10
    elif ap_plan == "ws":
        plan = [("none", 0)] * 3 + [("ws", 0)] * 8 + [("ws", s) for s in (4096, 65536, 1 << 20, (2 << 20) + 4096)] * 2 \
            + [("values", 0)] * 6 + [("none", 0)] * 2
    else:  # the value array at fresh allocations and byte offsets into them
        plan = [("none", 0)] * 2 + [("values", s) for s in (0, 0, 0, 0, 0, 0, 256, 4096, 65536, 1 << 20,
                                                             (2 << 20) + 4096, 0, 0, 0, 0, 0)]
    from pynama_amd.runtime import set_tuning
    for what, shift in plan:
        if what != "none":
            rc = lib.kle_probe_realloc(K._h, {"values": 1, "ws": 2, "full": 3}[what], shift)
            assert rc == 0
        us = timed()
        yy = y.getArray().copy()
        if y0 is None:
            y0 = yy
        rec = {"moved": what, "shift": shift, "spmv_us": us, "same_y": bool(np.array_equal(yy, y0))}
        if a.nostore:  # the same placement without the partial stores (probe 8, wrong y on purpose)
            set_tuning("spmv_sym_probe", 8)
            rec["nostore_us"] = timed()
            set_tuning("spmv_sym_probe", 0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
