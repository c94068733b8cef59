"""Time the node-block SpMV variants (and full CG iterations) on the bench
matrix in one process; prints one JSON object.  GPU tool (tools/, not product)."""
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402
from pynama_amd.petsc import KSP, PC  # noqa: E402


def main():
    nelem = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "20,16,16").split(",")]
    ngl = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ctx = pa.get_ctx()
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    K = mat.K
    x = K.createVecRight()
    x.setArray(np.random.default_rng(0).uniform(-1, 1, x.getLocalSize()))
    y = K.createVecLeft()
    nbytes = K.spmvBytes()
    out = {"n": K.getSize()[0], "bytes": nbytes, "stream_copy_gbps": ctx.stream_copy_gbps(),
           "stream_read_gbps": ctx.stream_read_gbps(), "variants": []}
    ref = None
    combos = [(64, u, 0, xcd, order) for u in (1, 2) for xcd in (0, 1) for order in (0, 1)]
    combos += [(64, 2, 1, 0, 0), (32, 2, 0, 1, 1)]
    for lpr, unr, pers, xcd, order in combos:
        K.setSpmvVariant(lpr, unr, pers)
        K.setSpmvLayout(xcd, order)
        for _ in range(5):
            K.mult(x, y)
        ctx.synchronize()
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(30):
            K.mult(x, y)
        c, ms = ctx.kernel_stats("spmv")
        ctx.set_profiling(False)
        yy = y.getArray()
        if ref is None:
            ref = yy
        err = float(np.abs(yy - ref).max() / np.abs(ref).max())
        kb = KSP().create()
        kb.setType("cg")
        pc = PC()
        pc.setType("jacobi")
        kb.setPC(pc)
        kb.setOperators(K)
        kb.setFixedIterations(50)
        xs = K.createVecRight()
        kb.solve(y, xs)
        ctx.synchronize()
        t = time.perf_counter()
        kb.solve(y, xs)
        ctx.synchronize()
        it_ms = (time.perf_counter() - t) / 50 * 1e3
        avg = ms / c
        out["variants"].append({"lpr": lpr, "unroll": unr, "persistent": pers, "xcd": xcd, "order": order,
                                "spmv_ms": avg,
                                "gbps": nbytes / (avg * 1e-3) / 1e9, "cg_iter_ms": it_ms, "maxdiff": err})
        print(json.dumps(out["variants"][-1]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
