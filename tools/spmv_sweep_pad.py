"""Row-padding x load-policy sweep of the node-block SpMV on the bench matrix.
GPU tool (tools/, not product).
Usage: python tools/spmv_sweep_pad.py [pads=1,8,16] [nts=0,1] [reps=30] [cg=1]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402
from pynama_amd.petsc import KSP, PC  # noqa: E402
from pynama_amd.runtime import set_row_padding  # noqa: E402


def main():
    pads = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,8,16").split(",")]
    nts = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    do_cg = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    ctx = pa.get_ctx()
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    ref = None
    for pad in pads:
        set_row_padding(pad)
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
        for nt in nts:
            K.setSpmvNontemporal(nt)
            for _ in range(3):
                K.mult(x, y)
            ctx.synchronize()
            ctx.set_profiling(True)
            ctx.reset_stats()
            for _ in range(reps):
                K.mult(x, y)
            c, ms = ctx.kernel_stats("spmv")
            ctx.set_profiling(False)
            yy = y.getArray()
            if ref is None:
                ref = yy
            rec = {"pad": pad, "nt": nt, "spmv_ms": ms / c, "gbps": K.spmvBytes() / (ms / c * 1e-3) / 1e9,
                   "bitexact": bool(np.array_equal(yy, ref))}
            if do_cg:
                kb = KSP().create()
                kb.setType("cg")
                pc = PC()
                pc.setType("jacobi")
                kb.setPC(pc)
                kb.setOperators(K)
                kb.setFixedIterations(100)
                xs = K.createVecRight()
                kb.solve(y, xs)
                ctx.synchronize()
                t = time.perf_counter()
                kb.solve(y, xs)
                ctx.synchronize()
                rec["cg_iter_ms"] = (time.perf_counter() - t) / 100 * 1e3
            print(json.dumps(rec), flush=True)
        del mat, dom, K
    set_row_padding(1)


if __name__ == "__main__":
    main()
