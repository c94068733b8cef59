"""Rows-per-wave x unroll x load-policy sweep of the node-block SpMV on the
bench matrix (padded rows).  GPU tool (tools/, not product).
Usage: python tools/spmv_sweep_seq.py [nelem=20,16,16] [ngl=5] [reps=30]"""
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
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    ctx = pa.get_ctx()
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    x = K.createVecRight()
    x.setArray(np.random.default_rng(0).uniform(-1, 1, x.getLocalSize()))
    y = K.createVecLeft()
    ref = None
    for seq in (1, 2, 4, 8, 16):
        for unr in (1, 2):
            for nt in (1, 0):
                K.setSpmvVariant(64, unr, 0)
                K.setSpmvRowsPerWave(seq)
                K.setSpmvNontemporal(nt)
                for _ in range(3):
                    K.mult(x, y)
                ctx.synchronize()
                ctx.set_profiling(True, only="spmv")
                ctx.reset_stats()
                for _ in range(reps):
                    K.mult(x, y)
                c, ms = ctx.kernel_stats("spmv")
                ctx.set_profiling(False)
                yy = y.getArray()
                if ref is None:
                    ref = yy
                rec = {"seq": seq, "unroll": unr, "nt": nt, "spmv_ms": ms / c,
                       "gbps": K.spmvBytes() / (ms / c * 1e-3) / 1e9, "bitexact": bool(np.array_equal(yy, ref))}
                kb = KSP().create()
                kb.setType("cg")
                pc = PC()
                pc.setType("jacobi")
                kb.setPC(pc)
                kb.setCGSingleReduction(True)
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


if __name__ == "__main__":
    main()
