"""Fixed-iteration CG timing with and without per-kernel event profiling
(how much the events themselves cost).  GPU tool, not product."""
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
    its = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ctx = pa.get_ctx()
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    b = K.createVecLeft()
    b.setArray(np.random.default_rng(0).uniform(-1, 1, b.getLocalSize()))
    out = {}
    for fused in (False, True):
        kb = KSP().create()
        kb.setType("cg")
        pc = PC()
        pc.setType("jacobi")
        kb.setPC(pc)
        kb.setCGSingleReduction(True)
        kb.setFusedDot(fused)
        kb.setOperators(K)
        x = K.createVecRight()
        kb.setFixedIterations(20)
        kb.solve(b, x)
        kb.setFixedIterations(its)
        for prof in (False, True):
            ctx.set_profiling(prof)
            ctx.reset_stats()
            ctx.synchronize()
            t = time.perf_counter()
            kb.solve(b, x)
            ctx.synchronize()
            ms = (time.perf_counter() - t) / its * 1e3
            rec = {"ms_per_it": ms}
            if prof:
                for k in ("spmv", "cg_update", "dot", "reduce"):
                    c, kms = ctx.kernel_stats(k)
                    rec[k] = kms / max(c, 1)
            ctx.set_profiling(False)
            out[f"fused{int(fused)}_prof{int(prof)}"] = rec
            print(json.dumps({f"fused{int(fused)}_prof{int(prof)}": rec}), flush=True)


if __name__ == "__main__":
    main()
