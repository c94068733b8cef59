"""Interleaved A/B: specialised default SpMV kernel vs the generic one on the
bench matrix.  GPU tool (tools/, not product)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    ctx = pa.get_ctx()
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0.0] * 3, "upper": [1.0] * 3}},
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
    res = {}
    for _ in range(rounds):
        for fast in (1, 0):
            K.setSpmvFast(fast)
            K.mult(x, y)
            ctx.set_profiling(True, only="spmv")
            ctx.reset_stats()
            for _ in range(20):
                K.mult(x, y)
            c, ms = ctx.kernel_stats("spmv")
            ctx.set_profiling(False)
            res.setdefault(fast, []).append(ms / c)
    for k, v in res.items():
        print(json.dumps({"fast": k, "median_ms": float(np.median(v)), "min_ms": min(v),
                          "gbps": K.spmvBytes() / (np.median(v) * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
