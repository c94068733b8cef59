"""Interleaved A/B of the node-block value layouts (0 padded streams, 1 chunked
+ packed tail) on the bench matrix, with structured columns on and off.
GPU tool (tools/, not product)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402
from pynama_amd.runtime import set_value_layout  # noqa: E402


def build(layout):
    set_value_layout(layout)
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    return dom, mat


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    ctx = pa.get_ctx()
    mats = {lay: build(lay) for lay in (0, 1)}
    x = mats[0][1].K.createVecRight()
    x.setArray(np.random.default_rng(0).uniform(-1, 1, x.getLocalSize()))
    res = {}
    ys = {}
    for _ in range(rounds):
        for lay in (0, 1):
            K = mats[lay][1].K
            for st in (1, 0):
                K.setSpmvStructured(st)
                y = K.createVecLeft()
                K.mult(x, y)
                ctx.set_profiling(True, only="spmv")
                ctx.reset_stats()
                for _ in range(20):
                    K.mult(x, y)
                c, ms = ctx.kernel_stats("spmv")
                ctx.set_profiling(False)
                res.setdefault((lay, st), []).append(ms / c)
                ys[(lay, st)] = y.getArray()
    ref = ys[(0, 0)]
    for (lay, st), v in res.items():
        print(json.dumps({"layout": lay, "structured": st, "median_ms": float(np.median(v)), "min_ms": min(v),
                          "bytes": mats[lay][1].K.spmvBytes() if st else None,
                          "bitexact": bool(np.array_equal(ys[(lay, st)], ref))}), flush=True)


if __name__ == "__main__":
    main()
