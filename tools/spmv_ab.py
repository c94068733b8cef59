"""Interleaved A/B timing of SpMV variants (median of rounds), to separate
small differences from box-to-box and run-to-run noise.  GPU tool."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402


def main():
    # [lanes per row, rows per wave, unroll, nt]
    variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [[64, 1, 2, 1], [64, 1, 1, 1]]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
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
    res = {str(v): [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            lpr, seq, unr, nt = v
            K.setSpmvVariant(lpr, unr, 0)
            K.setSpmvRowsPerWave(seq)
            K.setSpmvNontemporal(nt)
            K.mult(x, y)
            ctx.set_profiling(True, only="spmv")
            ctx.reset_stats()
            for _ in range(20):
                K.mult(x, y)
            c, ms = ctx.kernel_stats("spmv")
            ctx.set_profiling(False)
            res[str(v)].append(ms / c)
    for k, v in res.items():
        print(json.dumps({"variant(lpr,seq,unroll,nt)": k, "median_ms": float(np.median(v)), "min_ms": min(v),
                          "max_ms": max(v)}), flush=True)


if __name__ == "__main__":
    main()
