"""SpMV time over fresh allocations of the symmetric storage's value array
(kle_mat_move_values), with and without the contiguous allocator
(alloc_contig): does where the array lands set the product's speed?

  python tools/placement_spread.py [--nelem 20,16,16] [--ngl 5] [--moves 8] [--its 20]

One JSON line per allocation, then a summary per allocator (min / median /
max us and the spread (max - min) / min over the allocations).
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nelem", default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--moves", type=int, default=8)
    ap.add_argument("--its", type=int, default=20)
    ap.add_argument("--contig", default="1,0", help="alloc_contig values to compare")
    ap.add_argument("--pads", default="0", help="spmv_brick_pad values (doubles) to compare (rebuilds)")
    ap.add_argument("--stay", action="store_true", help="no moves: the same allocation timed each time (noise floor)")
    a = ap.parse_args()
    import pynama_amd as pa
    from pynama_amd.runtime import get_ctx, set_tuning
    nelem = [int(v) for v in a.nelem.split(",")]
    cfg = {"domain": {"ngl": a.ngl, "box-mesh": {"nelem": nelem, "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    ctx = get_ctx()
    x = K.createVecRight()
    y = K.createVecLeft()
    x.setArray(np.random.default_rng(1).uniform(-1, 1, x.getLocalSize()))
    K.mult(x, y)
    y0 = y.getArray().copy()
    res = {}
    for pad in [int(v) for v in a.pads.split(",")]:
      set_tuning("spmv_brick_pad", pad)
      K.setOption(K.Option.SPD, True)
      for rep in range(a.moves):
        for contig in [int(v) for v in a.contig.split(",")]:
            set_tuning("alloc_contig", contig)
            if not a.stay:
                K.moveValues(256 * rep)
            K.mult(x, y)
            same = bool(np.array_equal(y.getArray(), y0))
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
            us = 1e3 * ms / c
            res.setdefault(f"contig{contig}_pad{pad}", []).append(us)
            print(json.dumps({"move": rep, "shift": 256 * rep, "contig": contig, "pad": pad, "spmv_us": us,
                              "same_y": same,
                              "got_contiguous": K.getAllocInfo()["symmetric_values_contiguous"],
                              "addr": hex(K.getAllocInfo()["symmetric_values_address"]),
                              "kernel": K.spmvKernel()}), flush=True)
    set_tuning("alloc_contig", 1)
    set_tuning("spmv_brick_pad", 0)
    print(json.dumps({"summary": {str(k): {"min_us": min(v), "median_us": statistics.median(v), "max_us": max(v),
                                           "spread": (max(v) - min(v)) / min(v)} for k, v in res.items()},
                      "nelem": nelem, "ngl": a.ngl}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
