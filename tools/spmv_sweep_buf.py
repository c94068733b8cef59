"""Time the buffer-descriptor SpMV cache-policy variants (GPU tool)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402

ctx = pa.get_ctx()
cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0.0] * 3, "upper": [1.0] * 3}},
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
ref = None
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
only = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(0, 9))
for v in only:
    K.setSpmvBufferVariant(v)
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
    print(json.dumps({"buf_variant": v, "spmv_ms": ms / c, "gbps": nbytes / (ms / c * 1e-3) / 1e9,
                      "maxdiff": float(np.abs(yy - ref).max() / np.abs(ref).max())}), flush=True)
