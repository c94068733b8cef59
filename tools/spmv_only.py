"""Run the bench-matrix SpMV a fixed number of times (for rocprofv3 PMC passes).
GPU tool, not product.  Usage: python tools/spmv_only.py [reps] [lpr unroll persistent]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pynama_amd as pa  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0.0] * 3, "upper": [1.0] * 3}},
       "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
dom = pa.Domain()
dom.configure(cfg)
dom.setUp()
mat = pa.MatFS()
mat.setDomain(dom)
mat.build()
K = mat.K
if len(sys.argv) > 4:
    K.setSpmvVariant(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
if len(sys.argv) > 6:
    K.setSpmvLayout(int(sys.argv[5]), int(sys.argv[6]))
x = K.createVecRight()
x.setArray(np.random.default_rng(0).uniform(-1, 1, x.getLocalSize()))
y = K.createVecLeft()
for _ in range(reps):
    K.mult(x, y)
pa.get_ctx().synchronize()
print("spmv bytes/launch", K.spmvBytes(), "reps", reps)
