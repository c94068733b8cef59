"""One-rank RCCL communicator (KLE_RCCL_SELF=1) running the single-reduction
and pipelined CG loops on a 1/8-slab mesh, for `rocprofv3 --kernel-trace`:
the trace shows the resources (LDS, VGPRs, workgroup size) of the RCCL
kernels that run beside the SpMV on N > 1 ranks.
  KLE_RCCL_SELF=1 rocprofv3 --kernel-trace -d DIR -o rccl --output-format csv -- python3 tools/rccl_self_kernels.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    import pynama_amd as pa
    from pynama_amd.petsc import KSP, PC
    assert os.environ.get("KLE_RCCL_SELF") == "1"
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 2], "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    b = K.createVecLeft()
    b.setArray(np.random.default_rng(1).uniform(-1, 1, b.getLocalSize()))
    for kt in ("cg", "pipecg"):
        ksp = KSP().create()
        ksp.setType(kt)
        pc = PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setCGSingleReduction(True)
        ksp.setOperators(K)
        x = K.createVecRight()
        ksp.setFixedIterations(50)
        ksp.solve(b, x)
        print(kt, ksp.getConvergedReason(), flush=True)


if __name__ == "__main__":
    main()
