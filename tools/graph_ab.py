"""A/B: single-rank CG loop replayed from a hipGraph (KLE_GRAPH=1, default)
vs stream launches (KLE_GRAPH=0); fixed iterations, no per-launch timing."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(nelem, ngl, steps=200, reps=4):
    import pynama_amd as pa
    from pynama_amd import fields
    from pynama_amd.petsc import KSP, PC
    ctx = pa.get_ctx()
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    ctx.synchronize()
    t = time.perf_counter()
    mat.build(buildOperators=False)
    ctx.synchronize()
    t_asm = time.perf_counter() - t
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    f = fields.get("taylor_green3d")
    vort = mat.Rw.createVecRight()
    vort.setArray(f.vorticity(dom.getFullCoordArray(), f.alpha(0.02, 0.0)))
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, 0.02)
    b = sol.rhs(vort).copy()
    K = mat.K
    kb = KSP().create()
    kb.setType("cg")
    pc = PC()
    pc.setType("jacobi")
    kb.setPC(pc)
    kb.setCGSingleReduction(True)
    kb.setOperators(K)
    kb.setUp()
    x = K.createVecRight()
    out = {"nelem": nelem, "ngl": ngl, "assembly_s": t_asm,
           "host_pattern": os.environ.get("KLE_HOST_PATTERN", "0")}
    ys = K.createVecLeft()
    for _ in range(10):
        K.mult(b, ys)
    ctx.set_profiling(True, only="spmv")
    ctx.reset_stats()
    for _ in range(100):
        K.mult(b, ys)
    c, ms = ctx.kernel_stats("spmv")
    ctx.set_profiling(False)
    out["spmv_ms"] = ms / c
    for mode in ("1", "0") * reps:
        os.environ["KLE_GRAPH"] = mode  # 1: graph replay (opt-in), 0: stream launches
        kb.setFixedIterations(20)
        kb.solve(b, x)
        kb.setFixedIterations(steps)
        ctx.synchronize()
        t = time.perf_counter()
        kb.solve(b, x)
        ctx.synchronize()
        ms = (time.perf_counter() - t) / steps * 1e3
        out.setdefault("graph" if mode == "1" else "stream", []).append(ms)
    # converged solve equal either way
    res = {}
    for mode in ("1", "0"):
        os.environ["KLE_GRAPH"] = mode  # 1: graph replay (opt-in), 0: stream launches
        ksp = sol.getKSP()
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=100000)
        vel.set(0.0)
        dom.applyBoundaryConditions(vel, "velocity", 0.0, 0.02)
        sol.solve(vort)
        res[mode] = (ksp.getIterationNumber(), ksp.getTrueRelativeResidual(), vel.getArray().copy())
    out["solve_its"] = [res["1"][0], res["0"][0]]
    out["solve_true_rel"] = [res["1"][1], res["0"][1]]
    out["solve_bitwise_equal"] = bool((res["1"][2] == res["0"][2]).all())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    ne = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [20, 16, 16]
    main(ne, int(sys.argv[2]) if len(sys.argv) > 2 else 5)
