"""In-process A/B of libkle tuning knobs on the CG loop (config 2 by default).

Variants alternate block by block in ONE process on ONE assembled system, so
box-to-box and process-to-process noise cancels; each block continues the
same fixed-iteration recurrence (kle_ksp_continue) for --its iterations.

  python tools/cg_ab.py '[{"_ksp":"cg"},{"_ksp":"pipecg"}]' [--nelem 20,16,16] [--reps 6] [--its 200]
Prints one JSON line per (rep, variant) and a summary line (median ms/iter).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


DEFAULTS = {"spmv_waves": 0, "spmv_dyn_lds": -1, "spmv_xcd_chunk": 16, "spmv_x_lds": 1, "spmv_dict": 1, "upd_preload": 1, "upd_nt": 2, "spmv_sym": 1, "spmv_sym_det": 1, "spmv_sym_waves": 0, "spmv_sym_early": 0, "spmv_sym_align": 0, "spmv_sym_stpol": 0, "spmv_gsym_stpol": 2, "spmv_sym_tile64": 0, "spmv_sym_tile64_max": 640, "spmv_sym_ovl_b": 50, "spmv_sym_xcd": 0, "spmv_sym_brick": 1, "spmv_gather_wps": 0, "spmv_brick_max": 0, "spmv_brick_rounds": 1, "spmv_brick_split": 0, "spmv_gsym_brick": 1, "upd_unroll": 1, "spmv_brick_pair": 1, "spmv_brick_singles": 1}  # kle_set_tuning defaults


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--nelem", default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--its", type=int, default=200)
    ap.add_argument("--ksp", default="cg")
    ap.add_argument("--mesh", choices=["box", "unstructured"], default="box",
                    help="unstructured: the box written as a Gmsh file of perturbed, rotated, shuffled hexes "
                         "(bench.py --mesh unstructured)")
    a = ap.parse_args()
    variants = json.loads(a.variants)
    import numpy as np

    import pynama_amd as pa
    from pynama_amd.petsc import KSP, PC
    from pynama_amd.runtime import set_tuning
    ctx = pa.get_ctx()
    nelem = [int(v) for v in a.nelem.split(",")]
    cfg = {"domain": {"ngl": a.ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    if a.mesh == "unstructured":
        import tempfile
        from pynama_amd.meshgen import perturbed_box, write_gmsh
        V, Cc, F, T = perturbed_box(3, nelem, seed=5)
        path = os.path.join(tempfile.mkdtemp(prefix="kle_ab_"), "mesh.msh")
        write_gmsh(path, 3, V, Cc, F, T)
        cfg["domain"] = {"ngl": a.ngl, "gmsh-file": path}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    b = K.createVecLeft()
    b.setArray(np.random.default_rng(1).uniform(-1, 1, b.getLocalSize()))
    solvers = {}

    def solver(kt):  # one KSP (and x) per Krylov type, its recurrence started once
        if kt not in solvers:
            ksp = KSP().create()
            ksp.setType(kt)
            pc = PC()
            pc.setType("jacobi")
            ksp.setPC(pc)
            ksp.setCGSingleReduction(True)
            ksp.setOperators(K)
            x = K.createVecRight()
            ksp.setFixedIterations(20)
            ksp.solve(b, x)
            solvers[kt] = (ksp, x)
        return solvers[kt]
    res = {i: [] for i in range(len(variants))}
    for rep in range(a.reps):
        for i, v in enumerate(variants):
            prof = False
            ksp, x = solver(v.get("_ksp", a.ksp))
            for k, val in v.items():
                if k == "_ksp":  # Krylov type of this variant (cg | pipecg)
                    continue
                if k == "_prof_spmv":  # HIP events around every SpMV launch (bench.py's roofline timing)
                    prof = bool(val)
                else:
                    set_tuning(k, val)
            # a fresh fixed-iteration start per block: continuing one recurrence
            # for thousands of iterations runs it past round-off (the scalars
            # turn NaN and every kernel becomes a no-op)
            ksp.setFixedIterations(20)
            ksp.solve(b, x)
            ksp.solveContinue(b, x, 10)  # settle
            ctx.synchronize()
            if prof:
                ctx.set_profiling(True, only="spmv")
                ctx.reset_stats()
            t = time.perf_counter()
            ksp.solveContinue(b, x, a.its)
            ctx.synchronize()
            ms = (time.perf_counter() - t) / a.its * 1e3
            if prof:
                ctx.set_profiling(False)
            for k in v:  # back to the library defaults before the next variant
                if k in DEFAULTS:
                    set_tuning(k, DEFAULTS[k])
            if ksp.getConvergedReason() < 0:
                print(json.dumps({"rep": rep, "variant": v, "invalid": "recurrence diverged (reason %d)"
                                  % ksp.getConvergedReason()}), flush=True)
                continue
            res[i].append(ms)
            print(json.dumps({"rep": rep, "variant": v, "ms_per_iter": ms}), flush=True)
    print(json.dumps({"summary": [{"variant": v, "median_ms": statistics.median(res[i]) if res[i] else None,
                                   "min_ms": min(res[i]) if res[i] else None, "valid_reps": len(res[i])}
                                  for i, v in enumerate(variants)],
                      "nelem": nelem, "ngl": a.ngl, "its": a.its}), flush=True)


if __name__ == "__main__":
    main()
