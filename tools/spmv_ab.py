"""In-process A/B of SpMV tuning knobs on config 2's K (or --nelem/--ngl):
variants alternate block by block in ONE process; each block times --reps
products with HIP events around every SpMV launch (the gather included).
Knobs that are timing probes ("spmv_sym_probe") give wrong products on
purpose and exist only in the probe build: the script then loads
tools/libkle_probe.so (`make -C pynama_amd/csrc probe`) instead of libkle.so.

  python tools/spmv_ab.py '[{},{"spmv_sym_probe":1}]' [--nelem 20,16,16] [--reps 4] [--its 100]
"""
import argparse
import json
import os
import statistics
import sys

if "spmv_sym_probe" in " ".join(sys.argv[1:]):
    os.environ["KLE_LIBRARY"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkle_probe.so")
BUILD_KNOBS = {"spmv_brick_pair", "spmv_brick_singles", "spmv_gsym_brick", "spmv_brick_rounds", "spmv_brick_split", "spmv_brick_max", "spmv_sym_brick", "spmv_sym_tz", "spmv_gsym_rows", "spmv_gsym_waves", "spmv_sym_align", "spmv_sym_tile64", "spmv_sym_tile64_max"}  # read when the symmetric storage is built
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--nelem", default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--its", type=int, default=100)
    ap.add_argument("--mesh", choices=["box", "unstructured"], default="box",
                    help="unstructured: the box written as a Gmsh file of perturbed, rotated, shuffled hexes")
    a = ap.parse_args()
    import numpy as np
    import pynama_amd as pa
    from pynama_amd.runtime import get_tuning, set_tuning
    from cg_ab import DEFAULTS
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
    K.setOption(K.Option.SPD, True)
    x = K.createVecRight()
    y = K.createVecLeft()
    x.setArray(np.random.default_rng(1).uniform(-1, 1, x.getLocalSize()))
    variants = json.loads(a.variants)
    res = {i: [] for i in range(len(variants))}
    for rep in range(a.reps):
        for i, v in enumerate(variants):
            for k, val in v.items():
                set_tuning(k, val)
            if BUILD_KNOBS & set(v):
                K.setOption(K.Option.SPD, True)  # (re)build the symmetric storage with them
            name = K.spmvKernel()
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
            for k in v:
                if k in DEFAULTS:
                    set_tuning(k, DEFAULTS[k])
                elif k in ("spmv_sym_probe", "spmv_sym_tz"):
                    set_tuning(k, 0)
                elif k == "spmv_gsym_rows":
                    set_tuning(k, 64)
                elif k == "spmv_gsym_waves":
                    set_tuning(k, 0)
            if BUILD_KNOBS & set(v):
                K.setOption(K.Option.SPD, True)
            res[i].append(ms / c)
            print(json.dumps({"rep": rep, "variant": v, "kernel": name, "spmv_ms": ms / c}), flush=True)
    print(json.dumps({"summary": [{"variant": v, "median_ms": statistics.median(res[i]), "min_ms": min(res[i])}
                                  for i, v in enumerate(variants)], "nelem": nelem, "ngl": a.ngl,
                      "mesh": a.mesh, "spmv_bytes": K.spmvBytes()}), flush=True)


if __name__ == "__main__":
    main()
