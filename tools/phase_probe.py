"""Per-workgroup phase timeline of the symmetric SpMV tile kernels (probe build).

Loads tools/libkle_probe.so (`make -C pynama_amd/csrc probe`), whose
k_nb_spmv_sym_xl / k_nb_spmv_gsym record per workgroup (s_memrealtime,
100 MHz): start, x in LDS, item loop done, partials stored (after every
wave's vmcnt(0) -- the probe adds that wait and a barrier), HW_ID, XCC_ID.
Prints one JSON summary per run (phase medians / percentiles in us, kernel
span, workgroup-slot utilisation, per-XCD spans) and saves the raw records.

  python tools/phase_probe.py [--mesh box|unstructured] [--nelem 20,16,16] [--ngl 5] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KLE_LIBRARY"] = os.path.join(ROOT, "tools", "libkle_probe.so")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mesh", default="box", choices=["box", "unstructured"])
    ap.add_argument("--nelem", default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "phase"))
    ap.add_argument("--tuning", default="{}", help="JSON of kle_set_tuning knobs (probe bits included)")
    ap.add_argument("--cg", action="store_true",
                    help="record the last SpMV of 20 single-reduction CG iterations (the bench's loop: x is the "
                         "vector the update kernel just wrote) instead of repeated products of one x")
    a = ap.parse_args()
    import numpy as np

    import pynama_amd as pa
    from pynama_amd._lib import load
    from pynama_amd.runtime import set_tuning
    nelem = [int(v) for v in a.nelem.split(",")]
    cfg = {"domain": {"ngl": a.ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * 3, "upper": [1.0] * 3}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    if a.mesh == "unstructured":
        import tempfile
        from pynama_amd.meshgen import perturbed_box, write_gmsh
        V, Cc, F, T = perturbed_box(3, nelem, seed=5)
        path = os.path.join(tempfile.mkdtemp(prefix="kle_phase_"), "mesh.msh")
        write_gmsh(path, 3, V, Cc, F, T)
        cfg["domain"] = {"ngl": a.ngl, "gmsh-file": path}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    for k, v in json.loads(a.tuning).items():  # (build knobs included: set before the build)
        set_tuning(k, v)
    K.setOption(K.Option.SPD, True)  # (symmetric storage below spmv_sym_min_rows too)
    kern = K.spmvKernel()
    slots = 1 << 20
    set_tuning("spmv_sym_probe_ts", slots)
    lib = load()
    occ = {}
    for which in (0, 1):
        for lds in (0, 16384, 32768, 49152, 65536, 81920):
            b = C.c_int()
            if lib.kle_probe_occupancy(which, lds, C.byref(b)) == 0:
                occ[f"{'box' if which == 0 else 'gsym'}@{lds}"] = b.value
    print(json.dumps({"occupancy_api_blocks_per_cu": occ}), flush=True)
    x = K.createVecRight()
    x.setArray(np.random.default_rng(3).uniform(-1, 1, x.getLocalSize()))
    y = K.createVecLeft()
    ctx = pa.get_ctx()
    os.makedirs(a.out, exist_ok=True)
    ksp = None
    if a.cg:
        from pynama_amd.petsc import KSP, PC
        ksp = KSP().create()
        ksp.setType("cg")
        pc = PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setCGSingleReduction(True)
        ksp.setOperators(K)
        ksp.setFixedIterations(20)
        bvec = K.createVecLeft()
        bvec.setArray(np.random.default_rng(1).uniform(-1, 1, bvec.getLocalSize()))
        xs = K.createVecRight()
        ksp.solve(bvec, xs)
    for rep in range(a.reps + 1):
        if ksp is not None:
            ksp.solveContinue(bvec, xs, 20)
        else:
            K.mult(x, y)
        ctx.synchronize()
        buf = np.zeros(slots * 8, dtype=np.uint64)
        rc = lib.kle_probe_timestamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), C.c_int64(slots))
        assert rc == 0
        r = buf.reshape(slots, 8)
        r = r[r[:, 1] != 0]
        if rep == 0:
            continue  # (warm-up)
        t0 = r[:, 1].min()
        st, xr, lp, en = [(r[:, i].astype(np.int64) - int(t0)) / 100.0 for i in (1, 2, 3, 4)]  # us
        fill, loop, store, total = xr - st, lp - xr, en - lp, en - st
        span = en.max()
        xcc = (r[:, 6] & 0xF).astype(int)

        def pct(v):
            return {"p10": float(np.percentile(v, 10)), "med": float(np.median(v)), "p90": float(np.percentile(v, 90)),
                    "mean": float(v.mean())}
        # mean number of workgroups in flight and per-XCD spans
        per_xcd = {int(c): {"n": int((xcc == c).sum()), "span_us": float(en[xcc == c].max() - st[xcc == c].min())}
                   for c in np.unique(xcc)}
        if (r[:, 7] != 0).any():  # (the brick kernel: the latest wave's fill landed, its barrier arrival)
            fi = (r[:, 7] & 0xFFFFFFFF).astype(np.int64) / 100.0
            fl = (r[:, 7] >> 32).astype(np.int64) / 100.0
            extra = {"descriptors_in_max_wave_us": pct(fi), "barrier_arrival_max_wave_us": pct(fl)}
            if (r[:, 0] >> 32).any():  # (the latest wave's start after wave 0's)
                extra["wave_start_spread_us"] = pct((r[:, 0] >> 32).astype(np.int64) / 100.0)
            if (r[:, 5] >> 32).any():  # (the latest wave's first item issued: its row descriptors in)
                extra["first_item_issued_max_wave_us"] = pct((r[:, 5] >> 32).astype(np.int64) / 100.0)
        else:
            extra = {}
        summ = {"rep": rep, "kernel": kern, "mesh": a.mesh, "nelem": nelem, "ngl": a.ngl, "workgroups": int(len(r)),
                "span_us": float(span), "sum_total_us": float(total.sum()),
                "mean_in_flight": float(total.sum() / span),
                "fill_us": pct(fill), "loop_us": pct(loop), "store_us": pct(store), "total_us": pct(total),
                "share": {"fill": float(fill.sum() / total.sum()), "loop": float(loop.sum() / total.sum()),
                          "store": float(store.sum() / total.sum())},
                "last_start_us": float(st.max()), "first_end_us": float(en.min()),
                "loop_deciles_us": [float(np.percentile(loop, q)) for q in range(0, 101, 10)],
                "per_xcd": per_xcd, "tuning": json.loads(a.tuning), "cg": a.cg, **extra}
        print(json.dumps(summ), flush=True)
        np.save(os.path.join(a.out, f"phase_{a.mesh}_{rep}.npy"), r)
    set_tuning("spmv_sym_probe_ts", 0)


if __name__ == "__main__":
    main()
