"""Benchmark: KLE CG iterations/s + SpMV GB/s vs the HBM roofline on the
BASELINE.json config 2 workload (3-D KLE Laplacian, structured hex mesh
[20,16,16], p=4 / ngl=5, ~1M DoF, Taylor-Green-3D Dirichlet data).

  python bench.py [--gpus N] [--steps K] [--warmup W]
      (N > 1: starts torch.distributed.run with N ranks itself)
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

A "step" is one CG iteration on the assembled device matrix (single-
reduction CG + Jacobi: the fused vector update whose prologue applies the
previous scalar stage, the SpMV, the (u, A u) partials; pipelined CG on N>1);
the warm-up solve starts the recurrence and the K timed steps continue it
(no restart inside the timed region), between barriers, max over ranks.  Assembly (device
element kernels + gather) is untimed setup.  A full solve to rtol 1e-10 is
run once for the convergence record.  The roofline uses HIP-event timings of
the SpMV kernel inside the timed region and the algorithmic bytes of the
node-block format; `traffic` comes from the rocprofv3 PMC pass recorded in
profiles/ (or null).  cpu_baseline: the C oracle's CSR CG on the same
matrix, OpenMP on the host cores, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)
METRIC = "KLE CG iters/sec + SpMV GB/s (vs HBM roofline), 1M-DoF p=4 hex mesh"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nelem", type=str, default="20,16,16")
    ap.add_argument("--ngl", type=int, default=5)
    ap.add_argument("--mesh", choices=["box", "unstructured"], default="box",
                    help="box: structured box mesh (config 2/3); unstructured: the same box as a Gmsh file of "
                         "perturbed, randomly rotated and shuffled hexes (config 5's irregular path)")
    ap.add_argument("--msh", type=str, default=None, help="read this Gmsh 4.1 file instead (implies unstructured)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="OpenMP threads of the CPU baseline: 0 the runtime default (OMP_NUM_THREADS), "
                         "-1 every thread of the affinity mask")
    ap.add_argument("--no-solve", action="store_true")
    ap.add_argument("--no-aij", dest="aij", action="store_false",
                    help="skip the scalar-CSR (aij) SpMV leg (default: timed at N = 1)")
    ap.add_argument("--layout", type=int, choices=[0, 1], default=1,
                    help="node-block value layout: 1 = 16-block chunks + packed tail, 0 = padded row streams")
    ap.add_argument("--pad", type=int, default=16, help="row padding quantum of layout 0 (blocks)")
    ap.add_argument("--ops", dest="ops", action="store_const", const="on", default="auto",
                    help="also assemble Curl/SrT/DivSrT and time their SpMVs and the evalRHS operator chain "
                         "(default: at N = 1)")
    ap.add_argument("--no-ops", dest="ops", action="store_const", const="off")
    ap.add_argument("--ksp", choices=["auto", "cg", "pipecg"], default="auto",
                    help="auto: single-reduction CG on one GPU, pipelined CG (allreduce beside the SpMV) on N>1")
    ap.add_argument("--classic-cg", action="store_true",
                    help="two reductions per iteration instead of the single-reduction (Chronopoulos-Gear) CG")
    ap.add_argument("--traffic", type=str, default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args()


def bench_operators(pa, mat, ctx, sol, dim, reps=20):
    """Operators row: device assembly time, per-operator SpMV
    time / useful GB/s, and the evalRHS operator chain (base_problem.py:127-136)
    after the KLE solve: VtensV, SrT, scale/axpy, DivSrT, scale, Curl."""
    import numpy as np
    from pynama_amd._lib import call
    ctx.synchronize()
    t = time.perf_counter()
    mat.buildOperators()
    ctx.synchronize()
    out = {"assembly_s": time.perf_counter() - t}
    op = mat.getOperators()
    rng = np.random.default_rng(1)
    for nm in ("Curl", "SrT", "DivSrT"):
        A = getattr(op, nm)
        x, y = A.createVecRight(), A.createVecLeft()
        x.setArray(rng.uniform(-1, 1, x.getLocalSize()))
        A.mult(x, y)
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(reps):
            A.mult(x, y)
        c, ms = ctx.kernel_stats("spmv")
        ctx.set_profiling(False)
        nb = A.spmvBytes()
        out[nm] = {"avg_ms": ms / c, "bytes": nb, "gbps": nb / (ms / c * 1e-3) / 1e9,
                   "frac": nb / (ms / c * 1e-3) / 1e9 / HBM_PEAK_GBS}
    vel = sol.getSolution()
    vt = op.SrT.createVecLeft()
    aux = vt.duplicate()
    rhs = vel.duplicate()
    f = op.Curl.createVecLeft()
    rho, mu = 0.5, 0.01

    def chain():
        call("kle_vec_tensor_square", vel._h, dim, vt._h)
        op.SrT.mult(vel, aux)
        aux.scale(2.0 * mu)
        aux.axpy(-rho, vt)
        op.DivSrT.mult(aux, rhs)
        rhs.scale(1 / rho)
        op.Curl.mult(rhs, f)
    chain()
    ctx.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        chain()
    ctx.synchronize()
    out["evalRHS_chain_ms"] = (time.perf_counter() - t) / reps * 1e3
    return out


def comm_timeout_s():
    """Deadline (s) for every rank-to-rank rendezvous: the gloo bootstrap here
    and ncclCommInitRank inside libkle (KLE_COMM_TIMEOUT_S, default 300)."""
    return float(os.environ.get("KLE_COMM_TIMEOUT_S", "300"))


def init_dist(n):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        import datetime

        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=comm_timeout_s()))
        return dist
    return None


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, deadline_s=None):
    """`python bench.py --gpus N` without a torchrun around it: start
    torch.distributed.run with N ranks (one per GPU, LOCAL_RANK = device) as a
    child process group, forward rank 0's JSON line, and exit with the
    children's status.  This process never touches HIP (nothing here imports
    torch or pynama_amd), and it never exec()s: the ranks are children.  A
    rank that fails makes torchrun stop the others; a launch that exceeds the
    deadline (KLE_BENCH_DEADLINE_S, default 1200 s) is killed as a group and
    exits 124."""
    import signal
    import subprocess
    import threading
    if deadline_s is None:
        deadline_s = float(os.environ.get("KLE_BENCH_DEADLINE_S", "1200"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, start_new_session=True)
    lines = []

    def pump():
        for ln in proc.stdout:
            if ln.startswith("{"):
                lines.append(ln.strip())
            else:
                sys.stderr.write(ln)
    t = threading.Thread(target=pump, daemon=True)
    t.start()
    try:
        rc = proc.wait(timeout=deadline_s)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
        proc.wait()
        sys.stderr.write(f"bench: {n}-rank launch exceeded {deadline_s:.0f} s, killed\n")
        return 124
    t.join(timeout=10)
    if rc != 0:
        sys.stderr.write(f"bench: {n}-rank launch failed (exit {rc})\n")
        return rc
    if len(lines) != 1:
        sys.stderr.write(f"bench: expected one JSON line from rank 0, got {len(lines)}\n")
        return 1
    print(lines[0], flush=True)
    return 0


def main():
    args = parse()
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    dist = init_dist(args.gpus)
    import numpy as np

    import pynama_amd as pa
    from pynama_amd import fields
    from pynama_amd.petsc import KSP, PC

    ctx = pa.get_ctx()
    pa.runtime.set_row_padding(args.pad)
    pa.runtime.set_value_layout(args.layout)
    rank, nranks = ctx.rank, ctx.nranks
    nelem = [int(v) for v in args.nelem.split(",")]
    dim = len(nelem)
    cfg = {"domain": {"ngl": args.ngl, "box-mesh": {"nelem": nelem, "lower": [0.0] * dim, "upper": [1.0] * dim}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d" if dim == 3 else "taylor_green"}}}
    mesh_kind = "box"
    t_mesh = 0.0
    if args.msh or args.mesh == "unstructured":
        mesh_kind = "unstructured"
        path = args.msh
        if path is None:
            import tempfile
            from pynama_amd.meshgen import perturbed_box, write_gmsh
            tg = time.perf_counter()
            V, Cc, F, T = perturbed_box(dim, nelem, seed=5)
            path = os.path.join(tempfile.mkdtemp(prefix="kle_bench_"), "mesh.msh")
            write_gmsh(path, dim, V, Cc, F, T)
            t_mesh = time.perf_counter() - tg
        cfg["domain"] = {"ngl": args.ngl, "gmsh-file": path}
    # (Domain.create partitions Gmsh meshes by the domain entry's
    # "partitioner", inertial bisection unless it names another)
    partitioner = cfg["domain"].get("partitioner", "inertial")
    t0 = time.perf_counter()
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    ctx.synchronize()
    t1 = time.perf_counter()
    mat.build(buildOperators=False)
    ctx.synchronize()
    t_asm = time.perf_counter() - t1
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    f = fields.get(cfg["boundary-conditions"]["custom-func"]["name"])
    nu = 0.01 / 0.5  # taylor-green3d.yaml material (rho 0.5, mu 0.01)
    vort = mat.Rw.createVecRight()
    vort.setArray(f.vorticity(dom.getFullCoordArray(), f.alpha(nu, 0.0)))
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, nu)
    b = sol.rhs(vort).copy()
    t_setup = time.perf_counter() - t0

    K = mat.K
    n_global = K.getSize()[0]
    info = K.getInfo()
    nnz_local = info["nz_used"]
    spmv_bytes_local = K.spmvBytes()

    # --- full solve to convergence (correctness record, untimed for the metric)
    solve = {}
    if not args.no_solve:
        ksp = sol.getKSP()
        ksp.setType("pipecg" if (args.ksp == "pipecg" or (args.ksp == "auto" and nranks > 1)) else "cg")
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=200000)
        ksp.setCGSingleReduction(not args.classic_cg)
        # (CG and pipelined CG stop on their recursive residual; when the
        # true residual misses rtol -- the pipelined recurrence drifts to
        # 1.1-1.3e-10 -- libkle's default correction solve brings it under,
        # kle_ksp.hip refine; its iterations are part of the count)
        ctx.barrier()
        ts = time.perf_counter()
        sol.solve(vort)
        ctx.barrier()
        solve = {"rtol": 1e-10, "iterations": ksp.getIterationNumber(), "reason": ksp.getConvergedReason(),
                 "true_rel_residual": ksp.getTrueRelativeResidual(), "seconds": time.perf_counter() - ts,
                 "correction_iterations": ksp.getCorrectionIterations()}

    # --- timed fixed-iteration CG
    ksp_type = args.ksp if args.ksp != "auto" else ("pipecg" if nranks > 1 else "cg")
    kb = KSP().create()
    kb.setType(ksp_type)
    pc = PC()
    pc.setType("jacobi")
    kb.setPC(pc)
    kb.setCGSingleReduction(not args.classic_cg)
    kb.setOperators(K)
    kb.setUp()
    x = K.createVecRight()
    # the warm-up solve starts the recurrence (r = b, w = A u, first scalars);
    # the timed region continues it for exactly `steps` iterations
    kb.setFixedIterations(max(args.warmup, 1))
    kb.solve(b, x)
    # HIP events around one SpMV launch in `every` (sampled live inside the
    # timed region; timing every launch costs 0.8 % of an iteration at config
    # 2 and 6 % on a 1/8 slab: profiles/r02/cg_ab_events_*.jsonl)
    every = max(1, min(8, args.steps // 5))
    ctx.set_profiling(True, only="spmv", every=every)
    ctx.reset_stats()
    ctx.barrier()
    if dist is not None:
        dist.barrier()
    t_start = time.perf_counter()
    kb.solveContinue(b, x, args.steps)
    ctx.barrier()
    t_loc = time.perf_counter() - t_start
    ctx.set_profiling(False)
    if kb.getConvergedReason() < 0:
        # a recurrence continued far past round-off turns its scalars NaN and
        # every kernel into a no-op: such a timing would not be K iterations
        raise SystemExit(f"bench: the timed CG recurrence diverged (reason {kb.getConvergedReason()}); "
                         f"use fewer --steps")
    spmv_cnt, spmv_ms = ctx.kernel_stats("spmv")
    # per-kernel breakdown from a separate, untimed pass with every launch timed
    nb_its = min(args.steps, 50)
    ctx.set_profiling(True)
    ctx.reset_stats()
    kb.solveContinue(b, x, nb_its)
    ctx.set_profiling(False)
    brk = {k: ctx.kernel_stats(k)[1] / nb_its for k in ("spmv", "cg_update", "p_update", "reduce",
                                                        "halo", "allreduce")}
    t_max = t_loc
    # the timed products' algorithmic bytes (the bricks' own share where the CG
    # update gathers a split product; else K's, = the plain leg's)
    prod_bytes = kb.getProductBytes() or spmv_bytes_local
    tot_bytes = prod_bytes
    tot_nnz = nnz_local
    spmv_avg_ms = spmv_ms / max(spmv_cnt, 1)
    if dist is not None:
        import torch
        tt = torch.tensor([t_loc, spmv_avg_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max, spmv_avg_max = float(tt[0]), float(tt[1])
        sb = torch.tensor([prod_bytes, float(nnz_local)], dtype=torch.float64)
        dist.all_reduce(sb, op=dist.ReduceOp.SUM)
        tot_bytes, tot_nnz = float(sb[0]), int(sb[1])
    else:
        spmv_avg_max = spmv_avg_ms
    # which device each rank ran on (one distinct GPU per rank under RCCL),
    # what the RCCL communicator itself reports, and each rank's SpMV time
    dev = ctx.device_info()
    dev["rccl_count"], dev["rccl_rank"] = ctx.comm_info()
    dev["spmv_ms"] = spmv_avg_ms
    devices = [dev]
    if dist is not None:
        devices = [None] * nranks
        dist.all_gather_object(devices, dev)
    if "torch" in sys.modules:  # torch is only the launcher's plumbing here
        import torch
        if torch.cuda.is_initialized():  # never create a torch context just to sync it
            torch.cuda.synchronize()

    iters_per_s = args.steps / t_max
    achieved = tot_bytes / (spmv_avg_max * 1e-3) / 1e9 if spmv_avg_max > 0 else None
    # SURVEY 8(d)'s scalar-CSR bytes for the same product (12 B per nonzero,
    # int32 row pointers, x and y once): the rate a CSR kernel would need to
    # match this launch
    csr_bytes = 12.0 * tot_nnz + 4.0 * (n_global + 1) + 16.0 * n_global
    csr_equiv = csr_bytes / (spmv_avg_max * 1e-3) / 1e9 if spmv_avg_max > 0 else None

    # plain SpMV leg: x = uniform[-1,1) from splitmix64 seeded
    # 0x5EED, 10 warm-ups, 200 timed repetitions of y = K x
    lo, hi = K.getOwnershipRange()
    xs = K.createVecRight()
    xs.setArray(splitmix_uniform(0x5EED, lo, hi))
    ys = K.createVecLeft()
    for _ in range(10):
        K.mult(xs, ys)
    ctx.set_profiling(True, only="spmv")
    ctx.reset_stats()
    for _ in range(200):
        K.mult(xs, ys)
    pc_, pms = ctx.kernel_stats("spmv")
    ctx.set_profiling(False)
    # each rank's own part alone (no halo; ranks take turns, so ranks that
    # share a GPU do not slow each other): the per-rank skew of N > 1
    local_ms = None
    if dist is not None:
        for r in range(nranks):
            dist.barrier()
            if r == rank:
                try:
                    local_ms = K.timeLocalSpmv(xs, ys, 50)
                except pa.Error:  # (not a box-brick part)
                    local_ms = None
        dist.barrier()
    local_all = [local_ms]
    if dist is not None:
        local_all = [None] * nranks
        dist.all_gather_object(local_all, local_ms)
    spmv_plain = {"kernel": spmv_kernel(K, args.layout, args.ngl), "reps": pc_, "avg_ms": pms / max(pc_, 1),
                  "bytes": spmv_bytes_local,
                  "gbps": spmv_bytes_local / (pms / max(pc_, 1) * 1e-3) / 1e9,
                  "x": "uniform[-1,1) from splitmix64(0x5EED), global index order"}

    aij = None
    if args.aij and nranks == 1:
        A = K.convert("aij")
        xa = A.createVecRight()
        ya = A.createVecLeft()
        xa.setArray(np.random.default_rng(0).uniform(-1, 1, xa.getLocalSize()))
        for _ in range(5):
            A.mult(xa, ya)
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(50):
            A.mult(xa, ya)
        ctx.synchronize()
        c, ms = ctx.kernel_stats("spmv")
        ctx.set_profiling(False)
        ab = A.spmvBytes()
        aij = {"format": "aij (scalar CSR, int32 cols)", "bytes_per_spmv": ab, "avg_ms": ms / c,
               "gbps": ab / (ms / c * 1e-3) / 1e9, "frac": ab / (ms / c * 1e-3) / 1e9 / HBM_PEAK_GBS}
        del A

    # the kernel(s) the timed products ran (the bricks alone where the CG
    # update gathers the split product itself); the plain leg's is K's own
    kname = kb.getProductKernel() or spmv_kernel(K, args.layout, args.ngl)
    tkey = (f"{nelem}-{args.ngl}-{nranks}-" + ("umesh-" if mesh_kind != "box" else "") +
            ("chunk" if args.layout == 1 else f"pad{args.pad}") +
            "-nt-u1" + ("-struct" if K.isStructured() else "") +
            ("-sym" if kname.startswith("k_nb_spmv_sym") else
             "-gsym" if kname.startswith("k_nb_spmv_gsym") else
             {"k_nb_spmv_xl<8>": "-xl", "k_nb_spmv_dict": "-dict"}.get(kname, "")))
    traffic, traffic_status = lookup_traffic(args.traffic, tkey, kname, prod_bytes)

    ops = None
    if args.ops == "on" or (args.ops == "auto" and nranks == 1):
        try:
            ops = bench_operators(pa, mat, ctx, sol, dim)
        except pa.Error as e:
            # (the reference's full operator matrices at p = 6 on 3.9M DoF do
            # not fit beside K: reported, not fatal -- they are off the path)
            if args.ops == "on" or e.ierr != 55:
                raise
            ops = {"skipped": str(e)}

    cpu = None
    if rank == 0 and nranks == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(K, b, args.cpu_seconds, args.cpu_threads)

    if rank == 0:
        stream = ctx.stream_copy_gbps(1 << 30, 10)
        stream_rd = ctx.stream_read_gbps(1 << 32, 10)
        line = {
            "metric": METRIC,
            "value": iters_per_s,
            "unit": "CG iters/s",
            "n_gpus": nranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (Taylor-Green-3D vorticity + Dirichlet velocity on a generated box mesh)"
                     if mesh_kind == "box" else
                     "synthetic (Taylor-Green-3D vorticity + Dirichlet velocity on a generated unstructured hex "
                     "mesh: perturbed, rotated, shuffled cells read from Gmsh 4.1)"),
            "config": {"workload": (f"KLE Laplacian {dim}-D box {nelem} ngl={args.ngl} (p={args.ngl - 1}), "
                                    if mesh_kind == "box" else
                                    f"KLE Laplacian {dim}-D unstructured hex mesh ({int(np.prod(nelem))} cells, "
                                    f"{nelem} box topology) ngl={args.ngl} (p={args.ngl - 1}), ") +
                                   f"TG-{dim}D Dirichlet on all faces; one CG(+Jacobi) iteration per step",
                       "mesh": mesh_kind,
                       "nelem": nelem, "ngl": args.ngl, "n_dof": n_global, "nnz_K": tot_nnz,
                       "ksp": ksp_type if ksp_type == "pipecg" else
                       ("cg" if args.classic_cg else "cg (single reduction, Chronopoulos-Gear)"),
                       "pc": "jacobi", "matrix_format": info["format"], "value_layout": "chunk16+tail" if args.layout == 1 else f"row streams padded to {args.pad}",
                       "structured_columns": K.isStructured(),
                       "symmetric_storage": K.isSymmetricStorage(),
                       "parallelism": ((f"z-slab x{nranks}" if mesh_kind == "box" else
                                        f"cell slabs along the most-layered axis x{nranks}"
                                        if partitioner == "slab" else
                                        f"inertial recursive bisection x{nranks}") +
                                       ("" if nranks == 1 else
                                        " (RCCL halo + allreduce)" if dev["transport"] == "rccl" else
                                        " (IPC mailbox halo + allreduce: copy engines + stream wait/write-value)"
                                        if dev["transport"] == "ipc" else
                                        " (host-staged halo + allreduce over gloo, ranks sharing a GPU: test only)")),
                       "devices": [f"{d['device']}@{d['pci_bus_id']}" for d in devices],
                       # ncclCommCount / ncclCommUserRank per rank (0 / -1: no RCCL communicator)
                       "rccl_ranks": devices[0]["rccl_count"],
                       "rccl_user_ranks": [d["rccl_rank"] for d in devices],
                       "spmv_ms_per_rank": [d["spmv_ms"] for d in devices],
                       # each rank's part alone, ranks in turn (no halo): kle_mat_time_local_spmv
                       "spmv_local_ms_per_rank": local_all},
            # N > 1: bytes of all ranks over the slowest rank's SpMV time,
            # against N x the per-GPU peak
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS * nranks, "unit": "GB/s",
                         "frac": achieved / (HBM_PEAK_GBS * nranks) if achieved else None, "traffic": traffic,
                         "traffic_status": traffic_status, "traffic_key": tkey,
                         "traffic_over_bytes": traffic / prod_bytes if traffic else None,
                         "kernel": kname,
                         "bytes_per_launch": tot_bytes,
                         "csr_bytes_per_launch": csr_bytes, "csr_equiv_gbps": csr_equiv,
                         "avg_launch_ms": spmv_avg_max, "launches": spmv_cnt,
                         # this box's measured read-only streaming ceiling (per GPU;
                         # 16-B nontemporal loads, 4 in flight per lane): what HBM
                         # delivers here, against the 8 TB/s peak
                         "achievable_gbps": stream_rd,
                         "frac_of_achievable": achieved / (stream_rd * nranks) if achieved else None,
                         "read_ceiling_gbps": stream_rd,
                         "traffic_frac_of_read_ceiling": (traffic / (spmv_avg_max * 1e-3) / 1e9 / stream_rd
                                                          if traffic and spmv_avg_max > 0 and nranks == 1
                                                          else None)},
            "cpu_baseline": cpu,
            "spmv_gbps": achieved,
            "stream_copy_gbps": stream,
            "stream_read_gbps": stream_rd,  # read-only streaming ceiling (the SpMV is read-dominated)
            "breakdown_ms_per_iter": brk,
            "symmetric_bricks": K.getSymmetricBricks() if K.isSymmetricStorage() else None,
            "assembly_s": t_asm,
            "mesh_generation_s": t_mesh,
            "setup_s": t_setup,
            "solve": solve,
            "spmv_plain": spmv_plain,
            "aij_spmv": aij,
            "operators": ops,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def spmv_kernel(K, layout, ngl):
    """Name of the SpMV kernel(s) libkle launches for this rank's K with the
    current tuning (kle_mat_spmv_kernel: the library's own launch decision)."""
    return K.spmvKernel()


def lookup_traffic(path, key, kernel, alg_bytes):
    """HBM bytes per SpMV launch from the rocprofv3 PMC record `key` of
    profiles/traffic.json (tools/pmc_traffic.py), or None.  A record counts only
    if it was measured on this kernel: same launch names and the same
    algorithmic bytes per launch as the kernel running now (a kernel change
    that moves different bytes makes the old counter stale)."""
    try:
        rec = json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None, "no traffic file"
    if rec is None:
        return None, f"no PMC record {key}"
    alg = rec.get("algorithmic_bytes_per_launch")
    if alg is None or rec.get("kernel") != kernel:
        return None, f"stale: record {key} names no algorithmic bytes or another kernel ({rec.get('kernel')})"
    if abs(alg - alg_bytes) > 1e-9 * alg_bytes:
        return None, f"stale: record {key} measured a kernel of {alg:.0f} algorithmic bytes, this one moves {alg_bytes:.0f}"
    return rec["hbm_bytes_per_launch"], f"measured ({rec.get('source', key)})"


def splitmix_uniform(seed, lo, hi):
    """x[i] = uniform[-1, 1) from the splitmix64 stream of `seed` at global
    index i (same on every rank and on the CPU)."""
    import numpy as np
    i = np.arange(lo, hi, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(K, b, seconds, nthreads=0):
    """Oracle CSR CG (OpenMP) on the same matrix: bounded sample of ~`seconds`
    on the OpenMP thread count (nthreads: 0 the runtime default, -1 the
    affinity mask, else that many), ~seconds/3 on one thread, plus the host
    STREAM triad at both thread counts."""
    import numpy as np

    from oracle import oracle as O
    if nthreads < 0:
        nthreads = len(os.sched_getaffinity(0))
    if nthreads > 0:
        O.set_threads(nthreads)
    ip, ix, d = K.getValuesCSR()
    A = O.CSR.from_arrays(ip, ix, d, int(ip.shape[0] - 1))
    del ip, ix, d
    bb = b.getArray()
    threads = O.num_threads()

    def sample(secs, chunk):
        A.cg(bb, fixed_iters=True, maxit=min(chunk, 3))  # first touch of the host pages
        its, el = 0, 0.0
        while el < secs:  # bounded sample: chunks of iterations until ~secs
            A.cg(bb, fixed_iters=True, maxit=chunk)
            el += A.last_loop_seconds()  # the iteration loop only (no per-call setup)
            its += chunk
        return its, el

    its, el = sample(seconds, 10)
    triad = O.stream_triad_gbps()
    O.set_threads(1)
    its1, el1 = sample(seconds / 3, 2)
    triad1 = O.stream_triad_gbps()
    O.set_threads(threads)
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    reason = None
    if affinity is not None and threads < affinity:
        omp = os.environ.get("OMP_NUM_THREADS")
        reason = (f"OMP_NUM_THREADS={omp} in the environment: the GPU box's CPU share for one GPU "
                  f"(the affinity mask lists all {affinity} host threads, shared with the other GPUs' jobs)"
                  if omp else f"OpenMP runtime default of {threads} threads")
    return {"value": its / el, "unit": "CG iters/s", "cores": threads, "cores_reason": reason, "kind": "port",
            "sample": f"{its} fixed CG+Jacobi iterations of oracle/kle_oracle.c (CSR, OpenMP) on the same "
                      f"assembled K ({A.nnz} nnz), {el:.1f} s; 1 thread: {its1} iterations, {el1:.1f} s",
            "model": _cpu_model(), "nproc": os.cpu_count(),
            "affinity": affinity, "value_1core": its1 / el1, "stream_triad_gbps": triad, "stream_triad_gbps_1core": triad1,
            "spmv_gbps_equiv": 12.0 * A.nnz * its / el / 1e9}


if __name__ == "__main__":
    main()
