"""World-size-2 (and 3) CPU rehearsal of the multi-GPU path with gloo.

Each rank takes libkle's slab partition of the mesh (owned rows, ghosted
ext range, halo plan: who sends how many nodes to whom), builds its local
block of the oracle's assembled K with columns in the ext-local numbering,
and runs the same distributed Jacobi-CG as the device code: halo exchange of
p before every SpMV, allreduce of the dot products.  The result must equal
the single-rank oracle CG (same iteration count, solution to 1e-12).  This
checks the decomposition (ranges, ghost widths, send/recv plan) that the
RCCL path in libkle uses, without a GPU.
"""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, nelem, ngl, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=size)
    from oracle import oracle as O
    import pynama_amd as pa
    dim = len(nelem)
    faces = pa.mesh.FACES[dim]
    m = pa.BoxMesh(dim, nelem, [0] * dim, [1] * dim, ngl, rank, size)
    m.set_dirichlet_faces(faces)
    # global system from the oracle (the same numbering)
    om = O.BoxMesh(dim, nelem, [0] * dim, [1] * dim, ngl)
    flag = np.zeros(om.N, np.uint8)
    serial = pa.BoxMesh(dim, nelem, [0] * dim, [1] * dim, ngl)
    flag[serial.face_nodes(faces)] = 1
    K, Kr, Rw = om.assemble_fs(flag)
    rng = np.random.default_rng(123)
    b_glob = rng.uniform(-1, 1, K.m)
    bs = dim
    lo, hi = m.node_range
    elo, ehi = m.ext_range
    rows = np.arange(lo * bs, hi * bs)
    # local CSR with ext-local columns
    ip = [0]
    cols, vals = [], []
    for r in rows:
        c = K.indices[K.indptr[r]:K.indptr[r + 1]]
        assert c.min() >= elo * bs and c.max() < ehi * bs, "column outside the ghosted range"
        cols.extend((c - elo * bs).tolist())
        vals.extend(K.data[K.indptr[r]:K.indptr[r + 1]].tolist())
        ip.append(len(cols))
    ip, cols, vals = np.array(ip), np.array(cols), np.array(vals)
    diag = np.array([vals[ip[i]:ip[i + 1]][cols[ip[i]:ip[i + 1]] == (rows[i] - elo * bs)][0]
                     for i in range(len(rows))])
    h = m.halo()
    nown = len(rows)
    glo = (lo - elo) * bs
    ghi = (ehi - hi) * bs

    def halo(pext):
        own = pext[glo:glo + nown]
        reqs = []
        if h["lo_rank"] >= 0:
            reqs.append(dist.isend(torch.from_numpy(own[:h["send_lo_nodes"] * bs].copy()), h["lo_rank"]))
            buf_lo = torch.zeros(glo, dtype=torch.float64)
            reqs.append(dist.irecv(buf_lo, h["lo_rank"]))
        if h["hi_rank"] >= 0:
            reqs.append(dist.isend(torch.from_numpy(own[nown - h["send_hi_nodes"] * bs:].copy()), h["hi_rank"]))
            buf_hi = torch.zeros(ghi, dtype=torch.float64)
            reqs.append(dist.irecv(buf_hi, h["hi_rank"]))
        for rq in reqs:
            rq.wait()
        if h["lo_rank"] >= 0:
            pext[:glo] = buf_lo.numpy()
        if h["hi_rank"] >= 0:
            pext[glo + nown:] = buf_hi.numpy()

    def spmv(pext):
        halo(pext)
        y = np.zeros(nown)
        for i in range(nown):
            y[i] = vals[ip[i]:ip[i + 1]] @ pext[cols[ip[i]:ip[i + 1]]]
        return y

    def allsum(*v):
        t = torch.tensor(v, dtype=torch.float64)
        dist.all_reduce(t)
        return t.numpy()

    b = b_glob[rows]
    x = np.zeros(nown)
    r = b.copy()
    z = r / diag
    rz, rr = allsum(r @ z, r @ r)
    tol = 1e-10 * np.sqrt(rr)
    pext = np.zeros(glo + nown + ghi)
    it = 0
    while np.sqrt(rr) > tol and it < 5000:
        p_own = z + (0.0 if it == 0 else rz / rz_old) * pext[glo:glo + nown]
        pext[glo:glo + nown] = p_own
        w = spmv(pext)
        (pw,) = allsum(p_own @ w)
        a = rz / pw
        x += a * p_own
        r -= a * w
        z = r / diag
        rz_old = rz
        rz, rr = allsum(r @ z, r @ r)
        it += 1
    xs, its, _ = K.cg(b_glob, rtol=1e-10, jacobi=True)
    err = np.linalg.norm(x - xs[rows]) / max(np.linalg.norm(xs[rows]), 1e-300)
    q.put((rank, it, its, err))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("size,nelem,ngl", [(2, [3, 2, 4], 3), (3, [2, 3, 3], 4), (2, [4, 4], 5)])
def test_distributed_cg_matches_serial(size, nelem, ngl):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, nelem, ngl, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(size)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, it, its, err in res:
        assert abs(it - its) <= 1, (rank, it, its)
        assert err < 1e-9, (rank, err)


def _worker_graph(rank, size, port, nel, ngl, q):
    """Same rehearsal on an unstructured mesh cut by inertial bisection: any
    number of neighbours, ghosts grouped by owner, sends through index lists
    (kle_mesh_get_peers) -- the plan libkle's general halo exchange uses."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=size)
    from oracle import oracle as O
    from pynama_amd.mesh import UnstructuredMesh
    from pynama_amd.meshgen import perturbed_box
    V, Cc, F, T = perturbed_box(3, nel, seed=5)
    m = UnstructuredMesh(3, ngl, V, Cc, F, T, rank=rank, nranks=size, partitioner="inertial")
    um = O.UMesh(3, ngl, V, Cc, F, T)
    flag = ((um.tags_ & 0x3f) != 0).astype(np.uint8)
    K, Kr, Rw = um.assemble_fs(flag)
    allc = [None] * size
    dist.all_gather_object(allc, m.coords())
    to_orc = O.node_map(np.concatenate(allc), um.coords())  # our global id -> oracle id
    from_orc = np.argsort(to_orc)
    bs = 3
    lo, hi = m.node_range
    g = m.ext_gids()
    nown, glo = (hi - lo) * bs, (lo - m.ext_range[0]) * bs
    ip, cols, vals = [0], [], []
    for node in range(lo, hi):
        for a in range(bs):
            row = to_orc[node] * bs + a
            c = K.indices[K.indptr[row]:K.indptr[row + 1]]
            gn = from_orc[c // bs]
            pos = np.searchsorted(g, gn)
            assert (g[np.minimum(pos, len(g) - 1)] == gn).all(), "column outside the ext range"
            cols.extend((pos * bs + c % bs).tolist())
            vals.extend(K.data[K.indptr[row]:K.indptr[row + 1]].tolist())
            ip.append(len(cols))
    ip, cols, vals = np.array(ip), np.array(cols), np.array(vals)
    rows_orc = (to_orc[lo:hi, None] * bs + np.arange(bs)).ravel()
    diag = np.array([vals[ip[i]:ip[i + 1]][cols[ip[i]:ip[i + 1]] == glo + i][0] for i in range(nown)])
    peers = m.peers()
    owner = np.concatenate([[r] * len(c) for r, c in enumerate(allc)])

    def halo(pext):
        own = pext[glo:glo + nown].reshape(-1, bs)
        reqs, bufs = [], []
        for qr, (nrecv, sent) in sorted(peers.items()):
            reqs.append(dist.isend(torch.from_numpy(own[sent].ravel().copy()), qr))
            t = torch.zeros(nrecv * bs, dtype=torch.float64)
            reqs.append(dist.irecv(t, qr))
            first = int(np.nonzero(owner[g] == qr)[0][0])  # the peer's ghost group
            bufs.append((first * bs, t))
        for rq in reqs:
            rq.wait()
        for o, t in bufs:
            pext[o:o + len(t)] = t.numpy()

    def allsum(*v):
        t = torch.tensor(v, dtype=torch.float64)
        dist.all_reduce(t)
        return t.numpy()

    # The graph symmetric storage's N > 1 product (kle_sym.hip gsym_spmv),
    # restated: each rank keeps the blocks of its node rows from the diagonal
    # on in ext order (owned columns from the row's own, every higher rank's
    # ghost), adds B x_j to row i and B^T x_i to row j, then returns the upper
    # ghosts' sums to their owners (halo_reverse_plan: the forward plan
    # transposed) and adds what the lower peers send, in ascending rank order.
    xg = np.random.default_rng(11).uniform(-1, 1, K.m)
    pext = np.zeros(len(g) * bs)
    pext[glo:glo + nown] = xg[rows_orc]
    halo(pext)
    yext = np.zeros(len(g) * bs)
    n0 = glo // bs
    for i in range(nown // bs):
        pi = n0 + i
        blocks = {}  # node column -> 3x3 block (Dirichlet rows hold their diagonal only)
        for a in range(bs):
            for cc, v in zip(cols[ip[i * bs + a]:ip[i * bs + a + 1]], vals[ip[i * bs + a]:ip[i * bs + a + 1]]):
                blocks.setdefault(cc // bs, np.zeros((bs, bs)))[a, cc % bs] = v
        for pj, B in sorted(blocks.items()):
            if pj < pi:
                continue  # lower triangle: stored by the row pj's owner (here or a lower rank)
            yext[pi * bs:pi * bs + bs] += B @ pext[pj * bs:pj * bs + bs]
            if pj != pi:
                yext[pj * bs:pj * bs + bs] += B.T @ pext[pi * bs:pi * bs + bs]
    y = yext[glo:glo + nown].reshape(-1, bs)
    reqs, bufs = [], []
    for qr, (nrecv, sent) in sorted(peers.items()):
        if qr > rank:  # my ghosts of a higher rank: their sums go back to it
            first = int(np.nonzero(owner[g] == qr)[0][0])
            reqs.append(dist.isend(torch.from_numpy(yext[first * bs:(first + nrecv) * bs].copy()), qr))
        elif qr < rank:  # the sums a lower rank formed for the nodes it ghosts of mine
            t = torch.zeros(len(sent) * bs, dtype=torch.float64)
            reqs.append(dist.irecv(t, qr))
            bufs.append((sent, t))
    for rq in reqs:
        rq.wait()
    for sent, t in bufs:  # ascending sender rank
        y[sent] += t.numpy().reshape(-1, bs)
    y_ref = K.mult(xg)[rows_orc]
    sym_err = float(np.abs(y.ravel() - y_ref).max() / np.abs(y_ref).max())

    rng = np.random.default_rng(7)
    b_glob = rng.uniform(-1, 1, K.m)
    b = b_glob[rows_orc]
    x, r = np.zeros(nown), b.copy()
    z = r / diag
    rz, rr = allsum(r @ z, r @ r)
    tol = 1e-10 * np.sqrt(rr)
    pext = np.zeros(len(g) * bs)
    it = 0
    while np.sqrt(rr) > tol and it < 5000:
        pext[glo:glo + nown] = z + (0.0 if it == 0 else rz / rz_old) * pext[glo:glo + nown]
        halo(pext)
        w = np.array([vals[ip[i]:ip[i + 1]] @ pext[cols[ip[i]:ip[i + 1]]] for i in range(nown)])
        (pw,) = allsum(pext[glo:glo + nown] @ w)
        a = rz / pw
        x += a * pext[glo:glo + nown]
        r -= a * w
        z = r / diag
        rz_old = rz
        rz, rr = allsum(r @ z, r @ r)
        it += 1
    xs, its, _ = K.cg(b_glob, rtol=1e-10, jacobi=True)
    err = np.linalg.norm(x - xs[rows_orc]) / max(np.linalg.norm(xs[rows_orc]), 1e-300)
    q.put((rank, it, its, err, len(peers), sym_err))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("size,nel", [(2, [3, 3, 4]), (4, [4, 4, 3])])
def test_graph_partition_cg_matches_serial(size, nel):
    """Distributed Jacobi-CG on the graph plan == serial oracle; and the graph
    symmetric storage's product with its reverse halo == K x on every rank."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_graph, args=(r, size, port, nel, 3, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(size)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, it, its, err, npeers, sym_err in res:
        assert abs(it - its) <= 1, (rank, it, its)
        assert err < 1e-9, (rank, err)
        assert sym_err < 1e-13, (rank, sym_err)  # upper-triangle product + reverse halo == K x
    if size == 4:
        assert max(r[4] for r in res) >= 3  # more than a slab chain's two neighbours
