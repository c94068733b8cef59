"""ctypes front end of the CPU oracle (oracle/kle_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  The product never imports it.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_gauss.argtypes = [C.c_int, f64p, f64p]
        L.orc_lobatto.argtypes = [C.c_int, f64p, f64p]
        L.orc_spectral_order.argtypes = [C.c_int, C.c_int, i32p]
        L.orc_elem_create.restype = C.c_void_p
        L.orc_elem_create.argtypes = [C.c_int, C.c_int]
        L.orc_elem_destroy.argtypes = [C.c_void_p]
        L.orc_elem_table.argtypes = [C.c_void_p, C.c_int, C.c_int, f64p]
        L.orc_elem_npoints.argtypes = [C.c_void_p, C.c_int]
        L.orc_elem_kle.argtypes = [C.c_void_p, f64p, f64p, f64p, f64p]
        L.orc_elem_ops.argtypes = [C.c_void_p, f64p, f64p, f64p, f64p, f64p]
        L.orc_mesh_box.restype = C.c_void_p
        L.orc_mesh_box.argtypes = [C.c_int, i64p, f64p, f64p, C.c_int]
        L.orc_mesh_destroy.argtypes = [C.c_void_p]
        L.orc_mesh_from_arrays.restype = C.c_void_p
        L.orc_mesh_from_arrays.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int64, i64p, f64p]
        L.orc_mesh_nnodes.restype = C.c_int64
        L.orc_mesh_nnodes.argtypes = [C.c_void_p]
        L.orc_mesh_nelems.restype = C.c_int64
        L.orc_mesh_nelems.argtypes = [C.c_void_p]
        L.orc_mesh_conn.argtypes = [C.c_void_p, i64p]
        L.orc_mesh_corners.argtypes = [C.c_void_p, f64p]
        L.orc_mesh_coords.argtypes = [C.c_void_p, f64p]
        L.orc_assemble_fs.argtypes = [C.c_void_p, u8p, C.POINTER(C.c_void_p),
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.orc_assemble_ops.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 3 + [f64p]
        L.orc_csr_destroy.argtypes = [C.c_void_p]
        L.orc_csr_nnz.restype = C.c_int64
        L.orc_csr_nnz.argtypes = [C.c_void_p]
        L.orc_csr_rows.restype = C.c_int64
        L.orc_csr_rows.argtypes = [C.c_void_p]
        L.orc_csr_export.argtypes = [C.c_void_p, i64p, i64p, f64p]
        L.orc_csr_from.restype = C.c_void_p
        L.orc_csr_from.argtypes = [C.c_int64, C.c_int64, i64p, i64p, f64p]
        L.orc_spmv.argtypes = [C.c_void_p, f64p, f64p]
        L.orc_cg.restype = C.c_int
        L.orc_cg.argtypes = [C.c_void_p, f64p, f64p, C.c_double, C.c_double, C.c_int,
                             C.c_int, C.c_int, C.POINTER(C.c_double)]
        L.orc_num_threads.restype = C.c_int
        L.orc_set_num_threads.argtypes = [C.c_int]
        L.orc_cg_loop_seconds.restype = C.c_double
        L.orc_cg_loop_seconds.argtypes = []
        L.orc_stream_triad.restype = C.c_double
        L.orc_stream_triad.argtypes = [C.c_int64, C.c_int]
        _LIB = L
    return _LIB


def gauss(n):
    x, w = np.zeros(n), np.zeros(n)
    lib().orc_gauss(n, x, w)
    return x, w


def lobatto(n):
    x, w = np.zeros(n), np.zeros(n)
    lib().orc_lobatto(n, x, w)
    return x, w


def spectral_order(dim, n):
    out = np.zeros(n ** dim, dtype=np.int32)
    lib().orc_spectral_order(dim, n, out)
    return out


SETS = {"full": 0, "red": 1, "op": 2, "coo": 3, "cooRed": 4, "cooOp": 5}


class Element:
    """Restated Spectral(ngl, dim) (spectral.py:17-90)."""

    def __init__(self, ngl, dim):
        self.ngl, self.dim = ngl, dim
        self.nn = ngl ** dim
        self.dim_w = 1 if dim == 2 else 3
        self.dim_s = 3 if dim == 2 else 6
        self._h = lib().orc_elem_create(dim, ngl)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_elem_destroy(self._h)

    def table(self, which, what):
        s = SETS[which]
        nq = lib().orc_elem_npoints(self._h, s)
        nn = 2 ** self.dim if which.startswith("coo") else self.nn
        shape = {0: (nq, nn), 1: (nq, self.dim, nn), 2: (nq,), 3: (nq, self.dim)}[what]
        out = np.zeros(int(np.prod(shape)))
        lib().orc_elem_table(self._h, s, what, out)
        return out.reshape(shape)

    def kle(self, X):
        nd = self.dim * self.nn
        K = np.zeros((nd, nd))
        Rw = np.zeros((nd, self.dim_w * self.nn))
        Rd = np.zeros((nd, self.nn))
        lib().orc_elem_kle(self._h, np.ascontiguousarray(X, dtype=float), K, Rw, Rd)
        return K, Rw, Rd

    def ops(self, X):
        nd, nn = self.dim * self.nn, self.nn
        SrT = np.zeros((self.dim_s * nn, nd))
        Div = np.zeros((nd, self.dim_s * nn))
        Curl = np.zeros((self.dim_w * nn, nd))
        W = np.zeros(nn)
        lib().orc_elem_ops(self._h, np.ascontiguousarray(X, dtype=float), SrT, Div, Curl, W)
        return SrT, Div, Curl, W


class CSR:
    def __init__(self, handle, ncols=None):
        self._h = handle
        L = lib()
        self.m = L.orc_csr_rows(handle)
        self.nnz = L.orc_csr_nnz(handle)
        self.indptr = np.zeros(self.m + 1, dtype=np.int64)
        self.indices = np.zeros(max(self.nnz, 1), dtype=np.int64)
        self.data = np.zeros(max(self.nnz, 1))
        L.orc_csr_export(handle, self.indptr, self.indices, self.data)
        self.indices = self.indices[: self.nnz]
        self.data = self.data[: self.nnz]
        self.n = ncols

    @classmethod
    def from_arrays(cls, indptr, indices, data, ncols):
        h = lib().orc_csr_from(len(indptr) - 1, ncols, np.ascontiguousarray(indptr, np.int64),
                               np.ascontiguousarray(indices, np.int64),
                               np.ascontiguousarray(data, np.float64))
        return cls(h, ncols)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_csr_destroy(self._h)

    def mult(self, x):
        y = np.zeros(self.m)
        lib().orc_spmv(self._h, np.ascontiguousarray(x, np.float64), y)
        return y

    def cg(self, b, rtol=1e-10, atol=0.0, maxit=100000, jacobi=True, fixed_iters=False):
        x = np.zeros(self.m)
        rr = C.c_double(0)
        it = lib().orc_cg(self._h, np.ascontiguousarray(b, np.float64), x, rtol, atol, maxit,
                          int(jacobi), int(fixed_iters), C.byref(rr))
        return x, it, rr.value

    @staticmethod
    def last_loop_seconds():
        """Wall time of the last cg()'s iteration loop (no setup, no exit residual)."""
        return lib().orc_cg_loop_seconds()

    def dense(self):
        d = np.zeros((self.m, self.n))
        for r in range(self.m):
            d[r, self.indices[self.indptr[r]:self.indptr[r + 1]]] = \
                self.data[self.indptr[r]:self.indptr[r + 1]]
        return d


class BoxMesh:
    """Structured box mesh in the canonical numbering (see kle_oracle.c)."""

    def __init__(self, dim, nelem, lower, upper, ngl):
        self.dim, self.ngl = dim, ngl
        self.nelem = [int(v) for v in nelem]
        self.nn = ngl ** dim
        self._h = lib().orc_mesh_box(dim, np.array(list(nelem) + [1] * (3 - dim), np.int64),
                                     np.array(list(lower) + [0.0] * (3 - dim), float),
                                     np.array(list(upper) + [1.0] * (3 - dim), float), ngl)
        self.N = lib().orc_mesh_nnodes(self._h)
        self.E = lib().orc_mesh_nelems(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_mesh_destroy(self._h)

    def conn(self):
        out = np.zeros(self.E * self.nn, dtype=np.int64)
        lib().orc_mesh_conn(self._h, out)
        return out.reshape(self.E, self.nn)

    def corners(self):
        out = np.zeros(self.E * 2 ** self.dim * self.dim)
        lib().orc_mesh_corners(self._h, out)
        return out.reshape(self.E, 2 ** self.dim, self.dim)

    def coords(self):
        out = np.zeros(self.N * self.dim)
        lib().orc_mesh_coords(self._h, out)
        return out.reshape(self.N, self.dim)

    def assemble_fs(self, dir_flag):
        K, Kr, Rw = C.c_void_p(), C.c_void_p(), C.c_void_p()
        lib().orc_assemble_fs(self._h, np.ascontiguousarray(dir_flag, np.uint8),
                              C.byref(K), C.byref(Kr), C.byref(Rw))
        dw = 1 if self.dim == 2 else 3
        return (CSR(K.value, self.N * self.dim), CSR(Kr.value, self.N * self.dim),
                CSR(Rw.value, self.N * dw))


    def assemble_ops(self):
        """Operators Curl, SrT, DivSrT (weights applied) and the lumped nodal weights W."""
        Cu, S, D = C.c_void_p(), C.c_void_p(), C.c_void_p()
        W = np.zeros(self.N)
        lib().orc_assemble_ops(self._h, C.byref(Cu), C.byref(S), C.byref(D), W)
        dw, ds = (1, 3) if self.dim == 2 else (3, 6)
        return (CSR(Cu.value, self.N * self.dim), CSR(S.value, self.N * self.dim),
                CSR(D.value, self.N * ds), W)


# ------------------------------------------------------------ unstructured
def read_gmsh(path):
    """Gmsh MSH 4.1 ASCII -> (dim, vertices [nv,3], cells [nc, 2^dim] (Gmsh
    order, file order), facets [nf, 2^(dim-1)], facet physical tags [nf]).
    Restates what DMPlexCreateGmsh keeps of the file for GmshDom
    (dmplex.py:390-395): quads/hexes as cells, boundary lines/quads with their
    entity's first physical tag as the "Face Sets" value."""
    with open(path) as f:
        tok = f.read().split()
    i = 0
    phys = {}
    verts, index = [], {}
    blocks = []

    def take(n=1):
        nonlocal i
        out = tok[i:i + n]
        i += n
        return out if n > 1 else out[0]

    while i < len(tok):
        t = take()
        if t == "$Entities":
            cnt = [int(x) for x in take(4)]
            for d in range(4):
                for _ in range(cnt[d]):
                    tag = int(take())
                    take(3 if d == 0 else 6)
                    nph = int(take())
                    ph = [int(take()) for _ in range(nph)]
                    if ph:
                        phys[(d, tag)] = abs(ph[0])
                    if d > 0:
                        nb = int(take())
                        take(nb) if nb > 1 else (take() if nb == 1 else None)
        elif t == "$Nodes":
            nblk = int(take())
            take(3)
            for _ in range(nblk):
                edim, _etag, para, n = (int(x) for x in take(4))
                tags = [int(take()) for _ in range(n)]
                for tg in tags:
                    xyz = [float(take()) for _ in range(3)]
                    if para:
                        take(edim) if edim > 1 else take()
                    index[tg] = len(verts)
                    verts.append(xyz)
        elif t == "$Elements":
            nblk = int(take())
            take(3)
            for _ in range(nblk):
                edim, etag, etype, n = (int(x) for x in take(4))
                nv = {1: 2, 3: 4, 5: 8, 15: 1}[etype]
                rows = []
                for _ in range(n):
                    take()
                    rows.append([index[int(take())] for _ in range(nv)])
                blocks.append((edim, etag, etype, rows))
    dim = 3 if any(b[2] == 5 for b in blocks) else 2
    ctype, ftype = (5, 3) if dim == 3 else (3, 1)
    cells = [r for b in blocks if b[2] == ctype for r in b[3]]
    facets, ftags = [], []
    for edim, etag, etype, rows in blocks:
        if etype == ftype and edim == dim - 1:
            for r in rows:
                facets.append(r)
                ftags.append(phys.get((edim, etag), 0))
    return (dim, np.array(verts, float), np.array(cells, np.int64),
            np.array(facets, np.int64).reshape(-1, 2 ** (dim - 1)), np.array(ftags, np.int64))


# tensor corner t = x + 2y (+4z) -> Gmsh slot; DMPlex closure slot -> tensor corner
_T2G = {2: [0, 1, 3, 2], 3: [0, 1, 3, 2, 4, 5, 7, 6]}
_C2T = {2: [0, 1, 3, 2], 3: [0, 2, 3, 1, 4, 5, 7, 6]}


class UMesh(BoxMesh):
    """Unstructured quad/hex mesh for the oracle.  Node numbering is by
    coordinates: every cell's GLL nodes are placed by its multilinear map
    (computeFullCoordinates, dmplex.py:62-91) and points closer than `tol`
    are the same node (ids in order of first appearance) -- independent of
    the product's topological numbering (kle_umesh.cpp).  Cell frame: Gmsh
    vertex order, corners handed to the element in DMPlex closure order."""

    def __init__(self, dim, ngl, verts, cells, facets=None, ftags=None, tol=1e-9):
        from scipy.spatial import cKDTree
        self.dim, self.ngl = dim, ngl
        self.nn = ngl ** dim
        nc = 2 ** dim
        xi = (1.0 + lobatto(ngl)[0]) / 2.0
        tv = np.asarray(cells)[:, _T2G[dim]]
        X = np.asarray(verts, float)[:, :dim]
        self.E = len(cells)
        q = np.stack(np.meshgrid(*[np.arange(ngl)] * dim, indexing="ij")[::-1], -1).reshape(-1, dim)
        # shape functions of tensor corner t at local node l
        Nw = np.ones((self.nn, nc))
        for t in range(nc):
            for k in range(dim):
                Nw[:, t] *= xi[q[:, k]] if (t >> k) & 1 else 1.0 - xi[q[:, k]]
        pts = np.einsum("lt,etd->eld", Nw, X[tv]).reshape(-1, dim)
        scale = max(1.0, np.abs(pts).max())
        pairs = cKDTree(pts).query_pairs(tol * scale, output_type="ndarray")
        parent = np.arange(len(pts))

        def root(a):
            while parent[a] != a:
                parent[a] = parent[parent[a]]
                a = parent[a]
            return a

        for a, b in pairs:
            ra, rb = root(a), root(b)
            if ra != rb:
                parent[max(ra, rb)] = min(ra, rb)
        roots = np.array([root(a) for a in range(len(pts))])
        uniq, first = np.unique(roots, return_index=True)
        order = np.argsort(first)
        newid = np.empty(len(uniq), np.int64)
        newid[order] = np.arange(len(uniq))
        self.conn_ = newid[np.searchsorted(uniq, roots)].reshape(self.E, self.nn)
        self.N = len(uniq)
        self.coords_ = np.zeros((self.N, dim))
        self.coords_[self.conn_.ravel()] = pts  # last cell wins
        self.corners_ = np.ascontiguousarray(X[tv[:, _C2T[dim]]])
        # the element routines (restated Spectral) order local nodes as the
        # reference does (HCooOp of the closure-order corners): tensor index
        # of reference node q, for the C assembly
        unit = np.array([[(t >> k) & 1 for k in range(dim)] for t in _C2T[dim]], float)
        Hc = Element(ngl, dim).table("cooOp", 0)
        pos = Hc @ unit
        ti = np.array([[int(np.argmin(np.abs(xi - c))) for c in row] for row in pos])
        ref_to_tensor = sum(ti[:, k] * ngl ** k for k in range(dim))
        self.conn_ref_ = np.ascontiguousarray(self.conn_[:, ref_to_tensor])
        self.tags_ = np.zeros(self.N, np.int64)
        if facets is not None and len(facets):
            fmap = {}
            for f, t in zip(np.asarray(facets), np.asarray(ftags)):
                if 1 <= t <= 32:
                    k = tuple(sorted(f.tolist()))
                    fmap[k] = fmap.get(k, 0) | (1 << (int(t) - 1))
            for e in range(self.E):
                for d in range(dim):
                    for side in (0, 1):
                        k = tuple(sorted(tv[e, t] for t in range(nc) if ((t >> d) & 1) == side))
                        if k in fmap:
                            on = q[:, d] == (ngl - 1 if side else 0)
                            self.tags_[self.conn_[e, on]] |= fmap[k]
        self._h = lib().orc_mesh_from_arrays(dim, ngl, self.N, self.E,
                                             np.ascontiguousarray(self.conn_ref_.ravel()),
                                             np.ascontiguousarray(self.corners_.ravel()))

    @classmethod
    def from_gmsh(cls, path, ngl):
        dim, v, c, f, t = read_gmsh(path)
        return cls(dim, ngl, v, c, f, t)

    def conn(self):
        return self.conn_

    def corners(self):
        return self.corners_

    def coords(self):
        return self.coords_

    def face_nodes(self, mask):
        return np.nonzero(self.tags_ & mask)[0]


def node_map(coords_a, coords_b, tol=1e-9):
    """Index map m with coords_b[m[i]] == coords_a[i] (bijection checked)."""
    from scipy.spatial import cKDTree
    d, m = cKDTree(coords_b).query(coords_a)
    assert len(coords_a) == len(coords_b)
    assert d.max() <= tol * max(1.0, np.abs(coords_b).max()), d.max()
    assert len(np.unique(m)) == len(m)
    return m


def vtensv(vel, dim):
    """BaseProblem.computeVtensV (base_problem.py:138-154)."""
    v = np.asarray(vel).reshape(-1, dim)
    x, y = v[:, 0], v[:, 1]
    if dim == 2:
        return np.stack([x ** 2, x * y, y ** 2], 1).ravel()
    z = v[:, 2]
    return np.stack([x ** 2, x * y, y ** 2, y * z, z ** 2, z * x], 1).ravel()


def eval_rhs_chain(Curl, SrT, DivSrT, vel, rho, mu, dim):
    """The operator part of BaseProblem.evalRHS (base_problem.py:127-136) after
    the KLE solve: returns (VtensV, Aux1, f)."""
    vt = vtensv(vel, dim)
    aux = SrT.mult(vel)
    aux *= (2.0 * mu)
    aux += (-1.0 * rho) * vt
    rhs = DivSrT.mult(aux)
    rhs *= (1 / rho)
    return vt, aux, Curl.mult(rhs)


def set_threads(n):
    lib().orc_set_num_threads(int(n))


def num_threads():
    return lib().orc_num_threads()


def stream_triad_gbps(n=1 << 26, reps=10):
    """Host STREAM triad (GB/s, best of `reps`) on the current thread count."""
    return lib().orc_stream_triad(int(n), int(reps))


# ------------------------------------------------------------------ no-slip
FACE_AXIS = {"left": (0, 0), "right": (0, 1), "down": (1, 0), "up": (1, 1), "back": (2, 0), "front": (2, 1)}


def noslip_dofs(mesh, walls):
    """Tangential / normal DoF sets of the no-slip walls, in configuration order:
    Boundary.getTangDofs / getNormalDofs (boundary.py:98-115) collected by
    BoundaryConditions.getNoSlipTangDofs / getNoSlipNormalDofs(allGather=True)
    (boundary_conditions.py:205-238, incl. its left/right corner rule)."""
    dim = mesh.dim
    L = [int(n) * (mesh.ngl - 1) + 1 for n in mesh.nelem]
    lat = np.stack(np.meshgrid(*[np.arange(n) for n in L[::-1]], indexing="ij")[::-1], -1).reshape(-1, dim)
    tang, normal, remove = set(), set(), set()
    for name in walls:
        ax, side = FACE_AXIS[name]
        nodes = np.nonzero(lat[:, ax] == (0 if side == 0 else L[ax] - 1))[0]
        loc = set((nodes * dim + ax).tolist())
        if name in ("left", "right"):
            remove |= {i for i in loc if i + 1 in normal}
        normal |= loc
        for t in range(dim):
            if t != ax:
                tang |= set((nodes * dim + t).tolist())
    return tang, normal - remove


def _dok_csr(dok, m, n):
    rows = sorted(dok)
    ip = np.zeros(m + 1, np.int64)
    ix, dv = [], []
    for r in range(m):
        cols = sorted(dok.get(r, {}))
        ip[r + 1] = ip[r] + len(cols)
        ix += cols
        dv += [dok[r][c] for c in cols]
    del rows
    return CSR.from_arrays(ip, np.array(ix, np.int64), np.array(dv, float), n)


def assemble_ns(mesh, tang, normal):
    """MatNS.buildNS (mat_ns.py:47-145) restated on dict-of-keys matrices with
    PETSc ADD/INSERT semantics, cells ascending (single rank).  Small meshes
    only.  Returns dict of CSR: K, Krhs, Rw, Rd, Kfs, Krhsfs, Rwfs, Rdfs."""
    dim, nn = mesh.dim, mesh.nn
    dw = 1 if dim == 2 else 3
    el = Element(mesh.ngl, dim)
    conn, X = mesh.conn(), mesh.corners()
    mats = {k: {} for k in ("K", "Krhs", "Rw", "Rd", "Kfs", "Krhsfs", "Rwfs", "Rdfs")}

    def add(name, rows, cols, vals, addv=True):
        d = mats[name]
        for i, r in enumerate(rows):
            row = d.setdefault(r, {})
            for j, c in enumerate(cols):
                v = vals[i][j] if np.ndim(vals) else vals
                row[c] = (row.get(c, 0.0) + v) if addv else v

    ind1, ind1fs = set(), set()
    for e in range(mesh.E):
        Ke, Rwe, Rde = el.kle(X[e].ravel())
        nodes = conn[e].tolist()
        iv = [n * dim + d for n in nodes for d in range(dim)]
        iw = [n * dw + d for n in nodes for d in range(dw)]
        ivs = set(iv)
        nd_ = normal & ivs
        td = (tang & ivs) - nd_
        gfree = list(ivs - nd_ - td)
        dfree = [iv.index(i) for i in gfree]
        lnorm = [iv.index(i) for i in nd_]
        ltang = [iv.index(i) for i in td]
        gnorm, gtang = list(nd_), list(td)
        d2set = list(set(ltang) | set(lnorm))
        g2set = [iv[i] for i in d2set]
        if nd_ | td:
            add("Krhs", gfree, g2set, -Ke[np.ix_(dfree, d2set)])
            ind1.update(g2set)
            for i in g2set:
                add("Krhs", [i], [i], 0.0)
            add("Kfs", gtang, gfree, Ke[np.ix_(ltang, dfree)])
            add("Kfs", gfree, gtang, Ke[np.ix_(dfree, ltang)])
            add("Kfs", gtang, gtang, Ke[np.ix_(ltang, ltang)])
            ind1fs.update(gtang)
            add("Rwfs", gtang, iw, Rwe[ltang, :])
            add("Rdfs", gtang, nodes, Rde[ltang, :])
            add("Krhsfs", gtang, gnorm, -Ke[np.ix_(ltang, lnorm)])
            add("Krhsfs", gfree, gnorm, -Ke[np.ix_(dfree, lnorm)])
            for i in gnorm:
                add("Krhsfs", [i], [i], 0.0)
        add("K", gfree, gfree, Ke[np.ix_(dfree, dfree)])
        for i in g2set:
            add("K", [i], [i], 0.0)
        add("Rw", gfree, iw, Rwe[np.ix_(dfree, range(len(iw)))])
        add("Rd", gfree, nodes, Rde[np.ix_(dfree, range(len(nodes)))])
    for i in ind1:  # setIndices2One (mat_fs.py:115-120)
        add("Krhs", [i], [i], 1.0)
        add("K", [i], [i], 1.0)
    for i in ind1fs:
        add("Kfs", [i], [i], -1.0)
    for i in ind1 - ind1fs:
        add("Krhsfs", [i], [i], 1.0, addv=False)
    n = mesh.N * dim
    ncols = {"Rw": mesh.N * dw, "Rwfs": mesh.N * dw, "Rd": mesh.N, "Rdfs": mesh.N}
    return {k: _dok_csr(v, n, ncols.get(k, n)) for k, v in mats.items()}
