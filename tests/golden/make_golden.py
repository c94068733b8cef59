"""Generate the golden fixtures under tests/golden/ from the reference's OWN code.

Runs ONLY in the build container, where /root/reference exists.  The GPU box
never imports the reference: it only reads the .npz files written here.

What is executed from the reference (imported, unmodified):
  * src/domain/elements/utilities.py  gaussPoints / lobattoPoints      (a1)
  * src/domain/elements/spectral.py   Spectral tables, getSpectralOrder,
                                      getElemKLEMatrices/Operators      (a3-a5)
  * src/matrices/mat_fs.py            MatFS.build / Operators            (a8,a10,a12)
  * src/matrices/mat_ns.py            MatNS.build                        (a11)
  * src/solver/kle_solver.py          KleSolver.setUp / solve / solveFS  (a13)
  * src/boundaries/boundary*.py       DoF sets, setValuesToVec           (a13)
  * src/functions/taylor_green*.py    analytic inputs

What is stubbed (the reference needs PETSc/mpi4py, which are absent here):
  * mpi4py -> an empty module (only the unused import at element.py:3)
  * petsc4py.PETSc -> a small scipy-free dict-of-keys Mat / dense Vec /
    direct-solve KSP implementing exactly the subset listed in SURVEY.md 8(b).
    Mat.setValues keeps explicit zeros and sums ADD_VALUES in call order,
    like MatSetValues_SeqAIJ; KSP.__call__ is a dense direct solve (numpy),
    the stand-in for `-ksp_type preonly -pc_type lu` (makefile:7).
  * Domain/DMPlex -> FakeDomain below, on the build's canonical structured
    numbering (lattice node id = ix + Lx*(iy + Ly*iz), cells x-fastest, cell
    corners in DMPlex closure order, test_dmplex_wrapper.py:24-27,106-115).

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
import os
import sys
import types

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))  # repo root: oracle, meshgen
from oracle import oracle as O  # noqa: E402
from pynama_amd.meshgen import perturbed_box  # noqa: E402

# ---------------------------------------------------------------- stubs ----
_mpi = types.ModuleType("mpi4py")
_mpi.MPI = types.SimpleNamespace(COMM_WORLD=None)
sys.modules["mpi4py"] = _mpi
sys.modules["mpi4py.MPI"] = _mpi.MPI


class _Comm:
    rank = 0
    size = 1

    def tompi4py(self):
        return self

    def allgather(self, obj):
        return [obj]


class _Vec:
    def __init__(self, n=0):
        self.a = np.zeros(n)
        self.name = ""

    # petsc4py creation API
    def createMPI(self, size, comm=None):
        n = size[0] if isinstance(size, tuple) else size
        self.a = np.zeros(int(n))
        return self

    def createSeq(self, n):
        self.a = np.zeros(int(n))
        return self

    def createWithArray(self, arr):
        self.a = np.array(arr, dtype=float)
        return self

    def setName(self, s):
        self.name = s

    def getName(self):
        return self.name

    def getSize(self):
        return len(self.a)

    def getOwnershipRange(self):
        return (0, len(self.a))

    @property
    def owner_range(self):
        return (0, len(self.a))

    def setValues(self, idx, vals, addv=False):
        idx = np.atleast_1d(np.asarray(idx, dtype=np.int64))
        vals = np.broadcast_to(np.asarray(vals, dtype=float), idx.shape)
        if addv:
            for i, v in zip(idx, vals):
                self.a[i] += v
        else:
            self.a[idx] = vals

    def setValue(self, i, v):
        self.a[i] = v

    def assemble(self):
        pass

    def set(self, v):
        self.a[:] = v

    def getArray(self):
        return self.a

    def reciprocal(self):
        self.a = 1.0 / self.a

    def duplicate(self):
        return _Vec(len(self.a))

    def copy(self):
        v = _Vec()
        v.a = self.a.copy()
        return v

    def axpy(self, alpha, x):
        self.a += alpha * x.a

    def scale(self, s):
        self.a *= s

    def __imul__(self, s):
        self.a *= s
        return self

    def __add__(self, o):
        v = _Vec()
        v.a = self.a + o.a
        return v

    def __sub__(self, o):
        v = _Vec()
        v.a = self.a - o.a
        return v

    def __mul__(self, o):
        v = _Vec()
        v.a = self.a * (o.a if isinstance(o, _Vec) else o)
        return v

    def dot(self, o):
        return float(self.a @ o.a)

    def norm(self, norm_type=2):
        return float(np.linalg.norm(self.a))

    def destroy(self):
        pass

    def __array__(self, dtype=None, copy=None):
        return self.a


class _Mat:
    """Dict-of-keys AIJ: explicit zeros kept, ADD sums in call order."""

    def __init__(self):
        self.m = self.n = 0
        self.e = {}
        self.name = ""

    def createAIJ(self, size, nnz=None, comm=None):
        (self.m, _), (self.n, _) = size
        self.m, self.n = int(self.m), int(self.n)
        return self

    def setUp(self):
        pass

    def setName(self, s):
        self.name = s

    def getName(self):
        return self.name

    def getSize(self):
        return (self.m, self.n)

    def getOwnershipRange(self):
        return (0, self.m)

    def setValues(self, rows, cols, values, addv=False):
        rows = np.atleast_1d(np.asarray(rows, dtype=np.int64))
        cols = np.atleast_1d(np.asarray(cols, dtype=np.int64))
        vals = np.broadcast_to(np.asarray(values, dtype=float), (len(rows), len(cols)))
        for ii, r in enumerate(rows):
            for jj, c in enumerate(cols):
                k = (int(r), int(c))
                if addv:
                    self.e[k] = self.e.get(k, 0.0) + vals[ii, jj]
                else:
                    self.e[k] = vals[ii, jj]

    def assemble(self):
        pass

    def csr(self):
        keys = sorted(self.e.keys())
        indptr = np.zeros(self.m + 1, dtype=np.int64)
        for r, _ in keys:
            indptr[r + 1] += 1
        indptr = np.cumsum(indptr)
        indices = np.array([c for _, c in keys], dtype=np.int64)
        data = np.array([self.e[k] for k in keys], dtype=float)
        return indptr, indices, data

    def dense(self):
        d = np.zeros((self.m, self.n))
        for (r, c), v in self.e.items():
            d[r, c] = v
        return d

    def diagonalScale(self, L=None, R=None):
        for (r, c) in self.e:
            if L is not None:
                self.e[(r, c)] *= L.a[r]
            if R is not None:
                self.e[(r, c)] *= R.a[c]

    def createVecLeft(self):
        return _Vec(self.m)

    def createVecRight(self):
        return _Vec(self.n)

    def mult(self, x, y):
        out = np.zeros(self.m)
        for (r, c), v in self.e.items():
            out[r] += v * x.a[c]
        y.a[:] = out

    def __mul__(self, x):
        y = _Vec(self.m)
        self.mult(x, y)
        return y

    def __add__(self, o):
        s = _Mat()
        s.m, s.n = self.m, self.n
        s.e = dict(self.e)
        for k, v in o.e.items():
            s.e[k] = s.e.get(k, 0.0) + v
        return s

    def destroy(self):
        pass


class _PC:
    def create(self, comm=None):
        return self

    def setType(self, t):
        self.type = t


class _KSP:
    def create(self, comm=None):
        return self

    def setType(self, t):
        self.ksp_type = t

    def setPC(self, pc):
        self.pc = pc

    def setFromOptions(self):
        pass

    def setOperators(self, A):
        self.A = A

    def setUp(self):
        # direct solve standing in for the makefile's preonly + lu: dense up
        # to a few thousand unknowns (every fixture before cavity2d_full),
        # sparse LU (scipy SuperLU) beyond, where a dense copy would not fit
        if self.A.m <= 5000:
            self._dense = self.A.dense()
            self._lu = None
        else:
            import scipy.sparse as sp
            from scipy.sparse.linalg import splu
            ip, ix, d = self.A.csr()
            self._lu = splu(sp.csr_matrix((d, ix, ip), shape=(self.A.m, self.A.n)).tocsc())

    def __call__(self, b, x):
        if self._lu is None:
            x.a[:] = np.linalg.solve(self._dense, b.a)
        else:
            x.a[:] = self._lu.solve(b.a)


class _IS:
    def __init__(self):
        self.idx = np.zeros(0, dtype=np.int64)
        self.bs = 1

    def createGeneral(self, idx, comm=None):
        self.idx = np.asarray(idx, dtype=np.int64)
        return self

    def createBlock(self, bs, blocks, comm=None):
        self.bs = bs
        blocks = np.asarray(blocks, dtype=np.int64)
        self.idx = (blocks[:, None] * bs + np.arange(bs)[None, :]).ravel()
        return self

    def getIndices(self):
        return self.idx

    def getBlockIndices(self):
        return self.idx[:: self.bs] // self.bs

    def getBlockSize(self):
        return self.bs

    def union(self, o):
        r = _IS()
        r.idx = np.union1d(self.idx, o.idx)
        return r


_petsc = types.ModuleType("petsc4py.PETSc")
_petsc.COMM_WORLD = _Comm()
_petsc.Mat = _Mat
_petsc.Vec = _Vec
_petsc.KSP = _KSP
_petsc.PC = _PC
_petsc.IS = _IS
_p4 = types.ModuleType("petsc4py")
_p4.PETSc = _petsc
_p4.init = lambda *a, **k: None
sys.modules["petsc4py"] = _p4
sys.modules["petsc4py.PETSc"] = _petsc

sys.path.insert(0, REF_SRC)
from domain.elements.spectral import Spectral  # noqa: E402
from domain.elements.utilities import gaussPoints, lobattoPoints  # noqa: E402
from domain.indices import IndicesManager  # noqa: E402
from matrices.mat_fs import MatFS  # noqa: E402
from matrices.mat_ns import MatNS  # noqa: E402
from solver.kle_solver import KleSolver  # noqa: E402
from boundaries.boundary_conditions import BoundaryConditions  # noqa: E402
import functions.taylor_green as tg2d  # noqa: E402
import functions.taylor_green3d as tg3d  # noqa: E402

# BaseProblem.evalRHS (cases/base_problem.py:111-154) is called unbound on a
# namespace; the module's imports that are not on that path (viewer, TS, DMPlex
# domain, timers) are replaced by empty modules so it can be imported.
for _name in ("domain.domain", "viewer.paraviewer", "solver.ts_solver", "common.timer"):
    _m = types.ModuleType(_name)
    for _attr in ("Domain", "Paraviewer", "TsSolver", "Timer"):
        setattr(_m, _attr, object)
    sys.modules[_name] = _m
from cases.base_problem import BaseProblem  # noqa: E402

CORNERS = {
    2: [(0, 0), (1, 0), (1, 1), (0, 1)],
    3: [(0, 0, 0), (0, 1, 0), (1, 1, 0), (1, 0, 0),
        (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)],
}
FACES = {2: ["down", "right", "up", "left"],
         3: ["back", "front", "down", "up", "right", "left"]}
# face name -> (axis, side) ; DMPlex box "Face Sets" numbering (dmplex.py:173-176)
FACE_AXIS = {"left": (0, 0), "right": (0, 1), "down": (1, 0), "up": (1, 1),
             "back": (2, 0), "front": (2, 1)}


class FakeDomain:
    """Structured box mesh in the build's canonical numbering."""

    def __init__(self, dim, nelem, lower, upper, ngl, bc):
        self.dim = dim
        self.dim_w = 1 if dim == 2 else 3
        self.dim_s = 3 if dim == 2 else 6
        self.nelem = np.array(nelem)
        self.lower = np.array(lower, float)
        self.upper = np.array(upper, float)
        self.ngl = ngl
        p = ngl - 1
        self.p = p
        self.L = self.nelem * p + 1
        self.N = int(np.prod(self.L))
        self.E = int(np.prod(self.nelem))
        self.elem = Spectral(ngl, dim)
        self.h = (self.upper - self.lower) / self.nelem
        # local node -> lattice offset from the reference's own HCooOp (a9)
        unit = np.array(CORNERS[dim], float)
        # GLL nodes on [0,1]: the element's nodes are NOT equispaced
        xi = (1.0 + np.sort(lobattoPoints(ngl)[0])) / 2.0
        offs = []
        for q in range(len(self.elem.gpsOp)):
            x = self.elem.HCooOp[q] @ unit
            o = np.array([int(np.argmin(np.abs(xi - c))) for c in x])
            assert np.allclose(xi[o], x, atol=1e-13)
            offs.append(o)
        self.loc2lat = np.array(offs)
        self.xi = xi
        self.conn = np.zeros((self.E, ngl ** dim), dtype=np.int64)
        self.corners = np.zeros((self.E, 2 ** dim, dim))
        for e in range(self.E):
            eidx = np.array(np.unravel_index(e, self.nelem[::-1])[::-1])
            lat = eidx * p + self.loc2lat
            self.conn[e] = self.node_id(lat)
            self.corners[e] = self.lower + (eidx + unit) * self.h
        lat = np.stack(np.meshgrid(*[np.arange(n) for n in self.L[::-1]],
                                   indexing="ij")[::-1], -1).reshape(-1, dim)
        self.coords = self.lower + (lat // p + xi[lat % p]) * self.h
        top = lat == (self.L - 1)  # last lattice plane: xi index p of last element
        self.coords = np.where(top, self.upper, self.coords)
        self.lat = lat
        # boundary conditions through the reference's own BoundaryConditions
        self.bc = BoundaryConditions(FACES[dim])
        self.bc.setBoundaryConditions(bc)
        for name in self.bc.getNames():
            self.bc.setBoundaryNodes(name, self.border_nodes(name))
        for name in self.bc.getBordersNeedsCoords():
            inds = self.bc.getIndicesByName(name)
            nodes = inds[:: dim] // dim
            self.bc.setBoundaryCoords(name, self.coords[nodes].ravel().copy())
        # connectivity sets (a8): nodes sharing a cell
        adj = [set() for _ in range(self.N)]
        for e in range(self.E):
            s = set(self.conn[e].tolist())
            for n in self.conn[e]:
                adj[n] |= s
        self.adj = adj

    def node_id(self, lat):
        lat = np.atleast_2d(lat)
        idx = lat[:, -1].copy()
        for d in range(self.dim - 2, -1, -1):
            idx = idx * self.L[d] + lat[:, d]
        return idx

    def border_nodes(self, name):
        ax, side = FACE_AXIS[name]
        v = 0 if side == 0 else self.L[ax] - 1
        return np.nonzero(self.lat[:, ax] == v)[0].tolist()

    # ---- the Domain subset MatFS / MatNS / KleSolver call -------------
    def getDimension(self):
        return self.dim

    def getDimensions(self):
        return self.dim, self.dim_w, self.dim_s

    def getNodesRange(self):
        return (0, self.N)

    def getLocalCellRange(self):
        return (0, self.E)

    def getConnectivity(self):
        ind_d = np.zeros(self.N, dtype=object)
        ind_o = np.zeros(self.N, dtype=object)
        nd = np.zeros(self.N, dtype=np.int32)
        no = np.zeros(self.N, dtype=np.int32)
        for i in range(self.N):
            ind_d[i] = set(self.adj[i])
            ind_o[i] = set()
            nd[i] = len(ind_d[i])
        return ind_d, ind_o, nd, no

    def getNodesDirichlet(self, collect=False):
        return self.bc.getNodesByType("free-slip", allGather=collect)

    def getNodesNoSlip(self, collect=False):
        return self.bc.getNodesByType("no-slip", allGather=collect)

    def getTangDofs(self, collect=False):
        return self.bc.getNoSlipTangDofs(allGather=collect)

    def getNormalDofs(self, collect=False):
        return self.bc.getNoSlipNormalDofs(allGather=collect)

    def computeLocalKLEMats(self, cell):
        mats = self.elem.getElemKLEMatrices(self.corners[cell].ravel().copy())
        nodes = self.conn[cell].tolist()
        iv = [n * self.dim + d for n in nodes for d in range(self.dim)]
        iw = [n * self.dim_w + d for n in nodes for d in range(self.dim_w)]
        return nodes, (iv, iw), mats

    def computeLocalOperators(self, cell):
        ops = self.elem.getElemKLEOperators(self.corners[cell].ravel().copy())
        return self.conn[cell].tolist(), ops

    def applyBoundaryConditions(self, vec, name, t=None, nu=None):
        self.bc.setValuesToVec(vec, name, t, nu)

    def applyBoundaryConditionsNS(self, vec, name, t=None, nu=None):
        self.bc.setTangentialValuesToVec(vec, name, t, nu)


class FakeUDomain(FakeDomain):
    """Unstructured quad/hex mesh (GmshDom stand-in) on the oracle's
    coordinate numbering (oracle.UMesh); the element matrices, assembly, BCs
    and solve are the reference's own code as for FakeDomain.  Boundary name
    i = Face Sets value i + 1 (dmplex.py:175-178)."""

    def __init__(self, umesh, bc):
        dim, ngl = umesh.dim, umesh.ngl
        self.dim = dim
        self.dim_w = 1 if dim == 2 else 3
        self.dim_s = 3 if dim == 2 else 6
        self.ngl = ngl
        self.N, self.E = umesh.N, umesh.E
        self.elem = Spectral(ngl, dim)
        self.corners = umesh.corners().copy()
        self.coords = umesh.coords().copy()
        # the reference's element-local node order (spectral / closure order):
        # node q of cell e sits at HCooOp[q] @ corners (dmplex.py:62-91)
        from scipy.spatial import cKDTree
        tree = cKDTree(self.coords)
        H = np.array(self.elem.HCooOp)
        self.conn = np.zeros((self.E, len(H)), dtype=np.int64)
        for e in range(self.E):
            d, idx = tree.query(H @ self.corners[e])
            assert d.max() < 1e-9
            self.conn[e] = idx
        self.umesh = umesh
        self.bc = BoundaryConditions(FACES[dim])
        self.bc.setBoundaryConditions(bc)
        for name in self.bc.getNames():
            self.bc.setBoundaryNodes(name, self.border_nodes(name))
        for name in self.bc.getBordersNeedsCoords():
            inds = self.bc.getIndicesByName(name)
            nodes = inds[:: dim] // dim
            self.bc.setBoundaryCoords(name, self.coords[nodes].ravel().copy())
        adj = [set() for _ in range(self.N)]
        for e in range(self.E):
            st = set(self.conn[e].tolist())
            for n in self.conn[e]:
                adj[n] |= st
        self.adj = adj

    def border_nodes(self, name):
        return self.umesh.face_nodes(1 << FACES[self.dim].index(name)).tolist()


def csr_dict(prefix, mat):
    ip, ix, d = mat.csr()
    return {f"{prefix}_indptr": ip, f"{prefix}_indices": ix, f"{prefix}_data": d,
            f"{prefix}_shape": np.array(mat.getSize())}


def table_fixtures():
    out = {}
    for n in range(1, 9):
        x, w = gaussPoints(n)
        out[f"gauss_x_{n}"], out[f"gauss_w_{n}"] = x, w
    for n in range(2, 9):
        x, w = lobattoPoints(n)
        out[f"lobatto_x_{n}"], out[f"lobatto_w_{n}"] = x, w
    for n in range(1, 9):
        out[f"spectral_order_{n}"] = np.array(Spectral.getSpectralOrder(n))
    rng = np.arange(27)
    out["reorder3d"] = IndicesManager.reorderEntities3D(rng)
    out["reorder2d"] = IndicesManager.reorderEntities2D(np.arange(9))
    for dim, ngls in ((2, range(2, 9)), (3, range(2, 6))):
        for ngl in ngls:
            s = Spectral(ngl, dim)
            k = f"{dim}d_{ngl}"
            for nm in ("H", "Hrs", "HRed", "HrsRed", "HOp", "HrsOp", "HCoo",
                       "HrsCoo", "HCooRed", "HrsCooRed", "HCooOp"):
                out[f"{nm}_{k}"] = np.array(getattr(s, nm), dtype=float)
            for nm in ("gps", "gpsRed", "gpsOp"):
                out[f"{nm}_{k}"] = np.array([tuple(g) for g in getattr(s, nm)])
    np.savez_compressed(os.path.join(OUT, "tables.npz"), **out)


def element_fixtures():
    out = {}
    box = {2: np.array([0.3, 0.1, 0.55, 0.1, 0.55, 0.35, 0.3, 0.35]),
           3: None}
    c3 = np.array(CORNERS[3], float) * np.array([0.25, 0.2, 0.125]) + [0.1, 0.2, 0.3]
    box[3] = c3.ravel()
    skew = {2: np.array([0.0, 0.0, 1.1, 0.1, 1.3, 0.9, -0.1, 1.2]),
            3: (np.array(CORNERS[3], float)
                + 0.1 * np.array([[0, 0, 0], [0.2, 0, 0.1], [0.3, -0.2, 0],
                                  [0, 0.1, 0.2], [-0.1, 0, 0], [0, 0.3, 0.1],
                                  [0.2, 0.2, 0.2], [0.1, 0, -0.1]])).ravel()}
    # the legacy-test element (test_element.py:271-281)
    legacy = {2: np.array([1, 1, 0, 1, 0, 0, 1, 0], float),
              3: np.array([1, 1, 1, 0, 1, 1, 0, 0, 1, 1, 0, 1, 1, 1, 0, 1, 0, 0,
                           0, 0, 0, 0, 1, 0], float)}
    cases = [(2, n) for n in (2, 3, 5, 7)] + [(3, 2), (3, 3), (3, 5)]
    for dim, ngl in cases:
        s = Spectral(ngl, dim)
        geos = {"box": box[dim], "skew": skew[dim], "legacy": legacy[dim]}
        if (dim, ngl) == (3, 5):
            geos = {"box": box[dim]}
        for gname, X in geos.items():
            k = f"{dim}d_{ngl}_{gname}"
            out[f"X_{k}"] = X.copy()
            K, Rw, Rd = s.getElemKLEMatrices(X.copy())
            out[f"K_{k}"], out[f"Rw_{k}"], out[f"Rd_{k}"] = K, Rw, Rd
            SrT, DivSrT, Curl, W = s.getElemKLEOperators(X.copy())
            out[f"Curl_{k}"], out[f"W_{k}"] = Curl, W
            if ngl <= 3 or dim == 2:
                out[f"SrT_{k}"], out[f"DivSrT_{k}"] = SrT, DivSrT
    np.savez_compressed(os.path.join(OUT, "elements.npz"), **out)


def eval_rhs(dom, mat, solver, vort0, rho, mu, dim, t):
    """One reference evalRHS call at time t from the initial vorticity."""
    op = mat.getOperators()
    ns = types.SimpleNamespace(dom=dom, solverKLE=solver, operator=op, rho=rho, mu=mu, nu=mu / rho,
                               dim=dim, dim_w=1 if dim == 2 else 3, dim_s=3 if dim == 2 else 6)
    ns.vort = vort0.copy()
    ns._VtensV = op.SrT.createVecLeft()
    ns._Aux1 = ns._VtensV.duplicate()
    ns.computeVtensV = lambda vec: BaseProblem.computeVtensV(ns, vec)
    rec = {"rhs_t": t, "rhs_vort_in": ns.vort.a.copy()}
    f = op.Curl.createVecLeft()
    BaseProblem.evalRHS(ns, None, t, ns.vort, f)
    rec.update(rhs_vort_bc=ns.vort.a.copy(), rhs_vel=solver.getSolution().a.copy(), rhs_VtensV=ns._VtensV.a.copy(),
               rhs_Aux1=ns._Aux1.a.copy(), rhs_f=f.a.copy())
    if solver.isNS():
        rec["rhs_velFS"] = solver.getFreeSlipSolution().a.copy()
    return rec


def assembled_case(name, dim, nelem, ngl, bc, rho, mu, fn, ns=False, ops=True, umesh=None, extra=None,
                   vectors_only=False):
    """The reference's MatFS / MatNS, KleSolver and evalRHS on one case.
    vectors_only: keep the solve's vectors and the DoF sets, not the
    matrices, connectivity or coordinates (a case at a stated config size)."""
    lower = [0.0] * dim
    upper = [1.0] * dim
    dom = FakeDomain(dim, nelem, lower, upper, ngl, bc) if umesh is None else FakeUDomain(umesh, bc)
    mat = MatNS() if ns else MatFS()
    mat.setDomain(dom)
    if not ops:
        mat.buildOperators = lambda: None
        mat.build(buildOperators=False)
    else:
        mat.build()
    solver = KleSolver()
    solver.setMat(mat)
    solver.setUp()
    out = {"dim": dim, "nelem": np.array(nelem), "ngl": ngl, "lower": np.array(lower),
           "upper": np.array(upper), "conn": dom.conn, "coords": dom.coords,
           "corners": dom.corners, "rho": rho, "mu": mu}
    if umesh is None:
        out["loc2lat"] = dom.loc2lat
    out.update(extra or {})
    for m in ("K", "Krhs", "Rw"):
        out.update(csr_dict(m, getattr(mat, m)))
    if ns:
        for m in ("Rd", "Kfs", "Krhsfs", "Rwfs", "Rdfs"):
            out.update(csr_dict(m, getattr(mat, m)))
    if ops:
        op = mat.getOperators()
        for m in ("Curl", "SrT", "DivSrT"):
            out.update(csr_dict(m, getattr(op, m)))
    dirn = np.array(sorted(dom.getNodesDirichlet(collect=True)), dtype=np.int64)
    out["dir_nodes"] = dirn
    nu = mu / rho
    vel = solver.getSolution()
    vort = mat.Rw.createVecRight()
    if ns:  # cavity: vorticity IC 0, velocity from the walls only
        u_ex = np.zeros(dom.N * dim)
        w_ex = np.zeros(dom.N * dom.dim_w)
    elif fn is None:  # uniform [4,0]
        u_ex = np.tile([4.0, 0.0], dom.N)
        w_ex = np.zeros(dom.N * dom.dim_w)
    else:
        alpha = fn.alpha(nu, 0.0)
        u_ex = fn.velocity(dom.coords, alpha)
        w_ex = np.asarray(fn.vorticity(dom.coords, alpha)).ravel()
    vel.a[:] = u_ex  # initial condition (base_problem.py:193-211)
    vort.a[:] = w_ex
    if ns:
        dom.applyBoundaryConditions(vort, "vorticity", 0.0, nu)
        dom.applyBoundaryConditions(vel, "velocity", 0.0, nu)
        out["vel0"] = vel.a.copy()
        out["vort0"] = vort.a.copy()
        solver.solveFS(vort)
        velFS = solver.getFreeSlipSolution()
        out["velFS"] = velFS.a.copy()
        out["bFS"] = (mat.Rw * vort + mat.Rwfs * vort + mat.Krhsfs * vel).a.copy()
        out["tang_dofs"] = np.array(sorted(dom.getTangDofs(collect=True)))
        out["normal_dofs"] = np.array(sorted(dom.getNormalDofs(collect=True)))
    else:
        dom.applyBoundaryConditions(vel, "velocity", 0.0, nu)
        out["vel0"] = vel.a.copy()
        out["vort0"] = vort.a.copy()
    b = (mat.Rw * vort + mat.Krhs * vel).a.copy()
    solver.solve(vort)
    u = solver.getSolution().a.copy()
    if ops:
        out.update(eval_rhs(dom, mat, solver, vort, rho, mu, dim, 0.25))
        solver.getSolution().a[:] = u  # restore the t=0 solution
    out["b"] = b
    out["u"] = u
    out["u_exact"] = u_ex
    out["err_l2"] = np.linalg.norm(u - u_ex)
    if vectors_only:
        keep = ("dim", "nelem", "ngl", "lower", "upper", "rho", "mu", "dir_nodes", "vel0", "vort0", "velFS", "bFS",
                "tang_dofs", "normal_dofs", "b", "u", "rhs_t", "rhs_vort_in", "rhs_vort_bc", "rhs_vel", "rhs_velFS", "rhs_f",
                "err_l2")
        out = {k: v for k, v in out.items() if k in keep}
        out["K_nnz"] = np.array(len(mat.K.csr()[2]))
    np.savez_compressed(os.path.join(OUT, f"case_{name}.npz"), **out)
    print(name, "n =", len(u), "nnz(K) =", len(out["K_data"]) if "K_data" in out else int(out["K_nnz"]),
          "err =", out["err_l2"])


def xdmf_fixtures():
    """XDMF files from the reference's own XmlGenerator (viewer/xml_generator.py:4-120),
    driven in the call sequence of Paraviewer (viewer/paraviewer.py:21-70):
    saveMesh -> setUpDomainNodes(totalNodes) + generateXMLTemplate; each
    saveData -> generateMeshData("mesh1") + setTimeStamp + per vector a scalar
    attribute if its size equals the node count, else a vector attribute
    (saveStepInXML); writeXmf -> writeFile.  Paraviewer itself imports
    petsc4py, so the sequence is restated here; the element tree is the
    reference class's."""
    from viewer.xml_generator import XmlGenerator
    for dim, n in ((2, 13), (3, 17)):
        gen = XmlGenerator(dim, "vec-data")
        gen.setUpDomainNodes(totalNodes=n)
        gen.generateXMLTemplate()
        vecs = [("velocity", dim * n), ("vorticity", (1 if dim == 2 else 3) * n), ("num proc", n)]
        for step, t in ((1, 0.1), (2, 0.2), (10, 1.25)):
            grid = gen.generateMeshData("mesh1")
            gen.setTimeStamp(t, grid)
            for name, size in vecs:
                if size == gen.dimensions:
                    gen.setScalarAttribute(name, step, grid)
                else:
                    gen.setVectorAttribute(name, step, grid)
        gen.writeFile(os.path.join(OUT, f"xdmf_{dim}d"))


class _Sec:
    """Duck-typed PetscSection for IndicesManager.getSectionOffset
    (indices.py:111-118): closure point p owns `dof[p]` nodes from offset[p]."""

    def __init__(self, dofs):
        self.dof = list(dofs)
        self.off = list(np.concatenate([[0], np.cumsum(self.dof)[:-1]]).astype(int))

    def getOffset(self, p):
        return int(self.off[p])

    def getDof(self, p):
        return int(self.dof[p])


def orientation_fixtures():
    """IndicesManager.mapEntitiesToNodes (indices.py:69-92) on one cell's
    closure with a duck-typed section, for every orientation code of every
    edge / face slot (one slot at a time, the others 0) and for all slots at
    once.  Closure order (DMPlex): 3-D [cell, 6 faces, 12 edges, 8 vertices],
    2-D [cell, 4 edges, 4 vertices]; point p's nodes are the section range
    [off[p], off[p] + dof[p]) (dof per entity: getNumCompAndNumDof,
    indices.py:22-30).  Feeds tests/test_umesh.py's orientation-rule test."""
    comm = types.SimpleNamespace(rank=0)
    out = {}
    for dim, ngls in ((2, (3, 4, 5)), (3, (3, 4, 5))):
        for ngl in ngls:
            m = ngl - 2
            if dim == 3:
                dofs = [m ** 3] + [m * m] * 6 + [m] * 12 + [1] * 8
                slots = {"face": range(1, 7), "edge": range(7, 19), "cell": [0]}
            else:
                dofs = [m * m] + [m] * 4 + [1] * 4
                slots = {"edge": range(1, 5), "cell": [0]}
            im = IndicesManager(dim, ngl, comm)
            im.setGlobalIndicesSection(_Sec(dofs))
            ent = np.arange(len(dofs))
            codes = {"face": range(-4, 4), "edge": range(-2, 2), "cell": range(-1, 2)}
            k = f"d{dim}_n{ngl}"
            out[f"{k}_dofs"] = np.array(dofs)
            out[f"{k}_base"] = np.array(im.mapEntitiesToNodes(ent, np.zeros(len(dofs), int)))
            for kind, sl in slots.items():
                for slot in sl:
                    for o in codes[kind]:
                        ori = np.zeros(len(dofs), int)
                        ori[slot] = o
                        out[f"{k}_{kind}{slot}_o{o}"] = np.array(im.mapEntitiesToNodes(ent, ori))
            ori = np.array([1] * len(dofs))
            out[f"{k}_all1"] = np.array(im.mapEntitiesToNodes(ent, ori))
    np.savez_compressed(os.path.join(OUT, "orientation.npz"), **out)


def main(only=()):
    """Regenerate every fixture, or only the named cases (e.g. `gmsh2d`)."""
    uni = {"uniform": {"velocity": [4, 0]}}
    tg = {"custom-func": {"name": "taylor_green", "attributes": ["velocity", "vorticity", "alpha"]}}
    tg3 = {"custom-func": {"name": "taylor_green3d", "attributes": ["velocity", "vorticity", "alpha"]}}
    cav = {"no-slip": {"up": [2, 0], "down": [0, 0], "left": [0, 0], "right": [0, 0]}}
    NS3 = {"no-slip": {"up": [1, 0, 0.5], "down": [0, 0, 0], "left": [0, 0, 0], "right": [0, 0, 0],
                       "front": [0, 0, 0], "back": [0, 0, 0]}}

    def unstructured():
        um = O.UMesh.from_gmsh(os.path.join(OUT, "test.msh"), 3)
        V, Cc, F, T = perturbed_box(3, [2, 2, 2], seed=11)
        return um, O.UMesh(3, 3, V, Cc, F, T), {"mesh_vertices": V, "mesh_cells": Cc, "mesh_facets": F,
                                                 "mesh_tags": T}

    cases = {
        "tables": table_fixtures,
        "elements": element_fixtures,
        "xdmf": xdmf_fixtures,
        "orientation": orientation_fixtures,
        # test_solver.py:7-25  (uniform, 3x3, ngl=3, rho=1, mu=0.01)
        "uniform2d": lambda: assembled_case("uniform2d", 2, [3, 3], 3, uni, 1.0, 0.01, None),
        # test_solver.py:27-37 (Taylor-Green 2-D, 10x10, ngl=5)
        "tg2d": lambda: assembled_case("tg2d", 2, [10, 10], 5, tg, 0.5, 0.01, tg2d, ops=False),
        "tg2d_small": lambda: assembled_case("tg2d_small", 2, [4, 3], 4, tg, 0.5, 0.01, tg2d),
        "tg3d": lambda: assembled_case("tg3d", 3, [2, 2, 2], 3, tg3, 0.5, 0.01, tg3d),
        "tg3d_p4": lambda: assembled_case("tg3d_p4", 3, [1, 1, 2], 5, tg3, 0.5, 0.01, tg3d, ops=False),
        "cavity2d": lambda: assembled_case("cavity2d", 2, [4, 4], 3, cav, 0.5, 0.01, None, ns=True),
        # BASELINE config 1 as stated: src/cases/cavity-2d.yaml as-is (50 x 50,
        # ngl 3, rho 0.5, mu 0.01, no-slip walls, lid [2, 0]); vectors only
        "cavity2d_full": lambda: assembled_case("cavity2d_full", 2, [50, 50], 3, cav, 0.5, 0.01, None, ns=True,
                                                vectors_only=True),
        # unstructured: the reference's Gmsh fixture
        # src/tests/test.msh (copied to tests/golden/test.msh) and a rotated /
        # shuffled / perturbed hex mesh
        "gmsh2d": lambda: assembled_case("gmsh2d", 2, [0, 0], 3, tg, 0.5, 0.01, tg2d, umesh=unstructured()[0]),
        "umesh3d": lambda: assembled_case("umesh3d", 3, [0, 0, 0], 3, tg3, 0.5, 0.01, tg3d,
                                          umesh=unstructured()[1], extra=unstructured()[2]),
        # no-slip on the unstructured quad mesh: the fixture's single physical
        # group is the "down" wall (Face Sets value 1)
        "gmsh2d_ns": lambda: assembled_case("gmsh2d_ns", 2, [0, 0], 3, {"no-slip": {"down": [1, 0]}}, 0.5, 0.01,
                                            None, ns=True, umesh=unstructured()[0]),
        # lid-driven cube on the rotated hex mesh (walls by Face Sets name)
        "umesh3d_ns": lambda: assembled_case("umesh3d_ns", 3, [0, 0, 0], 3, NS3, 0.5, 0.01, None, ns=True,
                                             umesh=unstructured()[1], extra=unstructured()[2]),
    }
    for name, fn in cases.items():
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
