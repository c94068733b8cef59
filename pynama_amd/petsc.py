"""petsc4py-shaped Mat / Vec / KSP / PC / Options over libkle (device-resident).

Mirrors exactly the petsc4py subset Pynama's hot path uses:
  Mat: createAIJ, setUp, setName/getName, setValues(addv), assemble,
       diagonalScale(L=), createVecLeft/Right, getOwnershipRange, mult,
       Mat*Vec, Mat+Mat, destroy                 (mat_fs.py, kle_solver.py)
  Vec: createMPI, setValues(addv), setValue, assemble, set, reciprocal,
       duplicate, copy, getArray, axpy, scale, *=, +, -, *, dot, norm
                                                 (base_problem.py, mat_fs.py)
  KSP: create, setType, setPC, setFromOptions, setOperators, setUp, solve,
       __call__(b, x)                            (kle_solver.py:49-64)
  PC:  create, setType
  IS:  createGeneral, createBlock, union, getIndices, getBlockIndices
                                                 (boundary_conditions.py:1,187-250)
  COMM_WORLD.tompi4py().allgather                (boundary_conditions.py:201-271)
  Options: getString/getInt/getReal              (run_case.py:9-13)
The surface the reference's host files use is scanned from their source
(tools/scan_petsc4py_surface.py -> tests/golden/petsc4py_surface.json) and
tests/test_host.py checks that every entry exists here.
Errors raise ``Error`` (ierr = PETSc-style code).  Differences from petsc4py:
Vec.getArray() returns a host COPY of the owned part (device memory), use
setArray() to write back.
"""
import ctypes as C
import sys

import numpy as np

from ._lib import Error, call
from .runtime import COMM_WORLD, get_ctx

INSERT_VALUES, ADD_VALUES = 0, 1


def _h(obj):
    return obj._h if obj is not None else None


def _i64(a):
    if isinstance(a, (set, frozenset)):
        a = sorted(a)
    return np.ascontiguousarray(np.atleast_1d(np.asarray(a, dtype=np.int64)))


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


class Options(dict):
    """PETSc options database (-key value pairs from argv + programmatic)."""

    _db = None

    def __new__(cls, prefix=None):
        if Options._db is None:
            db = dict.__new__(cls)
            dict.__init__(db)
            argv = sys.argv[1:]
            i = 0
            while i < len(argv):
                a = argv[i]
                if a.startswith("-") and len(a) > 1 and not a[1:2].isdigit():
                    key = a.lstrip("-")
                    if i + 1 < len(argv) and not (argv[i + 1].startswith("-") and not argv[i + 1][1:2].isdigit()):
                        db[key] = argv[i + 1]
                        i += 1
                    else:
                        db[key] = "true"
                i += 1
            Options._db = db
        return Options._db

    def __init__(self, prefix=None):
        pass

    def getString(self, key, default=None):
        return str(self[key]) if key in self else default

    def getInt(self, key, default=None):
        return int(self[key]) if key in self else default

    def getReal(self, key, default=None):
        return float(self[key]) if key in self else default

    def getBool(self, key, default=None):
        if key not in self:
            return default
        return str(self[key]).lower() in ("1", "true", "yes", "on")

    def setValue(self, key, value):
        self[key.lstrip("-")] = value

    def delValue(self, key):
        self.pop(key.lstrip("-"), None)


class Vec:
    def __init__(self):
        self._h = None
        self._name = ""
        self._ctx = None

    # ------------------------------------------------------------ creation
    @classmethod
    def _wrap(cls, handle, ctx):
        v = cls()
        v._h = handle
        v._ctx = ctx
        return v

    def createMPI(self, size, comm=None):
        if isinstance(size, (tuple, list)):
            nl, ng = size[0], size[1] if len(size) > 1 else None
        else:
            nl, ng = size, None
        ctx = get_ctx()
        if nl is None:
            nl = ng // ctx.nranks + (1 if ctx.rank < ng % ctx.nranks else 0)
        h = C.c_void_p()
        call("kle_vec_create", ctx.h, int(nl), -1 if ng is None else int(ng), C.byref(h))
        self._h, self._ctx = h, ctx
        return self

    def createSeq(self, n, comm=None):
        return self.createMPI((n, n))

    def createWithArray(self, array, size=None, comm=None):
        a = _f64(array).ravel()
        self.createMPI((len(a), None))
        self.setArray(a)
        return self

    @classmethod
    def fromMesh(cls, mesh, bs):
        ctx = get_ctx()
        h = C.c_void_p()
        call("kle_vec_create_mesh", ctx.h, mesh._h, int(bs), C.byref(h))
        return cls._wrap(h, ctx)

    def duplicate(self):
        h = C.c_void_p()
        call("kle_vec_duplicate", self._h, C.byref(h))
        return Vec._wrap(h, self._ctx)

    def copy(self, result=None):
        if result is None:
            result = self.duplicate()
        call("kle_vec_copy", self._h, result._h)
        return result

    def destroy(self):
        if self._h:
            call("kle_vec_destroy", self._h)
            self._h = None
        return self

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    # --------------------------------------------------------------- sizes
    def setName(self, name):
        self._name = name

    def getName(self):
        return self._name

    def getSizes(self):
        nl, ng = C.c_int64(), C.c_int64()
        call("kle_vec_get_sizes", self._h, C.byref(nl), C.byref(ng))
        return nl.value, ng.value

    def getSize(self):
        return self.getSizes()[1]

    def getLocalSize(self):
        return self.getSizes()[0]

    def getOwnershipRange(self):
        lo, hi = C.c_int64(), C.c_int64()
        call("kle_vec_get_ownership_range", self._h, C.byref(lo), C.byref(hi))
        return lo.value, hi.value

    @property
    def owner_range(self):
        return self.getOwnershipRange()

    @property
    def size(self):
        return self.getSize()

    # -------------------------------------------------------------- values
    def setValues(self, indices, values, addv=False):
        idx = _i64(indices)
        vals = _f64(np.broadcast_to(np.asarray(values, dtype=np.float64), idx.shape))
        call("kle_vec_set_values", self._h, len(idx), idx, vals, int(bool(addv)))

    def setValue(self, index, value, addv=False):
        self.setValues([index], [value], addv)

    def getValues(self, indices):
        idx = _i64(indices)
        out = np.zeros(len(idx))
        call("kle_vec_get_values", self._h, len(idx), idx, out)
        return out

    def assemble(self):
        """VecAssemblyBegin/End: setValues already wrote the owned entries."""
        call("kle_vec_assemble", self._h)

    assemblyBegin = assemble
    assemblyEnd = assemble

    def set(self, alpha):
        call("kle_vec_set", self._h, float(alpha))

    def zeroEntries(self):
        self.set(0.0)

    def getArray(self, readonly=False):
        out = np.zeros(self.getLocalSize())
        call("kle_vec_get_array", self._h, out)
        return out

    def setArray(self, array):
        a = _f64(array).ravel()
        if len(a) != self.getLocalSize():
            raise Error(60, f"setArray: {len(a)} values for {self.getLocalSize()} local entries")
        call("kle_vec_set_array", self._h, a)

    @property
    def array(self):
        return self.getArray()

    def __array__(self, dtype=None, copy=None):
        a = self.getArray()
        return a.astype(dtype) if dtype is not None else a

    def ghostUpdate(self, *args, **kw):
        call("kle_vec_ghost_update", self._h)

    # ------------------------------------------------------------- BLAS-1
    def axpy(self, alpha, x):
        call("kle_vec_axpy", self._h, float(alpha), x._h)

    def aypx(self, alpha, x):
        call("kle_vec_aypx", self._h, float(alpha), x._h)

    def waxpy(self, alpha, x, y):
        call("kle_vec_waxpy", self._h, float(alpha), x._h, y._h)

    def scale(self, alpha):
        call("kle_vec_scale", self._h, float(alpha))

    def pointwiseMult(self, x, y):
        call("kle_vec_pointwise_mult", self._h, x._h, y._h)

    def reciprocal(self):
        call("kle_vec_reciprocal", self._h)

    def dot(self, v):
        out = C.c_double()
        call("kle_vec_dot", self._h, v._h, C.byref(out))
        return out.value

    def norm(self, norm_type=2):
        if norm_type not in (2, None, "2", "NORM_2"):
            raise Error(56, "only the 2-norm is provided")
        out = C.c_double()
        call("kle_vec_norm2", self._h, C.byref(out))
        return out.value

    def __imul__(self, alpha):
        self.scale(alpha)
        return self

    def __add__(self, other):
        out = self.copy()
        out.axpy(1.0, other)
        return out

    def __sub__(self, other):
        out = self.copy()
        out.axpy(-1.0, other)
        return out

    def __mul__(self, other):
        out = self.copy()
        if isinstance(other, Vec):
            out.pointwiseMult(self, other)
        else:
            out.scale(other)
        return out

    __rmul__ = __mul__


class Mat:
    def __init__(self):
        self._h = None
        self._name = ""
        self._ctx = None
        self._mesh = None    # node-block matrices: (mesh, row bs, col bs)
        self._rbs = self._cbs = 1

    @classmethod
    def _wrap(cls, handle, ctx, mesh=None, rbs=1, cbs=1):
        m = cls()
        m._h, m._ctx, m._mesh, m._rbs, m._cbs = handle, ctx, mesh, rbs, cbs
        return m

    def createAIJ(self, size, bsize=None, nnz=None, csr=None, comm=None):
        (ml, mg), (nl, ng) = size
        ctx = get_ctx()
        if ml is None:
            ml = mg
        if nl is None:
            nl = ng
        if csr is not None:
            ip, ix, v = (np.ascontiguousarray(np.asarray(a, dtype=t)) for a, t in zip(csr, (np.int64, np.int64, np.float64)))
            h = C.c_void_p()
            call("kle_mat_create_aij_csr", ctx.h, int(ml), int(nl), ip, ix if len(ix) else np.zeros(1, np.int64),
                 v if len(v) else np.zeros(1), C.byref(h))
            self._h, self._ctx = h, ctx
            return self
        d = None
        if nnz is not None:
            dn = nnz[0] if isinstance(nnz, (tuple, list)) else nnz
            if dn is not None:
                d = np.ascontiguousarray(np.asarray(dn, dtype=np.int32))
        h = C.c_void_p()
        call("kle_mat_create_aij", ctx.h, int(ml), int(nl), -1 if mg is None else int(mg),
             -1 if ng is None else int(ng), d.ctypes.data if d is not None else None, None, C.byref(h))
        self._h, self._ctx = h, ctx
        self._keep = d
        return self

    def setUp(self):
        return self

    def setName(self, name):
        self._name = name

    def getName(self):
        return self._name

    def destroy(self):
        if self._h:
            call("kle_mat_destroy", self._h)
            self._h = None
        return self

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def setValues(self, rows, cols, values, addv=False):
        r, c = _i64(rows), _i64(cols)
        v = _f64(np.broadcast_to(np.asarray(values, dtype=np.float64), (len(r), len(c))))
        call("kle_mat_set_values", self._h, len(r), r, len(c), c, v, int(bool(addv)))

    def setValue(self, row, col, value, addv=False):
        self.setValues([row], [col], [[value]], addv)

    def assemble(self, assembly=None):
        call("kle_mat_assemble", self._h)

    assemblyBegin = assemble
    assemblyEnd = assemble

    def getSize(self):
        m, n = C.c_int64(), C.c_int64()
        call("kle_mat_get_size", self._h, C.byref(m), C.byref(n))
        return m.value, n.value

    def getLocalSize(self):
        m, n = C.c_int64(), C.c_int64()
        call("kle_mat_get_local_size", self._h, C.byref(m), C.byref(n))
        return m.value, n.value

    def getOwnershipRange(self):
        lo, hi = C.c_int64(), C.c_int64()
        call("kle_mat_get_ownership_range", self._h, C.byref(lo), C.byref(hi))
        return lo.value, hi.value

    @property
    def owner_range(self):
        return self.getOwnershipRange()

    def setSpmvStructured(self, on=True):
        call("kle_mat_set_spmv_structured", self._h, int(bool(on)))

    def isStructured(self):
        v = C.c_int()
        call("kle_mat_is_structured", self._h, C.byref(v))
        return bool(v.value)

    class Option:
        """petsc4py Mat.Option names understood by setOption."""
        SYMMETRIC = "SYMMETRIC"
        SPD = "SPD"

    def setOption(self, option, flag):
        """MatSetOption: SYMMETRIC / SPD switch the SpMV to symmetric (SBAIJ
        upper-triangle) storage where libkle supports it (3x3 node-block
        matrices: box lattices on one rank or z slabs, unstructured rows on
        one rank or graph partitions; kle_mat_set_symmetric, collective) and
        leave other matrices as they are, as PETSc does for options a format
        ignores."""
        if option not in (self.Option.SYMMETRIC, self.Option.SPD):
            raise Error(56, f"Mat option {option!r} not supported")
        if not flag:
            call("kle_mat_set_symmetric", self._h, 0)
            return
        try:
            call("kle_mat_set_symmetric", self._h, 1)
        except Error as e:
            if e.ierr != 56:
                raise

    def isSymmetric(self, tol=0.0):
        """MatIsSymmetric (printMatsInfo, mat_fs.py:129): |A - A^T| <= tol
        entry by entry, over every rank's rows (collective).  Symmetric
        storage holds one triangle: symmetric by construction."""
        if self.isSymmetricStorage():
            return True
        import scipy.sparse as sp
        from .runtime import COMM_WORLD as W
        ip, ix, d = self.getValuesCSR()
        lo, _ = self.getOwnershipRange()
        rows = np.repeat(np.arange(len(ip) - 1, dtype=np.int64) + lo, np.diff(ip))
        parts = W.allgather((rows, ix, d))
        r = np.concatenate([p[0] for p in parts])
        c = np.concatenate([p[1] for p in parts])
        v = np.concatenate([p[2] for p in parts])
        m, n = self.getSize()
        if m != n:
            return False
        A = sp.csr_matrix((v, (r, c)), shape=(m, n))
        diff = abs(A - A.T)
        return bool(diff.nnz == 0 or diff.max() <= tol)

    def isSymmetricStorage(self):
        v = C.c_int()
        call("kle_mat_get_symmetric", self._h, C.byref(v))
        return bool(v.value)

    def getSymmetricBricks(self):
        """The brick decomposition of the symmetric SpMV (kle_mat_get_sym_bricks),
        or None when the product runs on something else."""
        n, dims, ent, mus = C.c_int(), (C.c_int * 3)(), C.c_double(), C.c_double()
        call("kle_mat_get_sym_bricks", self._h, C.byref(n), dims, C.byref(ent), C.byref(mus))
        if n.value == 0:
            return None
        return {"bricks": n.value, "dims": list(dims), "region_entries_per_row": ent.value, "model_us": mus.value}

    def moveValues(self, shift, fresh=True):
        """Diagnostic: the symmetric storage's values `shift` bytes into a
        fresh allocation, or (fresh=False) into the allocation of the previous
        fresh=False move: same pages, other offset (kle_mat_move_values)."""
        call("kle_mat_move_values", self._h, int(shift), int(bool(fresh)))

    def setHaloOverlap(self, on=True):
        call("kle_mat_set_halo_overlap", self._h, int(bool(on)))

    def getFormat(self):
        buf = C.create_string_buffer(16)
        call("kle_mat_get_format", self._h, buf, 16)
        return buf.value.decode()

    def getInfo(self):
        """MatGetInfo subset (kle_mat_get_info)."""
        from ._lib import MatInfo
        inf = MatInfo()
        call("kle_mat_get_info", self._h, C.byref(inf))
        return {"nz_used": inf.nz_used, "nz_allocated": inf.nz_used, "nz_unneeded": 0,
                "spmv_bytes": inf.spmv_bytes, "format": self.getFormat(),
                "block_size": (inf.block_rows, inf.block_cols)}

    def spmvBytes(self):
        b = C.c_double()
        call("kle_mat_spmv_bytes", self._h, C.byref(b))
        return b.value

    def spmvKernel(self):
        """Kernel name(s) MatMult launches with the current tuning (kle_mat_spmv_kernel)."""
        buf = C.create_string_buffer(96)
        call("kle_mat_spmv_kernel", self._h, buf, 96)
        return buf.value.decode()

    def createVecLeft(self):
        if self._mesh is not None:
            return Vec.fromMesh(self._mesh, self._rbs)
        lo, hi = self.getOwnershipRange()
        return Vec().createMPI((hi - lo, self.getSize()[0]))

    def createVecRight(self):
        if self._mesh is not None:
            return Vec.fromMesh(self._mesh, self._cbs)
        (_, n), (_, nl) = self.getSize(), self.getLocalSize()
        return Vec().createMPI((nl, n))

    def createVecs(self):
        return self.createVecRight(), self.createVecLeft()

    def mult(self, x, y):
        call("kle_mat_mult", self._h, x._h, y._h)

    def timeLocalSpmv(self, x, y, reps=50):
        """Average device ms of `reps` rank-local products (kle_mat_time_local_spmv:
        the bricks and their gather, no halo either way; no PETSc counterpart) --
        a part's own kernel time, for ranks that take turns on one GPU."""
        ms = C.c_double()
        call("kle_mat_time_local_spmv", self._h, x._h, y._h, int(reps), C.byref(ms))
        return ms.value

    def multAdd(self, x, v2, v3):
        call("kle_mat_mult_add", self._h, x._h, v2._h, v3._h)

    def __mul__(self, x):
        y = self.createVecLeft()
        self.mult(x, y)
        return y

    def diagonalScale(self, L=None, R=None):
        call("kle_mat_diagonal_scale", self._h, _h(L), _h(R))

    def getDiagonal(self, result=None):
        if result is None:
            result = self.createVecLeft()
        call("kle_mat_get_diagonal", self._h, result._h)
        return result

    def duplicate(self, copy=False):
        h = C.c_void_p()
        call("kle_mat_duplicate", self._h, int(bool(copy)), C.byref(h))
        return Mat._wrap(h, self._ctx, self._mesh, self._rbs, self._cbs)

    def axpy(self, alpha, X, structure=None):
        call("kle_mat_axpy", self._h, float(alpha), X._h)

    def __add__(self, other):
        """Mat + Mat.  Same pattern: device axpy.  Different patterns: PETSc's
        MatAXPY(DIFFERENT_NONZERO_PATTERN) on the union of the two CSR
        patterns (y + 1*x where both exist), as a device AIJ matrix."""
        try:
            out = self.duplicate(copy=True)
            out.axpy(1.0, other)
            return out
        except Error:
            pass
        a, b = self.getValuesCSR(), other.getValuesCSR()
        m = len(a[0]) - 1
        rows = np.concatenate([np.repeat(np.arange(m), np.diff(a[0])), np.repeat(np.arange(m), np.diff(b[0]))])
        cols = np.concatenate([a[1], b[1]])
        vals = np.concatenate([a[2], 1.0 * b[2]])
        first = np.concatenate([np.ones(len(a[1]), bool), np.zeros(len(b[1]), bool)])
        order = np.lexsort((~first, cols, rows))  # per (row, col): Y's entry first, then X's
        rows, cols, vals = rows[order], cols[order], vals[order]
        key = np.ones(len(rows), bool)
        key[1:] = (rows[1:] != rows[:-1]) | (cols[1:] != cols[:-1])
        grp = np.cumsum(key) - 1
        out_v = np.zeros(key.sum())
        np.add.at(out_v, grp, vals)  # y + x, in that order (at most two terms)
        ip = np.zeros(m + 1, np.int64)
        np.add.at(ip, rows[key] + 1, 1)
        ip = np.cumsum(ip)
        _, n = self.getSize()
        return Mat().createAIJ(((m, m), (n, n)), csr=(ip, cols[key], out_v))

    def convert(self, mat_type="aij"):
        if mat_type not in ("aij", "seqaij", "mpiaij"):
            raise Error(56, f"convert to {mat_type}")
        h = C.c_void_p()
        call("kle_mat_convert_aij", self._h, C.byref(h))
        m, n = self.getSize()
        return Mat._wrap(h, self._ctx)

    def getRow(self, row):
        """(cols, values) of owned global row `row` (PETSc pattern, explicit zeros kept)."""
        n = C.c_int64()
        call("kle_mat_get_row", self._h, int(row), C.byref(n), None, None)
        cols = np.zeros(max(n.value, 1), dtype=np.int64)
        vals = np.zeros(max(n.value, 1))
        call("kle_mat_get_row", self._h, int(row), C.byref(n), cols.ctypes.data, vals.ctypes.data)
        return cols[:n.value], vals[:n.value]

    def getValuesCSR(self):
        """(indptr, indices, data) of the owned rows, global column ids."""
        m, nz = C.c_int64(), C.c_int64()
        call("kle_mat_get_csr_size", self._h, C.byref(m), C.byref(nz))
        ip = np.zeros(m.value + 1, dtype=np.int64)
        ix = np.zeros(max(nz.value, 1), dtype=np.int64)
        d = np.zeros(max(nz.value, 1))
        call("kle_mat_get_csr", self._h, ip, ix, d)
        return ip, ix[: nz.value], d[: nz.value]


class IS:
    """petsc4py IS on the host: the index sets of the boundary-condition code
    (boundary_conditions.py:187-250 -- unions of the boundaries' node / dof
    sets, read back with getIndices / getBlockIndices).  Indices are global
    (owned or not, as the reference's lists are); a block IS of block size bs
    holds block indices and expands to bs * b + c."""

    def __init__(self):
        self._idx = np.zeros(0, dtype=np.int64)
        self._bs = 1

    def createGeneral(self, indices, comm=None):
        self._idx = np.asarray(list(indices) if isinstance(indices, (set, frozenset)) else indices,
                               dtype=np.int64).ravel()
        self._bs = 1
        return self

    def createBlock(self, bsize, indices, comm=None):
        if int(bsize) < 1:
            raise Error(62, "IS block size must be >= 1")
        self.createGeneral(indices)
        self._bs = int(bsize)
        return self

    def createStride(self, size, first=0, step=1, comm=None):
        return self.createGeneral(np.arange(int(size), dtype=np.int64) * int(step) + int(first))

    def getBlockSize(self):
        return self._bs

    def getSize(self):
        return len(self._idx) * self._bs

    getLocalSize = getSize

    def __len__(self):
        return self.getSize()

    def getIndices(self):
        """Every index (a block IS expanded: bs * b + c, c < bs)."""
        if self._bs == 1:
            return self._idx.copy()
        return (self._idx[:, None] * self._bs + np.arange(self._bs, dtype=np.int64)).ravel()

    def getBlockIndices(self):
        """The block indices (ISGetBlockIndices; a general IS: the indices)."""
        return self._idx.copy()

    @property
    def indices(self):
        return self.getIndices()

    def union(self, iset):
        """ISExpand (petsc4py IS.union): the sorted union without duplicates,
        block size 1 unless both sets share theirs."""
        out = IS()
        if self._bs == iset._bs:
            out.createBlock(self._bs, np.union1d(self._idx, iset._idx))
        else:
            out.createGeneral(np.union1d(self.getIndices(), iset.getIndices()))
        return out

    def destroy(self):
        self._idx = np.zeros(0, dtype=np.int64)
        return self


class PC:
    def __init__(self):
        self._type = "jacobi"

    def create(self, comm=None):
        return self

    def setType(self, t):
        self._type = str(t).lower()

    def getType(self):
        return self._type

    def destroy(self):
        return self


class KSP:
    """Krylov solver on the device.  Default type cg, PC jacobi."""

    def __init__(self):
        self._h = None
        self._pc = PC()
        self._type = "cg"
        self._A = None

    def create(self, comm=None):
        # (a subclass whose __init__ does not chain up -- kle_solver.py:49-53
        # KspSolver(KSP) -- gets its defaults here, as petsc4py's does)
        for k, v in (("_pc", None), ("_type", "cg"), ("_A", None)):
            if not hasattr(self, k):
                setattr(self, k, PC() if k == "_pc" else v)
        if getattr(self, "_h", None):
            call("kle_ksp_destroy", self._h)
        ctx = get_ctx()
        h = C.c_void_p()
        call("kle_ksp_create", ctx.h, C.byref(h))
        self._h = h
        self._ctx = ctx
        return self

    def _ensure(self):
        if getattr(self, "_h", None) is None:
            self.create()

    def setType(self, t):
        self._ensure()
        self._type = str(t).lower()
        call("kle_ksp_set_type", self._h, self._type.encode())

    def getType(self):
        return self._type

    def setPC(self, pc):
        self._ensure()
        self._pc = pc
        call("kle_ksp_set_pc_type", self._h, pc.getType().encode())

    def getPC(self):
        return self._pc

    def setTolerances(self, rtol=None, atol=None, divtol=None, max_it=None):
        self._ensure()
        call("kle_ksp_set_tolerances", self._h, -1.0 if rtol is None else float(rtol),
             -1.0 if atol is None else float(atol), -1.0 if divtol is None else float(divtol),
             -1 if max_it is None else int(max_it))

    def setFixedIterations(self, n):
        self._ensure()
        call("kle_ksp_set_fixed_iterations", self._h, int(n))

    def setCGSingleReduction(self, flag=True):
        self._ensure()
        call("kle_ksp_set_cg_single_reduction", self._h, int(bool(flag)))

    def setGMRESRestart(self, m):
        self._ensure()
        call("kle_ksp_set_gmres_restart", self._h, int(m))

    def setFromOptions(self):
        self._ensure()
        o = Options()
        if "ksp_type" in o:
            self.setType(o["ksp_type"])
        if "pc_type" in o:
            pc = PC()
            pc.setType(o["pc_type"])
            self.setPC(pc)
        self.setTolerances(o.getReal("ksp_rtol"), o.getReal("ksp_atol"), o.getReal("ksp_divtol"),
                           o.getInt("ksp_max_it"))
        if "ksp_cg_single_reduction" in o:
            self.setCGSingleReduction(o.getBool("ksp_cg_single_reduction", True))
        if "ksp_gmres_restart" in o:
            self.setGMRESRestart(o.getInt("ksp_gmres_restart"))

    def setOperators(self, A, P=None):
        self._ensure()
        self._A = A
        call("kle_ksp_set_operators", self._h, A._h)

    def setUp(self):
        self._ensure()
        call("kle_ksp_set_up", self._h)

    def solve(self, b, x):
        call("kle_ksp_solve", self._h, b._h, x._h)

    def solveContinue(self, b, x, n):
        """n more iterations of the preceding fixed-iteration solve on (b, x),
        continuing its recurrence without a restart (benchmarks)."""
        call("kle_ksp_continue", self._h, b._h, x._h, int(n))

    def __call__(self, b, x=None):
        if x is None:
            x = self._A.createVecRight()
        self.solve(b, x)
        return x

    def getIterationNumber(self):
        v = C.c_int()
        call("kle_ksp_get_iteration_number", self._h, C.byref(v))
        return v.value

    def getProductKernel(self):
        """Kernel name(s) of the last solve call's products (kle_ksp_get_product_kernel):
        the matrix's (Mat.spmvKernel), or the bricks alone where the CG update
        gathers the split product itself."""
        buf = C.create_string_buffer(160)
        call("kle_ksp_get_product_kernel", self._h, buf, 160)
        return buf.value.decode()

    def getProductBytes(self):
        """Algorithmic bytes of one of those products (kle_ksp_get_product_bytes)."""
        v = C.c_double()
        call("kle_ksp_get_product_bytes", self._h, C.byref(v))
        return v.value

    its = property(getIterationNumber)

    def getResidualNorm(self):
        v = C.c_double()
        call("kle_ksp_get_residual_norm", self._h, C.byref(v))
        return v.value

    def getConvergedReason(self):
        v = C.c_int()
        call("kle_ksp_get_converged_reason", self._h, C.byref(v))
        return v.value

    def getTrueRelativeResidual(self):
        v = C.c_double()
        call("kle_ksp_get_true_relative_residual", self._h, C.byref(v))
        return v.value

    def setCorrections(self, n):
        """Correction solves when the true residual misses rtol (kle.h
        kle_ksp_set_corrections; default 2, 0 = PETSc's plain recursive stop)."""
        call("kle_ksp_set_corrections", self._h, int(n))

    def getCorrectionIterations(self):
        """Iterations of the last solve's correction solves (0: none ran);
        not part of getIterationNumber (PETSc's count of the main solve)."""
        v = C.c_int()
        call("kle_ksp_get_correction_iterations", self._h, C.byref(v))
        return v.value

    def getCorrectionReason(self):
        """Converged reason of the last correction solve (0: none ran); the
        KSP's own getConvergedReason stays the main solve's."""
        v = C.c_int()
        call("kle_ksp_get_correction_reason", self._h, C.byref(v))
        return v.value

    def destroy(self):
        if getattr(self, "_h", None):
            call("kle_ksp_destroy", self._h)
            self._h = None
        return self

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


__all__ = ["Mat", "Vec", "KSP", "PC", "IS", "Options", "Error", "COMM_WORLD", "INSERT_VALUES", "ADD_VALUES"]
