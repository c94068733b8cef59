"""MatFS: device assembly of the KLE matrices.

Mirror of the reference's MatFS (matrices/mat_fs.py:5-209): same public
surface -- setDomain, build, K, Krhs, Rw, Rd, getOperators, bcType -- but the
per-cell Python loop of buildFS (mat_fs.py:150-192), which calls
Spectral.getElemKLEMatrices and MatSetValues once per element, is replaced by
one batch device assembly (libkle kle_assemble_kle): element matrices on the
GPU, deterministic gather into node-block CSR, PETSc pattern and ADD order.
"""
import ctypes as C

import numpy as np

from ._lib import Error, call
from .petsc import Mat
from .runtime import get_ctx


class MatFS:
    bcType = "FS"

    def __init__(self):
        self.kle = []
        self.K = self.Krhs = self.Rw = self.Rd = None
        self.operator = None

    def setDomain(self, dom):
        self.dom = dom

    def build(self, buildKLE=True, buildOperators=True):
        if self.dom.getBoundaryType() != "FS":
            raise Error(56, "MatFS needs free-slip (Dirichlet) boundaries")
        if buildKLE:
            self.buildFS()
        if buildOperators:
            self.buildOperators()

    def buildFS(self):
        ctx = get_ctx()
        mesh = self.dom.getMesh()
        hK, hKr, hRw = C.c_void_p(), C.c_void_p(), C.c_void_p()
        call("kle_assemble_kle", ctx.h, mesh._h, C.byref(hK), C.byref(hKr), C.byref(hRw))
        dim, dim_w, _ = self.dom.getDimensions()
        self.K = Mat._wrap(hK, ctx, mesh, dim, dim)
        self.Krhs = Mat._wrap(hKr, ctx, mesh, dim, dim)
        self.Rw = Mat._wrap(hRw, ctx, mesh, dim, dim_w)
        for m, n in ((self.K, "K"), (self.Krhs, "Krhs"), (self.Rw, "Rw")):
            m.setName(n)
        # Rd is preallocated but never filled in free slip (preAlloc_Rd_Rw,
        # mat_fs.py:54-94; buildFS adds no Rd entries): after assembleAll it is
        # an assembled [dim N x N] matrix without stored entries
        self.Rd = self._empty(dim)
        self.kle = [self.K, self.Krhs, self.Rw, self.Rd]

    def _empty(self, dim, name="Rd"):
        lo, hi = self.dom.getNodesRange()
        N = self.dom.getMesh().N
        A = Mat().createAIJ((((hi - lo) * dim, N * dim), (hi - lo, N)),
                            nnz=(np.zeros((hi - lo) * dim, dtype=np.int32), None))
        A.assemble()
        A.setName(name)
        return A

    def buildOperators(self):
        """Curl / SrT / DivSrT on the device (mat_fs.py:194-201)."""
        self.operator = Operators()
        self.operator.setDimensions(self.dom.getDimensions())
        self.operator.build(self.dom.getMesh())

    def getOperators(self):
        return self.operator

    def assembleAll(self):
        pass


class MatNS(MatFS):
    """Mirror of the reference's MatNS (matrices/mat_ns.py:5-161): no-slip walls.
    K, Krhs, Rw fix the no-slip nodes; Kfs, Krhsfs, Rwfs free their tangential
    DoFs for the free-slip pre-solve (solveFS).  One device pass
    (kle_assemble_ns) with PETSc's DoF-level patterns; K + Kfs, the operator of
    KleSolver.solverFS, is assembled directly (getKplusKfs)."""
    bcType = "NS"

    def __init__(self):
        super().__init__()
        self.Kfs = self.Krhsfs = self.Rwfs = self.Rdfs = None
        self._Ksum = None

    def build(self, buildKLE=True, buildOperators=True):
        if self.dom.getBoundaryType() != "NS":
            raise Error(56, "MatNS needs no-slip boundaries")
        if buildKLE:
            self.buildNS()
        if buildOperators:
            self.buildOperators()

    def buildNS(self):
        ctx = get_ctx()
        mesh = self.dom.getMesh()
        h = [C.c_void_p() for _ in range(9)]
        call("kle_assemble_ns", ctx.h, mesh._h, *[C.byref(x) for x in h])
        dim, dim_w, _ = self.dom.getDimensions()
        shapes = [(dim, dim), (dim, dim), (dim, dim_w), (dim, 1), (dim, dim), (dim, dim), (dim, dim_w), (dim, 1),
                  (dim, dim)]
        mats = [Mat._wrap(x, ctx, mesh, r, c) for x, (r, c) in zip(h, shapes)]
        (self.K, self.Krhs, self.Rw, self.Rd, self.Kfs, self.Krhsfs, self.Rwfs, self.Rdfs, self._Ksum) = mats
        for m, n in zip(mats, ("K", "Krhs", "Rw", "Rd", "Kfs", "Krhsfs", "Rwfs", "Rdfs", "K+Kfs")):
            m.setName(n)
        self.kle = mats[:8]

    def getKplusKfs(self):
        return self._Ksum


class Operators:
    """Mirror of the reference's Operators (mat_fs.py:211-271): the collocation
    operators Curl [dim_w N x dim N], SrT [dim_s N x dim N] and DivSrT
    [dim N x dim_s N], each left-scaled by the inverse lumped nodal weight.
    Assembled in one device pass (libkle kle_assemble_operators) instead of
    the per-cell setValues loop; same pattern (explicit zeros kept) and the
    same ascending-cell ADD order."""

    def __init__(self):
        self.Curl = self.SrT = self.DivSrT = None

    def setDimensions(self, dims):
        self.dim, self.dim_w, self.dim_s = dims

    def build(self, mesh):
        ctx = get_ctx()
        hc, hs, hd = C.c_void_p(), C.c_void_p(), C.c_void_p()
        call("kle_assemble_operators", ctx.h, mesh._h, C.byref(hc), C.byref(hs), C.byref(hd))
        self.Curl = Mat._wrap(hc, ctx, mesh, self.dim_w, self.dim)
        self.SrT = Mat._wrap(hs, ctx, mesh, self.dim_s, self.dim)
        self.DivSrT = Mat._wrap(hd, ctx, mesh, self.dim, self.dim_s)
        for m, n in ((self.Curl, "Curl"), (self.SrT, "SrT"), (self.DivSrT, "DivSrT")):
            m.setName(n)

    def assembleAll(self):
        pass  # assembled (and weight-scaled) on the device by build()
