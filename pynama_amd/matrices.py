"""MatFS: device assembly of the KLE matrices.

Mirror of the reference's MatFS (matrices/mat_fs.py:5-209): same public
surface -- setDomain, build, K, Krhs, Rw, Rd, getOperators, bcType -- but the
per-cell Python loop of buildFS (mat_fs.py:150-192), which calls
Spectral.getElemKLEMatrices and MatSetValues once per element, is replaced by
one batch device assembly (libkle kle_assemble_kle): element matrices on the
GPU, deterministic gather into node-block CSR, PETSc pattern and ADD order.
"""
import ctypes as C

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

    def build(self, buildKLE=True, buildOperators=False):
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
        self.kle = [self.K, self.Krhs, self.Rw]

    def buildOperators(self):
        # Curl / SrT / DivSrT (mat_fs.py:194-271) are the next row of the
        # scope table; not provided in this build.
        raise Error(56, "Operators (Curl/SrT/DivSrT) are not provided yet")

    def getOperators(self):
        return self.operator

    def assembleAll(self):
        pass
