"""KleSolver / KspSolver: the KLE velocity solve on the device.

Mirror of the reference's solver/kle_solver.py:5-64 (same methods and
behaviour): ``solve(vort)`` forms b = Rw*vort + Krhs*vel (vel carries the
Dirichlet values, written beforehand by applyBoundaryConditions) and solves
K vel = b in place.  The reference's KSP is gmres + PC lu, overridden to
preonly + lu by the makefile (makefile:7); K is SPD, so the device default is
CG + Jacobi at rtol 1e-10 (the north-star tolerance), overridable with the
usual -ksp_type / -pc_type / -ksp_rtol / -ksp_max_it options.  The makefile's
-ksp_type preonly -pc_type lu is a dense device LU (rocSOLVER getrf/getrs) for
sequential systems up to 40k unknowns (config 1, the unit cases); beyond that,
or on several ranks, it raises like PETSc without a parallel direct solver --
there is no CPU fallback.
"""
from .petsc import KSP, PC, Options

DEFAULT_RTOL = 1e-10


class KspSolver(KSP):
    def createSolver(self, mat):
        self.create()
        self.setType("cg")
        pc = PC().create()
        pc.setType("jacobi")
        self.setPC(pc)
        self.setTolerances(rtol=DEFAULT_RTOL, atol=0.0, max_it=100000)
        self.setFromOptions()
        self.setOperators(mat)
        self.setUp()


class KleSolver:
    def __init__(self):
        self.mat = None
        self._b = None

    def setMat(self, mat):
        self.mat = mat

    def setUp(self):
        K = self.mat.K
        self.solver = KspSolver()
        self.solver.createSolver(K)
        self.__vel = K.createVecRight()
        self.__vel.setName("velocity")
        self._b = K.createVecLeft()
        self._wtmp = K.createVecLeft()
        self.__isNS = False
        if self.mat.bcType == "NS":
            # solverFS on K + Kfs (kle_solver.py:22-28); MatNS assembles the sum
            # on the device with PETSc's union pattern and rounding
            self.solverFS = KspSolver()
            self.solverFS.createSolver(self.mat.getKplusKfs())
            self.__velFS = K.createVecRight()
            self.__velFS.setName("free-slip")
            self._bfs = K.createVecLeft()
            self.__isNS = True

    def isNS(self):
        return self.__isNS

    def rhs(self, vort, vec=None):
        """b = Rw * vort + Krhs * vel (kle_solver.py:35) without temporaries."""
        vel = self.__vel if vec is None else vec
        self.mat.Rw.mult(vort, self._b)
        self.mat.Krhs.mult(vel, self._wtmp)
        self._b.axpy(1.0, self._wtmp)
        return self._b

    def solve(self, vort, vec=None):
        vel = self.__vel if vec is None else vec
        b = self.rhs(vort, vel)
        self.solver(b, vel)

    def getSolution(self):
        return self.__vel

    def getKSP(self):
        return self.solver

    def rhsFS(self, vort):
        """b = Rw * vort + Rwfs * vort + Krhsfs * vel (kle_solver.py:39-41)."""
        self.mat.Rw.mult(vort, self._bfs)
        self.mat.Rwfs.mult(vort, self._wtmp)
        self._bfs.axpy(1.0, self._wtmp)
        self.mat.Krhsfs.mult(self.__vel, self._wtmp)
        self._bfs.axpy(1.0, self._wtmp)
        return self._bfs

    def solveFS(self, vort):
        self.solverFS(self.rhsFS(vort), self.__velFS)

    def getFreeSlipSolution(self):
        return self.__velFS
