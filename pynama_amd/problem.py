"""The caller of the KLE path: the vorticity right-hand side.

Host mirror of the part of the reference's BaseProblem / BaseProblemTest
(cases/base_problem.py:17-420) that drives the KLE solve and the operator
chain: setUpDomain, readMaterialData, setUpSolver, setUpInitialConditions,
evalRHS, computeVtensV, generateExactVecs, getKLEError, getConvective and
getDiffusive.  Same names, arguments and in-place semantics; everything
runs on the device through libkle (the KLE solve, the Curl / SrT / DivSrT
SpMVs, the v v^T tensor and the BLAS-1 updates).  Output (Paraviewer,
XDMF over HDF5, viewer.py) is written when the case names a "save-dir"; the
reference always writes it (base_problem.py:40-43,65-70,93-101).
"""
import numpy as np

from . import fields
from ._lib import call
from .domain import Domain
from .matrices import MatFS, MatNS
from .solver import KleSolver


class BaseProblem:
    def __init__(self, config, **kwargs):
        self.config = config
        self.opts = kwargs
        self.case = kwargs.get("case", "uniform")
        self.caseName = config.get("name")
        self.readMaterialData()
        ts = config.get("time-solver") or {}
        self.initTime = float(kwargs.get("initTime", ts.get("start-time", 0.0)))
        self.ts = None
        if "time-solver" in config:
            self.setUpTimeSolver()

    def setUpTimeSolver(self):
        """base_problem.py:71-80: TS rk/5bs over [start-time, end-time]."""
        from .ts import TsSolver
        options = self.config.get("time-solver")
        self.ts = TsSolver()
        self.ts.setUpTimes(options["start-time"], options["end-time"], options["max-steps"])
        self.ts.initSolver(self.evalRHS, self.convergedStepFunction)

    def convergedStepFunction(self, ts):
        """Post-step hook (base_problem.py:93-101): velocity and vorticity of
        the step to HDF5 + the case's XDMF (when a viewer is set up)."""
        self.lastStep = (ts.step_number, ts.time, ts.getTimeStep())
        if getattr(self, "viewer", None) is not None:
            vel = self.solverKLE.getSolution()
            vort = ts.getSolution()
            self.viewer.saveData(ts.step_number, ts.time, vel, vort)
            self.viewer.writeXmf(self.caseName)

    def startSolver(self):
        """timeSolving (run_case.py:153-163): integrate the vorticity in place."""
        self.ts.solve(self.vort)

    def setUp(self):
        self.setUpDomain()
        self.viewer = None
        if self.config.get("save-dir"):
            self.setUpViewer()
            self.createMesh()

    def setUpViewer(self):
        from .viewer import Paraviewer
        self.viewer = Paraviewer()

    def createMesh(self, saveMesh=True):
        """base_problem.py:65-70: configure the viewer, save the node coordinates."""
        self.viewer.configure(self.dim, self.config.get("save-dir"))
        if saveMesh:
            self.viewer.saveMesh(self.dom.getFullCoordArray())

    def setUpDomain(self):
        self.dom = Domain()
        self.dom.configure(self.config)
        self.dom.setOptions(**{k: v for k, v in self.opts.items() if k in ("ngl", "nelem", "lower", "upper")})
        self.dom.setUp()
        self.dim = self.dom.getDimension()
        self.dim_w = 1 if self.dim == 2 else 3
        self.dim_s = 3 if self.dim == 2 else 6

    def readMaterialData(self):
        materialData = self.config.get("material-properties")
        self.rho = materialData["rho"]
        self.mu = materialData["mu"]
        self.nu = self.mu / self.rho

    def setUpSolver(self):
        """base_problem.py:156-179 (free-slip / Dirichlet boundaries)."""
        bcType = self.dom.getBoundaryType()
        if bcType == "FS":
            mat = MatFS()
        elif bcType == "NS":
            mat = MatNS()
        else:
            raise Exception("FSNS Mat not implemented")
        mat.setDomain(self.dom)
        mat.build()
        self.mat = mat
        self.solverKLE = KleSolver()
        self.solverKLE.setMat(mat)
        self.solverKLE.setUp()
        self.operator = mat.getOperators()
        self._VtensV = self.operator.SrT.createVecLeft()
        self._Aux1 = self._VtensV.duplicate()
        assert "initial-conditions" in self.config, "Initial conditions not defined"
        self.setUpInitialConditions()

    def setUpInitialConditions(self):
        """base_problem.py:181-222."""
        vort = self.operator.Curl.createVecLeft()
        vort.setName("vorticity")
        vel = self.solverKLE.getSolution()
        ic = self.config["initial-conditions"]
        if "custom-func" in ic:
            f = fields.get(ic["custom-func"]["name"])
            alpha = f.alpha(self.nu, self.initTime)
            coords = self.dom.getFullCoordArray()
            vort.setArray(np.asarray(f.vorticity(coords, alpha), dtype=np.float64).ravel())
            vel.setArray(np.asarray(f.velocity(coords, alpha), dtype=np.float64).ravel())
        elif "velocity" in ic and "vorticity" not in ic:
            nodes = self.dom.getAllNodes()
            vel.setArray(np.tile(np.asarray(ic["velocity"], dtype=np.float64), len(nodes)))
        self.vort = vort

    def evalRHS(self, ts, t, vort, f):
        """Evaluate the KLE right-hand side (base_problem.py:111-136):
        f = Curl( DivSrT( 2 mu SrT u - rho u u^T ) / rho ), u = KLE(vort).
        As in the reference, the KLE solve uses self.vort (with its boundary
        values refreshed), not the stage vector `vort`."""
        self.dom.applyBoundaryConditions(self.vort, "vorticity", t, self.nu)
        vel = self.solverKLE.getSolution()
        self.dom.applyBoundaryConditions(vel, "velocity", t, self.nu)
        if self.solverKLE.isNS():
            self.solverKLE.solveFS(self.vort)
            velFS = self.solverKLE.getFreeSlipSolution()
            self.dom.applyBoundaryConditionsNS(velFS, "velocity", t, self.nu)
            self.operator.Curl.mult(velFS, self.vort)
        self.solverKLE.solve(self.vort)
        self.computeVtensV(vel)
        self.operator.SrT.mult(vel, self._Aux1)
        self._Aux1 *= (2.0 * self.mu)
        self._Aux1.axpy(-1.0 * self.rho, self._VtensV)
        rhs = vel.duplicate()
        self.operator.DivSrT.mult(self._Aux1, rhs)
        rhs.scale(1 / self.rho)
        self.operator.Curl.mult(rhs, f)

    def computeVtensV(self, vec):
        """base_problem.py:138-154 as one device kernel."""
        call("kle_vec_tensor_square", vec._h, self.dim, self._VtensV._h)


class BaseProblemTest(BaseProblem):
    """Known-answer helpers of the reference's BaseProblemTest (base_problem.py:232-420)."""

    def generateExactVecs(self, vel=None, vort=None, time=None):
        exactVel = self.mat.K.createVecRight()
        exactVort = self.mat.Rw.createVecRight()
        n = len(self.dom.getAllNodes())
        if vel and vort:
            arrVel, arrVort = np.tile(vel, n), np.tile(vort, n)
        else:
            f = fields.get(self.config["tests"]["custom-func"]["name"])
            alpha = f.alpha(self.nu, time)
            coords = self.dom.getFullCoordArray()
            arrVel, arrVort = f.velocity(coords, alpha), f.vorticity(coords, alpha)
        exactVort.setArray(np.asarray(arrVort, dtype=np.float64).ravel())
        exactVel.setArray(np.asarray(arrVel, dtype=np.float64).ravel())
        return exactVel, exactVort

    def getKLEError(self, viscousTimes=None, startTime=0.0, endTime=1.0, steps=10):
        if viscousTimes is None:
            viscousTimes = np.arange(startTime, endTime, (endTime - startTime) / steps)
        errors = []
        for time in [(tau ** 2) / (4 * self.nu) for tau in viscousTimes]:
            exactVel, exactVort = self.generateExactVecs(time=time)
            self.dom.applyBoundaryConditions(self.vort, "vorticity", time, self.nu)
            vel = self.solverKLE.getSolution()
            self.dom.applyBoundaryConditions(vel, "velocity", time, self.nu)
            self.solverKLE.solve(exactVort)
            errors.append((exactVel - vel).norm())
        return errors

    def getConvective(self, exactVel, exactConv):
        convective = exactConv.copy()
        vel = self.solverKLE.getSolution()
        self.computeVtensV(vel)
        aux = vel.copy()
        self.operator.DivSrT.mult(self._VtensV, aux)
        self.operator.Curl.mult(aux, convective)
        return convective

    def getDiffusive(self, exactVel, exactDiff):
        diffusive = exactDiff.copy()
        vel = self.solverKLE.getSolution()
        self.operator.SrT.mult(exactVel, self._Aux1)
        aux = vel.copy()
        self._Aux1 *= (2.0 * self.mu)
        self.operator.DivSrT.mult(self._Aux1, aux)
        aux.scale(1 / self.rho)
        self.operator.Curl.mult(aux, diffusive)
        return diffusive
