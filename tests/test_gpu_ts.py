"""GPU checks of the Runge-Kutta integrator (pynama_amd.ts):
order of accuracy on a linear test ODE held in device vectors, the adaptive
controller meeting its tolerance, and the full vorticity solver
(BaseProblem.evalRHS as the RHS, KLE solve per stage) reproducing the decay
of a 2-D Taylor-Green vortex.  Parity with PETSc's TSRK is unpinned (no
PETSc here); these are known-answer tests."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _linear(pa, name, T, nsteps=None, tol=None):
    from pynama_amd.petsc import Vec
    from pynama_amd.ts import TsSolver
    n = 1000
    lam_h = -np.linspace(0.5, 2.0, n)
    lam = Vec().createMPI((n, n))
    lam.setArray(lam_h)
    u = Vec().createMPI((n, n))
    u0 = np.cos(np.arange(n) * 0.01) + 1.5
    u.setArray(u0)

    def rhs(ts, t, Y, F):
        F.pointwiseMult(lam, Y)

    ts = TsSolver()
    ts.setRKType(name)
    ts.setUpTimes(0.0, T, 100000)
    ts.setRHSFunction(rhs)
    if nsteps:
        ts.setAdaptType("none")
        ts.setTimeStep(T / nsteps)
    else:
        ts.setTolerances(rtol=tol, atol=tol)
        ts.setTimeStep(0.01)
    ts.solve(u)
    err = np.abs(u.getArray() - u0 * np.exp(lam_h * T)).max()
    return err, ts


@pytest.mark.parametrize("name,order", [("3", 3), ("4", 4), ("5f", 5), ("5bs", 5)])
def test_rk_order(pa, name, order):
    e1, ts1 = _linear(pa, name, 2.0, nsteps=16)
    e2, ts2 = _linear(pa, name, 2.0, nsteps=32)
    assert ts1.getStepNumber() == 16 and ts2.getStepNumber() == 32
    assert abs(ts2.getTime() - 2.0) < 1e-14
    rate = np.log2(e1 / e2)
    assert order - 0.4 < rate < order + 1.0, (name, e1, e2, rate)


@pytest.mark.parametrize("name", ["3", "5f", "5bs"])
def test_rk_adaptive_meets_tolerance(pa, name):
    err, ts = _linear(pa, name, 3.0, tol=1e-7)
    assert abs(ts.getTime() - 3.0) < 1e-12  # MATCHSTEP lands on the final time
    assert err < 1e-5
    assert ts.getStepNumber() < 400


def test_taylor_green_decay(pa):
    """BaseProblem + TsSolver (run_case.py:159 timeSolving): the vorticity of a
    2-D Taylor-Green vortex decays as exp(-2 nu (2 pi)^2 t) (taylor_green.py)."""
    from pynama_amd.ts import TsSolver
    cfg = {"name": "tg", "material-properties": {"rho": 0.5, "mu": 0.01},
           "domain": {"ngl": 5, "box-mesh": {"nelem": [8, 8], "lower": [0, 0], "upper": [1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green"}},
           "initial-conditions": {"custom-func": {"name": "taylor_green"}},
           "time-solver": {"start-time": 0.0, "end-time": 0.3, "max-steps": 200}}
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    prob.setUpSolver()
    prob.solverKLE.getKSP().setTolerances(rtol=1e-12)
    ts = TsSolver()
    ts.setUpTimes(0.0, 0.3, 200)
    ts.initSolver(prob.evalRHS, None)
    ts.setAdaptType("none")  # the stage-blind RHS makes the embedded estimate ~0 (see ts.py)
    ts.setTimeStep(0.01)
    w0 = prob.vort.getArray().copy()
    ts.solve(prob.vort)
    assert abs(ts.getTime() - 0.3) < 1e-12
    f = pa.fields.get("taylor_green")
    decay = f.alpha(prob.nu, 0.3) / f.alpha(prob.nu, 0.0)
    w = prob.vort.getArray()
    rel = np.linalg.norm(w - decay * w0) / np.linalg.norm(decay * w0)
    assert rel < 2e-2, (rel, ts.getStepNumber())
    assert np.linalg.norm(w) < np.linalg.norm(w0)


def test_time_steps_are_written_for_paraview(pa, tmp_path):
    """convergedStepFunction (base_problem.py:93-101) with a "save-dir": the
    mesh and every step's velocity / vorticity land in HDF5 (or raw binary)
    behind the case's XDMF, on an unstructured Gmsh mesh."""
    import os
    import xml.etree.ElementTree as ET
    from pynama_amd.viewer import _find_hdf5
    msh = os.path.join(os.path.dirname(__file__), "golden", "test.msh")
    out = tmp_path / "run"
    cfg = {"name": "tg-gmsh", "material-properties": {"rho": 0.5, "mu": 0.01}, "save-dir": str(out),
           "domain": {"ngl": 3, "gmsh-file": msh},
           "boundary-conditions": {"custom-func": {"name": "taylor_green"}},
           "initial-conditions": {"custom-func": {"name": "taylor_green"}},
           "time-solver": {"start-time": 0.0, "end-time": 0.02, "max-steps": 2}}
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    prob.setUpSolver()
    prob.setUpInitialConditions()
    prob.ts.setAdaptType("none")
    prob.ts.setTimeStep(0.01)
    prob.startSolver()
    assert prob.ts.getStepNumber() == 2
    root = ET.parse(out / "tg-gmsh.xmf").getroot()
    grids = root.find("Domain").find("Grid").findall("Grid")
    assert len(grids) == 2
    vel = prob.solverKLE.getSolution().getArray()
    h5 = _find_hdf5()
    if h5 is not None:
        np.testing.assert_array_equal(h5.read(str(out / "vec-data-00002.h5"), "/fields/velocity"), vel)
        np.testing.assert_array_equal(h5.read(str(out / "vec-data-00002.h5"), "/fields/vorticity"),
                                      prob.vort.getArray())
        np.testing.assert_array_equal(h5.read(str(out / "mesh.h5"), "/fields/mesh"),
                                      prob.dom.getFullCoordArray().ravel())
