"""GPU parity of the Operators row: Curl / SrT / DivSrT
assembled on the device vs the golden matrices produced by the reference's
own Operators (mat_fs.py:194-271) and vs the CPU oracle; SpMV with them; and
size-independent properties at larger sizes (GLL collocation differentiates
polynomials of degree <= p exactly, so the assembled operators reproduce
analytic curl / strain rate / divergence at the nodes).

Tolerances (fp64): pattern bit-exact; values <= 1e-12 * max|ref| (J^-1 and
Lagrange-derivative tables are computed with different but equivalent
formulas); SpMV <= 1e-13 relative 2-norm; polynomial identities <= 1e-9
relative (derivatives amplify rounding by 1/h)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
OPS = ("Curl", "SrT", "DivSrT")


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _domain(pa, dim, nelem, ngl, lower=None, upper=None):
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": list(nelem), "lower": lower or [0.0] * dim,
                                                "upper": upper or [1.0] * dim}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d" if dim == 3 else "taylor_green"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    return dom


def _ops(pa, dom):
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildKLE=False, buildOperators=True)
    return mat.getOperators()


@pytest.mark.parametrize("case", ["uniform2d", "tg2d_small", "tg3d", "cavity2d"])
def test_operators_match_golden(pa, case):
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim = int(g["dim"])
    dom = _domain(pa, dim, list(g["nelem"]), int(g["ngl"]), list(g["lower"]), list(g["upper"]))
    op = _ops(pa, dom)
    rng = np.random.default_rng(5)
    for nm in OPS:
        A = getattr(op, nm)
        ip, ix, d = A.getValuesCSR()
        np.testing.assert_array_equal(ip, g[nm + "_indptr"])
        np.testing.assert_array_equal(ix, g[nm + "_indices"])
        ref = g[nm + "_data"]
        assert np.abs(d - ref).max() <= 1e-12 * np.abs(ref).max(), nm
        R = O.CSR.from_arrays(g[nm + "_indptr"], g[nm + "_indices"], ref, int(g[nm + "_shape"][1]))
        x = A.createVecRight()
        xa = rng.uniform(-1, 1, x.getLocalSize())
        x.setArray(xa)
        y = (A * x).getArray()
        yr = R.mult(xa)
        assert np.linalg.norm(y - yr) <= 1e-13 * np.linalg.norm(yr), nm


def test_operators_match_oracle_3d_p4(pa):
    dom = _domain(pa, 3, [3, 2, 2], 5, [0.1, 0.0, -0.2], [0.7, 0.5, 0.4])
    op = _ops(pa, dom)
    om = O.BoxMesh(3, [3, 2, 2], [0.1, 0.0, -0.2], [0.7, 0.5, 0.4], 5)
    refs = dict(zip(OPS, om.assemble_ops()[:3]))
    for nm in OPS:
        ip, ix, d = getattr(op, nm).getValuesCSR()
        R = refs[nm]
        np.testing.assert_array_equal(ip, R.indptr)
        np.testing.assert_array_equal(ix, R.indices)
        assert np.abs(d - R.data).max() <= 1e-12 * np.abs(R.data).max(), nm


def test_operator_polynomial_identities(pa):
    """Degree-<=p fields: Curl u, SrT u and DivSrT s are exact at the nodes."""
    dim, nelem, ngl = 3, [6, 5, 4], 5
    dom = _domain(pa, dim, nelem, ngl)
    op = _ops(pa, dom)
    X = dom.getFullCoordArray().reshape(-1, 3)
    x, y, z = X[:, 0], X[:, 1], X[:, 2]
    u = np.stack([y * y * z, x * z * z, x * y * x], 1)          # degree <= 3
    curl = np.stack([x * x - 2 * x * z, y * y - 2 * x * y, z * z - 2 * y * z], 1)
    # strain rate 0.5 (grad u + grad u^T): xx, xy, yy, yz, zz, zx
    ux = [np.zeros_like(x), z * z, 2 * x * y]
    uy = [2 * y * z, np.zeros_like(x), x * x]
    uz = [y * y, 2 * x * z, np.zeros_like(x)]
    # grad[i][j] = d u_i / d x_j
    gr = [[ux[0] * 0, 2 * y * z, y * y], [z * z, 0 * x, 2 * x * z], [2 * x * y, x * x, 0 * x]]
    S = np.stack([gr[0][0], 0.5 * (gr[0][1] + gr[1][0]), gr[1][1], 0.5 * (gr[1][2] + gr[2][1]), gr[2][2],
                  0.5 * (gr[2][0] + gr[0][2])], 1)
    v = op.Curl.createVecRight()
    v.setArray(u.ravel())
    w = (op.Curl * v).getArray().reshape(-1, 3)
    assert np.abs(w - curl).max() <= 1e-9 * np.abs(curl).max()
    s = (op.SrT * v).getArray().reshape(-1, 6)
    assert np.abs(s - S).max() <= 1e-9 * np.abs(S).max()
    # div of a polynomial symmetric tensor: sigma = (x^2, xy, y^2, yz, z^2, zx)
    sig = np.stack([x * x, x * y, y * y, y * z, z * z, z * x], 1)
    divs = np.stack([2 * x + x + x, y + 2 * y + y, z + 2 * z + z], 1)  # d_j sigma_ij
    sv = op.DivSrT.createVecRight()
    sv.setArray(sig.ravel())
    d = (op.DivSrT * sv).getArray().reshape(-1, 3)
    assert np.abs(d - divs).max() <= 1e-9 * np.abs(divs).max()
    del ux, uy, uz


def _problem(pa, g, case):
    dim = int(g["dim"])
    bc = ({"uniform": {"velocity": [4, 0]}} if case == "uniform2d" else
          {"custom-func": {"name": "taylor_green3d" if dim == 3 else "taylor_green"}})
    cfg = {"name": case, "material-properties": {"rho": float(g["rho"]), "mu": float(g["mu"])},
           "domain": {"ngl": int(g["ngl"]), "box-mesh": {"nelem": [int(v) for v in g["nelem"]],
                                                        "lower": list(g["lower"]), "upper": list(g["upper"])}},
           "boundary-conditions": bc, "initial-conditions": {"velocity": [4, 0]} if case == "uniform2d" else bc}
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    prob.setUpSolver()
    return prob


@pytest.mark.parametrize("case", ["uniform2d", "tg2d_small", "tg3d"])
def test_eval_rhs_matches_reference(pa, case):
    """BaseProblem.evalRHS (base_problem.py:111-154) against the reference's
    own evalRHS output: (1) the operator chain from the reference's KLE
    velocity, tight; (2) the whole call incl. the KLE solve (CG at rtol 1e-13
    vs the reference's direct solve)."""
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    prob = _problem(pa, g, case)
    scale = max(1.0, np.abs(g["rhs_f"]).max())
    # (1) chain only
    vel = prob.solverKLE.getSolution().duplicate()
    vel.setArray(g["rhs_vel"])
    prob.computeVtensV(vel)
    np.testing.assert_array_equal(prob._VtensV.getArray(), g["rhs_VtensV"])
    prob.operator.SrT.mult(vel, prob._Aux1)
    prob._Aux1 *= (2.0 * prob.mu)
    prob._Aux1.axpy(-1.0 * prob.rho, prob._VtensV)
    assert np.abs(prob._Aux1.getArray() - g["rhs_Aux1"]).max() <= 1e-12 * max(1.0, np.abs(g["rhs_Aux1"]).max())
    rhs = vel.duplicate()
    prob.operator.DivSrT.mult(prob._Aux1, rhs)
    rhs.scale(1 / prob.rho)
    f = prob.operator.Curl.createVecLeft()
    prob.operator.Curl.mult(rhs, f)
    assert np.abs(f.getArray() - g["rhs_f"]).max() <= 1e-10 * scale
    # (2) the full call
    prob.solverKLE.getKSP().setTolerances(rtol=1e-13)
    prob.vort.setArray(g["rhs_vort_in"])
    f2 = prob.operator.Curl.createVecLeft()
    prob.evalRHS(None, float(g["rhs_t"]), prob.vort, f2)
    np.testing.assert_allclose(prob.vort.getArray(), g["rhs_vort_bc"], rtol=0, atol=1e-14)
    u = prob.solverKLE.getSolution().getArray()
    assert np.linalg.norm(u - g["rhs_vel"]) <= 1e-9 * max(1.0, np.linalg.norm(g["rhs_vel"]))
    assert np.abs(f2.getArray() - g["rhs_f"]).max() <= 1e-6 * scale
