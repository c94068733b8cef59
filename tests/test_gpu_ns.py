"""GPU parity of the no-slip row: MatNS assembled
on the device vs the reference's own matrices (cavity fixture) and vs the
oracle restatement (oracle.assemble_ns) on larger 2-D / 3-D meshes; the
free-slip pre-solve solveFS (kle_solver.py:39-41) and the no-slip branch of
evalRHS (base_problem.py:118-122).

Tolerances (fp64): DoF-level patterns bit-exact; values <= 1e-12 * max|ref|;
solutions of CG (rtol 1e-13) vs the reference's direct solve <= 1e-9
relative; evalRHS output <= 1e-6 of its scale (third derivatives of the
solved field)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
NS_MATS = ("K", "Krhs", "Rw", "Rd", "Kfs", "Krhsfs", "Rwfs", "Rdfs")
CAVITY = {"up": [2, 0], "down": [0, 0], "left": [0, 0], "right": [0, 0]}


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _matns(pa, dim, nelem, ngl, walls):
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": [0] * dim, "upper": [1] * dim}},
           "boundary-conditions": {"no-slip": walls}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatNS()
    mat.setDomain(dom)
    mat.build()
    return dom, mat


def _check(A, ip, ix, d, name):
    a_ip, a_ix, a_d = A.getValuesCSR()
    np.testing.assert_array_equal(a_ip, ip, err_msg=name)
    np.testing.assert_array_equal(a_ix, ix, err_msg=name)
    assert np.abs(a_d - d).max() <= 1e-12 * max(1.0, np.abs(d).max()), name


def test_matns_matches_golden(pa):
    g = np.load(os.path.join(G, "case_cavity2d.npz"))
    dom, mat = _matns(pa, 2, [4, 4], 3, CAVITY)
    for k in NS_MATS:
        _check(getattr(mat, k), g[k + "_indptr"], g[k + "_indices"], g[k + "_data"], k)
    # K + Kfs: device-assembled sum == PETSc union of the reference's K and Kfs
    K = O.CSR.from_arrays(g["K_indptr"], g["K_indices"], g["K_data"], 162)
    Kfs = O.CSR.from_arrays(g["Kfs_indptr"], g["Kfs_indices"], g["Kfs_data"], 162)
    S = K.dense() + Kfs.dense()
    mask = (K.dense() != 0) | (Kfs.dense() != 0)
    pat = np.zeros_like(mask)
    for M in (K, Kfs):
        for r in range(M.m):
            pat[r, M.indices[M.indptr[r]:M.indptr[r + 1]]] = True
    ip, ix, d = mat.getKplusKfs().getValuesCSR()
    dense = np.zeros_like(S)
    got = np.zeros_like(pat)
    for r in range(len(ip) - 1):
        dense[r, ix[ip[r]:ip[r + 1]]] = d[ip[r]:ip[r + 1]]
        got[r, ix[ip[r]:ip[r + 1]]] = True
    np.testing.assert_array_equal(got, pat)
    assert np.abs(dense - S).max() <= 1e-12 * np.abs(S).max()
    del mask
    # generic Mat + Mat (different patterns -> union AIJ) agrees with it
    U = mat.K + mat.Kfs
    u_ip, u_ix, u_d = U.getValuesCSR()
    np.testing.assert_array_equal(u_ip, ip)
    np.testing.assert_array_equal(u_ix, ix)
    assert np.abs(u_d - d).max() <= 1e-12 * np.abs(d).max()


@pytest.mark.parametrize("dim,nelem,ngl,walls", [
    (2, [6, 5], 4, {"down": [0, 0], "up": [1.5, 0], "right": [0, -0.5], "left": [0, 0]}),
    (2, [5, 4], 3, {"left": [0, 1], "up": [2, 0], "down": [0, 0]}),
    (3, [3, 2, 2], 3, {"up": [1, 0, 0.5], "down": [0, 0, 0], "left": [0, 0, 0], "right": [0, 0, 0],
                       "front": [0, 0, 0], "back": [0, 0, 0]}),
])
def test_matns_matches_oracle(pa, dim, nelem, ngl, walls):
    dom, mat = _matns(pa, dim, nelem, ngl, walls)
    om = O.BoxMesh(dim, nelem, [0] * dim, [1] * dim, ngl)
    T, N = O.noslip_dofs(om, list(walls))
    assert sorted(dom.getTangDofs(collect=True)) == sorted(T)
    assert sorted(dom.getNormalDofs(collect=True)) == sorted(N)
    ref = O.assemble_ns(om, T, N)
    for k in NS_MATS:
        R = ref[k]
        _check(getattr(mat, k), R.indptr, R.indices, R.data, k)


def test_solvefs_and_solve_match_golden(pa):
    g = np.load(os.path.join(G, "case_cavity2d.npz"))
    dom, mat = _matns(pa, 2, [4, 4], 3, CAVITY)
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    assert sol.isNS()
    sol.getKSP().setTolerances(rtol=1e-13)
    sol.solverFS.setTolerances(rtol=1e-13)
    vort = mat.Rw.createVecRight()
    vort.setArray(g["vort0"])
    vel = sol.getSolution()
    vel.setArray(g["vel0"])
    np.testing.assert_allclose(sol.rhsFS(vort).getArray(), g["bFS"], rtol=0, atol=1e-12 * np.abs(g["bFS"]).max())
    sol.solveFS(vort)
    vfs = sol.getFreeSlipSolution().getArray()
    assert np.linalg.norm(vfs - g["velFS"]) <= 1e-9 * np.linalg.norm(g["velFS"])
    sol.solve(vort)
    u = vel.getArray()
    assert np.linalg.norm(u - g["u"]) <= 1e-9 * np.linalg.norm(g["u"])


def test_eval_rhs_noslip_matches_reference(pa):
    g = np.load(os.path.join(G, "case_cavity2d.npz"))
    cfg = {"name": "cavity", "material-properties": {"rho": float(g["rho"]), "mu": float(g["mu"])},
           "domain": {"ngl": 3, "box-mesh": {"nelem": [4, 4], "lower": [0, 0], "upper": [1, 1]}},
           "boundary-conditions": {"no-slip": CAVITY}, "initial-conditions": {"velocity": [0, 0]}}
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    prob.setUpSolver()
    prob.solverKLE.getKSP().setTolerances(rtol=1e-13)
    prob.solverKLE.solverFS.setTolerances(rtol=1e-13)
    prob.solverKLE.getSolution().setArray(g["vel0"])
    prob.vort.setArray(g["rhs_vort_in"])
    f = prob.operator.Curl.createVecLeft()
    prob.evalRHS(None, float(g["rhs_t"]), prob.vort, f)
    vfs = prob.solverKLE.getFreeSlipSolution().getArray()
    assert np.linalg.norm(vfs - g["rhs_velFS"]) <= 1e-9 * np.linalg.norm(g["rhs_velFS"])
    np.testing.assert_allclose(prob.vort.getArray(), g["rhs_vort_bc"], rtol=0,
                               atol=1e-9 * np.abs(g["rhs_vort_bc"]).max())
    u = prob.solverKLE.getSolution().getArray()
    assert np.linalg.norm(u - g["rhs_vel"]) <= 1e-9 * np.linalg.norm(g["rhs_vel"])
    scale = max(1.0, np.abs(g["rhs_f"]).max())
    assert np.abs(f.getArray() - g["rhs_f"]).max() <= 1e-6 * scale


def test_config1_cavity_at_stated_size_matches_reference(pa):
    """BASELINE config 1 at its stated size: src/cases/cavity-2d.yaml as-is
    (50 x 50 cells, ngl 3, rho 0.5, mu 0.01, no-slip walls with the lid at
    [2, 0]; 20,402 velocity DoF).  Golden vectors from the reference's own
    MatNS / KleSolver.solveFS + solve / BaseProblem.evalRHS
    (make_golden.py cavity2d_full: cavity-2d.yaml:1-29, mat_ns.py:47-145,
    kle_solver.py:39-41, base_problem.py:111-136; direct solves as the
    makefile's preonly + lu).  Device: free-slip rhs and solution, no-slip
    solution <= 1e-9 relative, evalRHS <= 1e-6 of its scale; K's nonzero
    count and the tangential / normal DoF sets exact."""
    g = np.load(os.path.join(G, "case_cavity2d_full.npz"))
    cfg = {"name": "cavity", "material-properties": {"rho": float(g["rho"]), "mu": float(g["mu"])},
           "domain": {"ngl": 3, "box-mesh": {"nelem": [50, 50], "lower": [0, 0], "upper": [1, 1]}},
           "boundary-conditions": {"no-slip": CAVITY}, "initial-conditions": {"velocity": [0, 0]}}
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    prob.setUpSolver()
    dom, sol = prob.dom, prob.solverKLE
    assert sorted(dom.getTangDofs(collect=True)) == sorted(g["tang_dofs"].tolist())
    assert sorted(dom.getNormalDofs(collect=True)) == sorted(g["normal_dofs"].tolist())
    sol.getKSP().setTolerances(rtol=1e-13)
    sol.solverFS.setTolerances(rtol=1e-13)
    assert prob.mat.K.getInfo()["nz_used"] == int(g["K_nnz"])
    # solveFS + solve on the initial state (kle_solver.py:33-41)
    vort = prob.mat.Rw.createVecRight()
    vort.setArray(g["vort0"])
    vel = sol.getSolution()
    vel.setArray(g["vel0"])
    np.testing.assert_allclose(sol.rhsFS(vort).getArray(), g["bFS"], rtol=0, atol=1e-12 * np.abs(g["bFS"]).max())
    sol.solveFS(vort)
    vfs = sol.getFreeSlipSolution().getArray()
    assert np.linalg.norm(vfs - g["velFS"]) <= 1e-9 * np.linalg.norm(g["velFS"])
    sol.solve(vort)
    assert np.linalg.norm(vel.getArray() - g["u"]) <= 1e-9 * np.linalg.norm(g["u"])
    # one evalRHS (base_problem.py:111-136) at t = rhs_t
    vel.setArray(g["vel0"])
    prob.vort.setArray(g["rhs_vort_in"])
    f = prob.operator.Curl.createVecLeft()
    prob.evalRHS(None, float(g["rhs_t"]), prob.vort, f)
    vfs = sol.getFreeSlipSolution().getArray()
    assert np.linalg.norm(vfs - g["rhs_velFS"]) <= 1e-9 * np.linalg.norm(g["rhs_velFS"])
    np.testing.assert_allclose(prob.vort.getArray(), g["rhs_vort_bc"], rtol=0,
                               atol=1e-9 * np.abs(g["rhs_vort_bc"]).max())
    u = sol.getSolution().getArray()
    assert np.linalg.norm(u - g["rhs_vel"]) <= 1e-9 * np.linalg.norm(g["rhs_vel"])
    scale = max(1.0, np.abs(g["rhs_f"]).max())
    assert np.abs(f.getArray() - g["rhs_f"]).max() <= 1e-6 * scale


def test_getrow_matches_csr(pa):
    """Mat.getRow (petsc4py, dmplex.py:332,363) on node-block matrices with and
    without DoF-level masks, and on a scalar AIJ matrix."""
    dom, mat = _matns(pa, 2, [4, 4], 3, CAVITY)
    rng = np.random.default_rng(2)
    for A in (mat.K, mat.Kfs, mat.Krhsfs, mat.Rwfs, mat.getKplusKfs(), mat.getOperators().SrT, mat.K + mat.Kfs):
        ip, ix, d = A.getValuesCSR()
        lo, _ = A.getOwnershipRange()
        for r in rng.choice(len(ip) - 1, 12, replace=False):
            cols, vals = A.getRow(lo + r)
            np.testing.assert_array_equal(cols, ix[ip[r]:ip[r + 1]])
            np.testing.assert_array_equal(vals, d[ip[r]:ip[r + 1]])
