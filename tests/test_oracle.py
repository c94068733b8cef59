"""Pin the CPU oracle (oracle/kle_oracle.c) against the golden vectors the
reference's own code produced (tests/golden/make_golden.py).

Reference known answers carried over:
  * gaussPoints(2) exactly [-1/sqrt3, 1/sqrt3], weights exactly [1,1]
    (test_element.py:181-191)
  * GLL / Gauss tables, 12 decimals (test_element.py:13-229)
  * element K / Rd at 14 decimals (test_element.py:285-296)
  * KLE solve, uniform flow 3x3 ngl=3: ||u-u_exact|| < 1e-12 (test_solver.py:18-25)
  * KLE solve, Taylor-Green 2-D 10x10 ngl=5: < 1e-5 (test_solver.py:30-37)
"""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["uniform2d", "tg2d", "tg2d_small", "tg3d", "tg3d_p4"]


@pytest.fixture(scope="module")
def tables():
    return np.load(os.path.join(G, "tables.npz"))


@pytest.fixture(scope="module")
def elements():
    return np.load(os.path.join(G, "elements.npz"))


def test_gauss_exact_n2():
    x, w = O.gauss(2)
    g = 1 / math.sqrt(3)
    np.testing.assert_array_equal(x, [-g, g])
    np.testing.assert_array_equal(w, [1.0, 1.0])


@pytest.mark.parametrize("n", range(1, 9))
def test_gauss_golden(tables, n):
    x, w = O.gauss(n)
    np.testing.assert_allclose(x, tables[f"gauss_x_{n}"], rtol=0, atol=2e-15)
    np.testing.assert_allclose(w, tables[f"gauss_w_{n}"], rtol=0, atol=2e-15)


@pytest.mark.parametrize("n", range(2, 9))
def test_lobatto_golden_bitexact(tables, n):
    x, w = O.lobatto(n)
    np.testing.assert_array_equal(x, tables[f"lobatto_x_{n}"])
    np.testing.assert_array_equal(w, tables[f"lobatto_w_{n}"])


@pytest.mark.parametrize("n", range(1, 9))
def test_spectral_order_bitexact(tables, n):
    np.testing.assert_array_equal(O.spectral_order(3, n), tables[f"spectral_order_{n}"])


NAMES = {"H": ("full", 0), "Hrs": ("full", 1), "HRed": ("red", 0), "HrsRed": ("red", 1),
         "HOp": ("op", 0), "HrsOp": ("op", 1), "HCoo": ("coo", 0), "HrsCoo": ("coo", 1),
         "HCooRed": ("cooRed", 0), "HrsCooRed": ("cooRed", 1), "HCooOp": ("cooOp", 0)}


@pytest.mark.parametrize("dim,ngl", [(2, n) for n in range(2, 9)] + [(3, n) for n in range(2, 6)])
def test_basis_tables(tables, dim, ngl):
    e = O.Element(ngl, dim)
    for nm, (which, what) in NAMES.items():
        ref = tables[f"{nm}_{dim}d_{ngl}"]
        t = e.table(which, what)
        np.testing.assert_allclose(t, ref.reshape(t.shape), rtol=0, atol=1e-12 * max(1, np.abs(ref).max()))
    g = tables[f"gps_{dim}d_{ngl}"]
    np.testing.assert_allclose(e.table("full", 3), g[:, :dim], atol=1e-15)
    np.testing.assert_allclose(e.table("full", 2), g[:, dim], atol=2e-15)


def _elem_keys(E):
    return sorted(k[2:] for k in E.files if k.startswith("K_"))


def test_element_matrices(elements):
    E = elements
    for tag in _elem_keys(E):
        dim, ngl = int(tag[0]), int(tag.split("_")[1])
        e = O.Element(ngl, dim)
        X = E["X_" + tag]
        K, Rw, Rd = e.kle(X)
        S, D, Cu, W = e.ops(X)
        for nm, t in (("K", K), ("Rw", Rw), ("Rd", Rd), ("SrT", S), ("DivSrT", D),
                      ("Curl", Cu), ("W", W)):
            if nm + "_" + tag not in E.files:
                continue
            ref = E[nm + "_" + tag]
            scale = np.abs(ref).max()
            assert np.abs(ref - t).max() <= 1e-13 * scale, (nm, tag)
        if tag.endswith("legacy") and ngl == 2:  # test_element.py:285-296 (ngl=2), decimal=14
            np.testing.assert_array_almost_equal(K, E["K_" + tag], decimal=14)
            np.testing.assert_array_almost_equal(Rd, E["Rd_" + tag], decimal=14)


@pytest.mark.parametrize("case", CASES)
def test_assembly_and_solve(case):
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim, ngl = int(g["dim"]), int(g["ngl"])
    m = O.BoxMesh(dim, g["nelem"], g["lower"], g["upper"], ngl)
    np.testing.assert_array_equal(m.conn(), g["conn"])          # bit-exact connectivity
    np.testing.assert_allclose(m.coords(), g["coords"], atol=1e-15)
    flag = np.zeros(m.N, np.uint8)
    flag[g["dir_nodes"]] = 1
    K, Kr, Rw = m.assemble_fs(flag)
    for nm, A in (("K", K), ("Krhs", Kr), ("Rw", Rw)):
        np.testing.assert_array_equal(A.indptr, g[nm + "_indptr"])     # bit-exact pattern
        np.testing.assert_array_equal(A.indices, g[nm + "_indices"])
        d = g[nm + "_data"]
        assert np.abs(A.data - d).max() <= 1e-13 * np.abs(d).max(), nm
    b = Rw.mult(g["vort0"]) + Kr.mult(g["vel0"])
    np.testing.assert_allclose(b, g["b"], rtol=0, atol=1e-13 * np.abs(g["b"]).max())
    x, it, rr = K.cg(b, rtol=1e-14, maxit=50000)
    assert rr < 1e-13
    assert np.linalg.norm(x - g["u"]) <= 1e-12 * np.linalg.norm(g["u"])
    if case == "uniform2d":
        assert np.linalg.norm(x - g["u_exact"]) < 1e-12
    if case == "tg2d":
        assert np.linalg.norm(x - g["u_exact"]) < 1e-5


@pytest.mark.parametrize("case", ["uniform2d", "tg2d_small", "tg3d", "cavity2d"])
def test_operators_golden(case):
    """Operators (mat_fs.py:194-271): pattern bit-exact, values to a few ulps of
    the reference's assembled Curl / SrT / DivSrT."""
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim = int(g["dim"])
    m = O.BoxMesh(dim, list(g["nelem"]), list(g["lower"]), list(g["upper"]), int(g["ngl"]))
    Cu, S, D, W = m.assemble_ops()
    for nm, A in (("Curl", Cu), ("SrT", S), ("DivSrT", D)):
        np.testing.assert_array_equal(A.indptr, g[nm + "_indptr"])
        np.testing.assert_array_equal(A.indices, g[nm + "_indices"])
        ref = g[nm + "_data"]
        assert np.abs(A.data - ref).max() <= 1e-14 * np.abs(ref).max(), nm
    # lumped weights sum to the domain measure
    assert abs(W.sum() - np.prod(np.asarray(g["upper"]) - np.asarray(g["lower"]))) < 1e-12


@pytest.mark.parametrize("case", ["uniform2d", "tg2d_small", "tg3d"])
def test_eval_rhs_chain_golden(case):
    """The operator chain of BaseProblem.evalRHS (base_problem.py:111-136),
    restated on the oracle's operators, reproduces the reference's own evalRHS
    output from the same KLE velocity."""
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim = int(g["dim"])
    m = O.BoxMesh(dim, list(g["nelem"]), list(g["lower"]), list(g["upper"]), int(g["ngl"]))
    Cu, S, D, _ = m.assemble_ops()
    vt, aux, f = O.eval_rhs_chain(Cu, S, D, g["rhs_vel"], float(g["rho"]), float(g["mu"]), dim)
    np.testing.assert_array_equal(vt, g["rhs_VtensV"])
    assert np.abs(aux - g["rhs_Aux1"]).max() <= 1e-12 * max(1.0, np.abs(g["rhs_Aux1"]).max())
    scale = max(1.0, np.abs(g["rhs_f"]).max())
    assert np.abs(f - g["rhs_f"]).max() <= 1e-10 * scale


NS_MATS = ("K", "Krhs", "Rw", "Rd", "Kfs", "Krhsfs", "Rwfs", "Rdfs")


def test_noslip_golden():
    """MatNS.buildNS restated (oracle.assemble_ns) against the reference's own
    no-slip matrices (cavity, 4x4, ngl=3): DoF sets and patterns exact, values
    to a few ulps."""
    g = np.load(os.path.join(G, "case_cavity2d.npz"))
    m = O.BoxMesh(2, [4, 4], [0, 0], [1, 1], 3)
    T, N = O.noslip_dofs(m, ["up", "down", "left", "right"])
    assert sorted(T) == sorted(g["tang_dofs"].tolist())
    assert sorted(N) == sorted(g["normal_dofs"].tolist())
    mats = O.assemble_ns(m, T, N)
    for k in NS_MATS:
        A = mats[k]
        np.testing.assert_array_equal(A.indptr, g[k + "_indptr"])
        np.testing.assert_array_equal(A.indices, g[k + "_indices"])
        assert np.abs(A.data - g[k + "_data"]).max() <= 1e-14 * np.abs(g[k + "_data"]).max(), k


@pytest.mark.parametrize("nelem,ngl", [([3, 2, 2], 5), ([2, 2, 2], 3), ([2, 1, 1], 6)])
def test_kle_k_is_symmetric_with_upper_tails(nelem, ngl):
    """What the symmetric-storage SpMV relies on, stated on the
    oracle's K (mat_fs.py:150-192): K == K^T to rounding, and in the box's
    lexicographic node order each row's columns at or after its own node
    (the stored upper tail) hold exactly its entries with j >= i."""
    import scipy.sparse as sp
    m = O.BoxMesh(3, nelem, [0, 0, 0], [1, 1, 1], ngl)
    xo = m.coords()
    flag = ((xo == 0.0) | (xo == 1.0)).any(axis=1).astype(np.uint8)
    K, _, _ = m.assemble_fs(flag)
    A = sp.csr_matrix((K.data, K.indices, K.indptr), shape=(K.m, K.m))
    D = abs(A - A.T)
    assert D.max() <= 1e-12 * abs(A).max()
    # upper triangle + strictly lower triangle reconstruct K
    U = sp.triu(A, 0)
    assert abs((U + sp.triu(A, 1).T) - A).max() <= 1e-12 * abs(A).max()
    # half the blocks (plus the diagonal) are kept: 3x3 node blocks
    n = K.m // 3
    rows = np.repeat(np.arange(K.m), np.diff(K.indptr)) // 3
    cols = K.indices // 3
    blocks = np.unique(rows * n + cols)
    r, c = blocks // n, blocks % n
    assert np.count_nonzero(c >= r) == (len(blocks) + n) // 2
