"""The unstructured symmetric SpMV on row bricks (kle_gbrick.hip; DESIGN 3,
round 5).

Same product as the full storage -- the MatMult of the reference's KSPSolve
(kle_solver.py:35) on the SPD K of MatFS.buildFS (mat_fs.py:150-192) built on
a Gmsh mesh (config 5's path) -- from the stored upper blocks, one
contiguous range of Hilbert-ordered rows per CU with its dictionary's x and
exact fixed-point sums in LDS.  Tolerances (another summation order than the
full storage):
  * vs the column-dictionary full-storage kernel and the exported PETSc CSR:
    <= 1e-14 relative (2-norm), max|diff| <= 1e-13 * max|y|;
  * vs the 64-row dictionary groups (the same exact fixed-point transposed
    sums, other scales): <= 1e-14 relative;
  * bitwise reproducible: repeated products are identical.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _umat(pa, tmp_path, nelem, ngl, seed=5):
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    V, Cc, F, T = perturbed_box(3, nelem, seed=seed)
    path = tmp_path / f"g{seed}.msh"
    write_gmsh(path, 3, V, Cc, F, T)
    cfg = {"domain": {"ngl": ngl, "gmsh-file": str(path)},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    return dom, mat


def _close(y, ref):
    assert np.linalg.norm(y - ref) <= 1e-14 * np.linalg.norm(ref)
    assert np.abs(y - ref).max() <= 1e-13 * np.abs(ref).max()


@pytest.mark.parametrize("nelem,ngl", [([3, 2, 2], 5), ([12, 10, 6], 5), ([7, 5, 4], 3), ([6, 5, 3], 2),
                                       ([3, 4, 2], 6), ([1, 1, 1], 4), ([9, 7, 5], 4)])
def test_gbrick_spmv_matches_full_storage_csr_and_groups(pa, tmp_path, nelem, ngl):
    from pynama_amd.runtime import set_tuning
    _, mat = _umat(pa, tmp_path, nelem, ngl)
    K = mat.K
    assert not K.isStructured()
    K.setOption(K.Option.SPD, False)
    x = K.createVecRight()
    xa = np.random.default_rng(7).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y0 = (K * x).getArray().copy()
    ip, ix, d = K.getValuesCSR()
    yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
    K.setOption(K.Option.SPD, True)
    assert K.spmvKernel().startswith("k_nb_spmv_gsym_brick"), K.spmvKernel()
    yb = (K * x).getArray().copy()
    for ref in (y0, yh):
        _close(yb, ref)
    for _ in range(3):
        np.testing.assert_array_equal((K * x).getArray(), yb)
    set_tuning("spmv_gsym_brick", 0)
    try:
        K.setOption(K.Option.SPD, True)
        assert K.spmvKernel().startswith("k_nb_spmv_gsym<"), K.spmvKernel()
        yg = (K * x).getArray().copy()
    finally:
        set_tuning("spmv_gsym_brick", 1)
        K.setOption(K.Option.SPD, True)
    assert np.linalg.norm(yb - yg) <= 1e-14 * np.linalg.norm(yg)
    np.testing.assert_array_equal((K * x).getArray(), yb)


def test_gbrick_spmv_edge_inputs(pa, tmp_path):
    """x = 0 gives y = 0 exactly; 1e300 / 1e-300 scale as a floating-point
    product would; one nonzero entry; a NaN in x turns the product NaN;
    Dirichlet identity rows return x bit for bit."""
    _, mat = _umat(pa, tmp_path, [6, 5, 4], 5)
    K = mat.K
    K.setOption(K.Option.SPD, False)
    x = K.createVecRight()
    n = x.getLocalSize()
    rng = np.random.default_rng(3)
    base = rng.uniform(-1, 1, n)
    cases = {"zero": np.zeros(n), "big": base * 1e300, "tiny": base * 1e-300, "one": np.eye(1, n, n // 2)[0] * 3.5}
    refs = {}
    for nm, xa in cases.items():
        x.setArray(xa)
        refs[nm] = (K * x).getArray().copy()
    K.setOption(K.Option.SPD, True)
    assert K.spmvKernel().startswith("k_nb_spmv_gsym_brick")
    for nm, xa in cases.items():
        x.setArray(xa)
        y = (K * x).getArray()
        if nm == "zero":
            assert not y.any()
        else:
            assert np.isfinite(y).all(), nm
            _close(y, refs[nm])
    # identity rows (Dirichlet): y_i = x_i exactly
    x.setArray(base)
    y = (K * x).getArray()
    ip, ix, d = K.getValuesCSR()
    ident = [i for i in range(n) if ip[i + 1] - ip[i] == 1 and ix[ip[i]] == i and d[ip[i]] == 1.0]
    assert ident and np.array_equal(y[ident], base[ident])
    xa = base.copy()
    xa[n // 3] = np.nan
    x.setArray(xa)
    assert np.isnan((K * x).getArray()).any()
    x.setArray(base)
    assert np.isfinite((K * x).getArray()).all()


def test_gbrick_cg_reproducible_and_matches_oracle(pa, tmp_path):
    """CG through the graph-brick SpMV: the oracle's Jacobi-CG iteration count
    within 2, the solution within 1e-7, two solves bitwise equal."""
    from oracle import oracle as O
    from pynama_amd.petsc import KSP, PC
    _, mat = _umat(pa, tmp_path, [8, 6, 5], 4)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.spmvKernel().startswith("k_nb_spmv_gsym_brick")
    b = K.createVecLeft()
    ba = np.random.default_rng(5).uniform(-1, 1, b.getLocalSize())
    b.setArray(ba)
    sols, its = [], []
    for _ in range(2):
        ksp = KSP().create()
        ksp.setType("cg")
        pc = PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setOperators(K)
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
        ksp.setUp()
        xv = K.createVecRight()
        ksp.solve(b, xv)
        assert ksp.getConvergedReason() > 0
        sols.append(xv.getArray().copy())
        its.append(ksp.getIterationNumber())
    np.testing.assert_array_equal(sols[0], sols[1])
    assert its[0] == its[1]
    ip, ix, d = K.getValuesCSR()
    A = O.CSR.from_arrays(ip, ix, d, int(ip.shape[0] - 1))
    xo, ito, _ = A.cg(ba, rtol=1e-10)
    assert abs(its[0] - ito) <= 2, (its[0], ito)
    assert np.linalg.norm(sols[0] - xo) <= 1e-7 * np.linalg.norm(xo)
