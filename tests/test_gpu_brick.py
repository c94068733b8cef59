"""The box symmetric SpMV on bricks (kle_brick.hip).

Same product as the full storage -- the MatMult of the reference's KSPSolve
(kle_solver.py:35) on the SPD K of MatFS.buildFS (mat_fs.py:150-192) -- from
the stored upper blocks, one brick per CU with the brick region's sums in
LDS.  Tolerances (another summation order than the full storage):
  * vs the full-storage kernel and the exported PETSc CSR: <= 1e-14 relative
    (2-norm), max|diff| <= 1e-13 * max|y|;
  * vs the 128-row tile kernel (the same exact fixed-point transposed sums,
    other scales): <= 1e-14 relative;
  * bitwise reproducible: repeated products are identical (fixed-point sums
    are order-free, the gather sums the bricks in a fixed order).
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


def _mat(pa, nelem, ngl):
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": [0, 0, 0], "upper": [1, 1, 1]}},
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
                                       ([3, 4, 2], 6), ([1, 1, 1], 4), ([3, 3, 2], 7), ([9, 7, 5], 4),
                                       ([1, 1, 1], 3)])  # (3^3 nodes: every row of one stored block, no brick)
def test_brick_spmv_matches_full_storage_csr_and_tiles(pa, nelem, ngl):
    from pynama_amd.runtime import set_tuning
    _, mat = _mat(pa, nelem, ngl)
    K = mat.K
    K.setOption(K.Option.SPD, False)
    x = K.createVecRight()
    xa = np.random.default_rng(7).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y0 = (K * x).getArray().copy()
    ip, ix, d = K.getValuesCSR()
    yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
    K.setOption(K.Option.SPD, True)
    assert K.spmvKernel().startswith("k_nb_spmv_sym_brick"), K.spmvKernel()
    yb = (K * x).getArray().copy()
    for ref in (y0, yh):
        _close(yb, ref)
    for _ in range(3):
        np.testing.assert_array_equal((K * x).getArray(), yb)
    # the gather with 1, 2 or 4 waves per 64-row slice (its parts summed in
    # another grouping): the same product to rounding, each bitwise repeatable
    for wps in (1, 2, 4):
        set_tuning("spmv_gather_wps", wps)
        try:
            yw = (K * x).getArray().copy()
            np.testing.assert_array_equal((K * x).getArray(), yw)
        finally:
            set_tuning("spmv_gather_wps", 0)
        for ref in (y0, yh):
            _close(yw, ref)
    # the one-block rows as items of their bricks (spmv_brick_singles 0)
    # instead of formed by the gather (another plan: other regions and
    # scales) -- the same product to rounding
    set_tuning("spmv_brick_singles", 0)
    try:
        K.setOption(K.Option.SPD, True)
        ys = (K * x).getArray().copy()
    finally:
        set_tuning("spmv_brick_singles", 1)
        K.setOption(K.Option.SPD, True)
    for ref in (y0, yh):
        _close(ys, ref)
    set_tuning("spmv_sym_brick", 0)
    try:
        K.setOption(K.Option.SPD, True)
        assert K.spmvKernel().startswith("k_nb_spmv_sym_xl"), K.spmvKernel()
        yt = (K * x).getArray().copy()
    finally:
        set_tuning("spmv_sym_brick", 1)
        K.setOption(K.Option.SPD, True)
    assert np.linalg.norm(yb - yt) <= 1e-14 * np.linalg.norm(yt)
    np.testing.assert_array_equal((K * x).getArray(), yb)


@pytest.mark.parametrize("nelem,ngl,split", [([12, 10, 6], 5, 12 + 100 * 10 + 10000 * 6),
                                             ([8, 8, 6], 7, 8 + 100 * 8 + 10000 * 6)])
def test_brick_spmv_whole_rounds_per_cu(pa, nelem, ngl, split):
    """More bricks than CUs (k whole rounds of one brick per CU, as the planner
    takes when one round's regions do not fit the LDS -- config 4 at p = 6):
    the same product as the full storage and the exported CSR to rounding,
    bitwise repeatable."""
    from pynama_amd.runtime import set_tuning
    _, mat = _mat(pa, nelem, ngl)
    K = mat.K
    K.setOption(K.Option.SPD, False)
    x = K.createVecRight()
    xa = np.random.default_rng(11).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y0 = (K * x).getArray().copy()
    ip, ix, d = K.getValuesCSR()
    yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
    set_tuning("spmv_brick_rounds", 4)
    set_tuning("spmv_brick_split", split)
    try:
        K.setOption(K.Option.SPD, True)
        assert K.spmvKernel().startswith("k_nb_spmv_sym_brick"), K.spmvKernel()
        yb = (K * x).getArray().copy()
        np.testing.assert_array_equal((K * x).getArray(), yb)
    finally:
        set_tuning("spmv_brick_rounds", 1)
        set_tuning("spmv_brick_split", 0)
        K.setOption(K.Option.SPD, True)
    for ref in (y0, yh):
        _close(yb, ref)


def test_brick_spmv_edge_inputs(pa):
    """x = 0 gives y = 0 exactly; extreme magnitudes (1e300, 1e-300) scale
    exactly as a floating-point product would (the fixed-point scale follows
    max |x| per brick); one nonzero entry; a NaN in x turns the product NaN
    (no silent finite result)."""
    _, mat = _mat(pa, [6, 5, 4], 5)
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
    assert K.spmvKernel().startswith("k_nb_spmv_sym_brick")
    for nm, xa in cases.items():
        x.setArray(xa)
        y = (K * x).getArray()
        if nm == "zero":
            assert not y.any()
        else:
            assert np.isfinite(y).all(), nm
            _close(y, refs[nm])
    xa = base.copy()
    xa[n // 3] = np.nan
    x.setArray(xa)
    assert np.isnan((K * x).getArray()).any()
    x.setArray(base)
    assert np.isfinite((K * x).getArray()).all()  # (the next product is clean again)


def test_local_product_timing_on_one_rank_is_the_product(pa):
    """kle_mat_time_local_spmv (bench.py's per-rank part timing at N > 1): on
    one rank the local product is the product -- y bitwise equal to K x --
    and the average time is positive; a matrix without bricks is refused."""
    _, mat = _mat(pa, [6, 5, 4], 5)
    K = mat.K
    x = K.createVecRight()
    x.setArray(np.random.default_rng(4).uniform(-1, 1, x.getLocalSize()))
    y = K.createVecLeft()
    K.setOption(K.Option.SPD, False)
    with pytest.raises(pa.Error):
        K.timeLocalSpmv(x, y, 3)
    K.setOption(K.Option.SPD, True)
    ref = (K * x).getArray().copy()
    ms = K.timeLocalSpmv(x, y, 7)
    assert ms > 0.0
    np.testing.assert_array_equal(y.getArray(), ref)


def test_brick_cg_reproducible_and_matches_oracle(pa):
    """CG through the brick SpMV: the oracle's Jacobi-CG iteration count within
    2, the solution within 1e-7, two solves bitwise equal."""
    from oracle import oracle as O
    from pynama_amd.petsc import KSP, PC
    dom, mat = _mat(pa, [8, 6, 5], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.spmvKernel().startswith("k_nb_spmv_sym_brick")
    b = K.createVecLeft()
    rng = np.random.default_rng(5)
    ba = rng.uniform(-1, 1, b.getLocalSize())
    b.setArray(ba)
    sols = []
    its = []
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
    assert abs(its[0] - ito) <= 2 + 0 * its[0], (its[0], ito)
    assert np.linalg.norm(sols[0] - xo) <= 1e-7 * np.linalg.norm(xo)
