"""GPU parity tests: libkle.so (HIP, gfx950) against the CPU oracle and the
golden fixtures produced by the reference's own code.

Tolerances (fp64):
  * connectivity / patterns: bit-exact
  * element + assembled matrices: max|diff| <= 1e-12 * max|ref| (different
    but equivalent fp64 summation orders: factored vs B^T B form)
  * SpMV: <= 1e-13 relative in the 2-norm
  * KLE solution vs the reference direct solve: <= 1e-9 relative at
    rtol 1e-13 (CG stops on ||r|| <= rtol ||b||)
  * known answers: uniform < 1e-12, Taylor-Green 2-D p=4 < 1e-5
    (test_solver.py:18-37)
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["uniform2d", "tg2d", "tg2d_small", "tg3d", "tg3d_p4"]


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _golden(case):
    return np.load(os.path.join(G, f"case_{case}.npz"))


def _my_index(loc2lat, ngl):
    """reference local node l -> tensor index of libkle's element order"""
    idx = np.zeros(len(loc2lat), dtype=np.int64)
    for d in range(loc2lat.shape[1]):
        idx += loc2lat[:, d] * ngl ** d
    return idx


def _domain(pa, g):
    dim = int(g["dim"])
    cfg = {"domain": {"ngl": int(g["ngl"]), "box-mesh": {"nelem": list(g["nelem"]),
                                                          "lower": list(g["lower"]), "upper": list(g["upper"])}},
           "boundary-conditions": {"uniform": {"velocity": [4, 0]}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    dom.mesh.set_dirichlet_nodes(g["dir_nodes"])
    return dom


@pytest.mark.parametrize("case", CASES)
def test_assembly_matches_golden(pa, case):
    g = _golden(case)
    dom = _domain(pa, g)
    # bit-exact connectivity (reference local order via the golden loc2lat)
    conn = dom.mesh.conn()
    np.testing.assert_array_equal(conn[:, _my_index(g["loc2lat"], int(g["ngl"]))], g["conn"])
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    for nm in ("K", "Krhs", "Rw"):
        ip, ix, d = getattr(mat, nm).getValuesCSR()
        np.testing.assert_array_equal(ip, g[nm + "_indptr"])
        np.testing.assert_array_equal(ix, g[nm + "_indices"])
        ref = g[nm + "_data"]
        assert np.abs(d - ref).max() <= 1e-12 * np.abs(ref).max(), nm


@pytest.mark.parametrize("kernel", ["mfma", "valu"])
@pytest.mark.parametrize("dim,ngl", [(2, 2), (2, 3), (2, 5), (2, 7), (3, 2), (3, 3), (3, 5), (3, 6), (3, 7)])
def test_element_kernel_vs_oracle(pa, dim, ngl, kernel):
    """k_element_mfma (FP64 MFMA, the default) and k_element (FP64 VALU,
    KLE_ELEMENT_VALU=1) against the oracle's element matrices."""
    import ctypes as C
    from pynama_amd._lib import call
    mesh = pa.BoxMesh(dim, [2] * dim, [0.1] * dim, [0.7, 0.5, 0.4][:dim], ngl)
    ctx = pa.get_ctx()
    n = ngl ** dim
    dw = 1 if dim == 2 else 3
    Ke = np.zeros((dim * n, dim * n))
    Rwe = np.zeros((dim * n, dw * n))
    os.environ["KLE_ELEMENT_VALU"] = "1" if kernel == "valu" else "0"
    try:
        call("kle_element_kle", ctx.h, mesh._h, 1, Ke, Rwe)
    finally:
        os.environ.pop("KLE_ELEMENT_VALU", None)
    el = O.Element(ngl, dim)
    X = mesh.corners()[1]
    Kr, Rwr, _ = el.kle(X.ravel())
    # oracle (reference local order) -> tensor order via geometry
    om = O.BoxMesh(dim, [2] * dim, [0.1] * dim, [0.7, 0.5, 0.4][:dim], ngl)
    ref_conn = om.conn()[1]
    my_conn = mesh.conn()[1]
    perm = np.array([np.where(my_conn == c)[0][0] for c in ref_conn])
    pv = (perm[:, None] * dim + np.arange(dim)[None, :]).ravel()
    pw = (perm[:, None] * dw + np.arange(dw)[None, :]).ravel()
    Kt = np.zeros_like(Kr)
    Kt[np.ix_(pv, pv)] = Kr
    Rt = np.zeros_like(Rwr)
    Rt[np.ix_(pv, pw)] = Rwr
    assert np.abs(Ke - Kt).max() <= 1e-12 * np.abs(Kt).max()
    assert np.abs(Rwe - Rt).max() <= 1e-12 * np.abs(Rt).max()


@pytest.mark.parametrize("case", CASES)
def test_spmv_and_solve(pa, case):
    g = _golden(case)
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    K = O.CSR.from_arrays(g["K_indptr"], g["K_indices"], g["K_data"], int(g["K_shape"][1]))
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, K.m)
    xv = mat.K.createVecRight()
    xv.setArray(x)
    yv = mat.K * xv
    y = K.mult(x)
    assert np.linalg.norm(yv.getArray() - y) <= 1e-13 * np.linalg.norm(y)
    # KLE solve: b = Rw w + Krhs vel0 ; K u = b
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    ksp = sol.getKSP()
    ksp.setTolerances(rtol=1e-13)
    vort = mat.Rw.createVecRight()
    vort.setArray(g["vort0"])
    vel = sol.getSolution()
    vel.setArray(g["vel0"])
    b = sol.rhs(vort)
    np.testing.assert_allclose(b.getArray(), g["b"], rtol=0, atol=1e-12 * np.abs(g["b"]).max())
    sol.solve(vort)
    u = vel.getArray()
    assert ksp.getConvergedReason() > 0
    assert ksp.getTrueRelativeResidual() < 1e-12
    assert np.linalg.norm(u - g["u"]) <= 1e-9 * np.linalg.norm(g["u"])
    if case == "uniform2d":
        assert np.linalg.norm(u - g["u_exact"]) < 1e-12  # test_solver.py:25
    if case == "tg2d":
        assert np.linalg.norm(u - g["u_exact"]) < 1e-5   # test_solver.py:37


@pytest.mark.parametrize("single", [False, True, "pipecg"])
@pytest.mark.parametrize("case", ["tg2d", "tg3d_p4"])
def test_cg_iterations_match_oracle(pa, case, single):
    g = _golden(case)
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    K = O.CSR.from_arrays(g["K_indptr"], g["K_indices"], g["K_data"], int(g["K_shape"][1]))
    xo, it_o, rr_o = K.cg(g["b"], rtol=1e-10, jacobi=True)
    ksp = pa.petsc.KSP().create()
    ksp.setType("pipecg" if single == "pipecg" else "cg")
    pc = pa.petsc.PC()
    pc.setType("jacobi")
    ksp.setPC(pc)
    ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
    if single != "pipecg":
        ksp.setCGSingleReduction(single)  # Chronopoulos-Gear: same iterates in exact arithmetic
    ksp.setOperators(mat.K)
    b = mat.K.createVecLeft()
    b.setArray(g["b"])
    x = mat.K.createVecRight()
    ksp.solve(b, x)
    # pipelined CG: same iterates in exact arithmetic, recurrences drift more in fp64
    tol_its = {False: 1, True: 2, "pipecg": 4}[single]
    assert abs(ksp.getIterationNumber() - it_o) <= tol_its
    assert ksp.getTrueRelativeResidual() <= 1.01e-10  # (default correction solve: the true residual meets rtol)
    assert np.linalg.norm(x.getArray() - xo) <= 1e-7 * np.linalg.norm(xo)


@pytest.mark.parametrize("typ", ["cg", "pipecg"])
def test_correction_keeps_main_reason_near_maxit(pa, typ):
    """A solve that converges on its recursive residual at exactly max_it
    stays CONVERGED_RTOL with PETSc's iteration count (KSPGetIterationNumber
    of the recurrence), whatever the correction solve does afterwards; the
    correction's iterations and reason are reported apart."""
    g = _golden("tg3d_p4")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    b = mat.K.createVecLeft()
    b.setArray(g["b"])

    def solve(maxit, corr):
        ksp = pa.petsc.KSP().create()
        ksp.setType(typ)
        pc = pa.petsc.PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=maxit)
        ksp.setCorrections(corr)
        ksp.setOperators(mat.K)
        x = mat.K.createVecRight()
        ksp.solve(b, x)
        return ksp

    plain = solve(10000, 0)
    n = plain.getIterationNumber()
    assert plain.getConvergedReason() > 0 and plain.getCorrectionIterations() == 0
    assert plain.getCorrectionReason() == 0
    for corr in (2, 1):
        k = solve(n, corr)  # (converges at the last allowed iteration)
        assert k.getConvergedReason() == plain.getConvergedReason()
        assert k.getIterationNumber() == n
        assert k.getResidualNorm() == plain.getResidualNorm()
        if k.getCorrectionIterations():
            assert k.getCorrectionReason() != 0
            if k.getCorrectionReason() > 0:
                assert k.getTrueRelativeResidual() <= 1.01e-10
        else:
            assert plain.getTrueRelativeResidual() <= 1e-10
    # one iteration short: DIVERGED_ITS from the main solve, no correction runs
    k = solve(n - 1, 2)
    assert k.getConvergedReason() < 0 and k.getIterationNumber() == n - 1
    assert k.getCorrectionIterations() == 0 and k.getCorrectionReason() == 0


@pytest.mark.parametrize("typ", ["cg", "pipecg"])
def test_failed_correction_keeps_x(pa, typ):
    """A correction solve that ends in NaN (the ksp_corr_fault test hook:
    refine runs it, then its result is NaN and its reason DIVERGED_NANORINF)
    leaves x as the main solve made it -- bitwise, finite -- and the main
    solve's reason, count and residual norm stand; the failed correction is
    reported apart."""
    from pynama_amd.runtime import set_tuning
    g = _golden("tg3d_p4")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    b = mat.K.createVecLeft()
    b.setArray(g["b"])

    def solve(corr):
        ksp = pa.petsc.KSP().create()
        ksp.setType(typ)
        pc = pa.petsc.PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
        ksp.setCorrections(corr)
        ksp.setOperators(mat.K)
        x = mat.K.createVecRight()
        ksp.solve(b, x)
        return ksp, x.getArray().copy()

    plain, x0 = solve(0)
    set_tuning("ksp_corr_fault", 1)
    try:
        k, x1 = solve(2)
    finally:
        set_tuning("ksp_corr_fault", 0)
    assert np.isfinite(x1).all()
    np.testing.assert_array_equal(x1, x0)
    assert k.getConvergedReason() == plain.getConvergedReason() > 0
    assert k.getIterationNumber() == plain.getIterationNumber()
    assert k.getResidualNorm() == plain.getResidualNorm()
    assert k.getCorrectionReason() == -9  # (KSP_DIVERGED_NANORINF)
    assert k.getTrueRelativeResidual() == plain.getTrueRelativeResidual()


def test_gmres_and_aij(pa):
    g = _golden("tg2d_small")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    A = mat.K.convert("aij")
    assert A.getFormat() == "aij"
    ip, ix, d = A.getValuesCSR()
    np.testing.assert_array_equal(ip, g["K_indptr"])
    x = mat.K.createVecRight()
    x.setArray(np.random.default_rng(1).uniform(-1, 1, x.getLocalSize()))
    xa = A.createVecRight()
    xa.setArray(x.getArray())
    np.testing.assert_allclose((A * xa).getArray(), (mat.K * x).getArray(), rtol=1e-13, atol=1e-11)
    ksp = pa.petsc.KSP().create()
    ksp.setType("gmres")
    ksp.setTolerances(rtol=1e-12, max_it=5000)
    ksp.setOperators(mat.K)
    b = mat.K.createVecLeft()
    b.setArray(g["b"])
    u = mat.K.createVecRight()
    ksp.solve(b, u)
    assert ksp.getConvergedReason() > 0
    assert np.linalg.norm(u.getArray() - g["u"]) <= 1e-9 * np.linalg.norm(g["u"])


def test_generic_aij_setvalues(pa):
    P = pa.petsc
    n = 7
    A = P.Mat().createAIJ(((n, None), (n, None)), nnz=([3] * n, None))
    A.setUp()
    rng = np.random.default_rng(3)
    dense = np.zeros((n, n))
    for _ in range(20):  # ADD_VALUES in call order, explicit zeros kept
        r = rng.integers(0, n, 2)
        c = rng.integers(0, n, 2)
        v = rng.uniform(-1, 1, (2, 2))
        A.setValues(r, c, v, addv=True)
        for i in range(2):
            for j in range(2):
                dense[r[i], c[j]] += v[i, j]
    A.setValues([0], [0], [[5.0]], addv=False)
    dense[0, 0] = 5.0
    A.assemble()
    x = P.Vec().createSeq(n)
    xv = rng.uniform(-1, 1, n)
    x.setArray(xv)
    y = A * x
    np.testing.assert_allclose(y.getArray(), dense @ xv, rtol=1e-14, atol=1e-14)
    pattern = {(r, c) for r in range(n) for c in range(n)}
    A_ip, A_ix, _ = A.getValuesCSR()
    present = {(r, int(c)) for r in range(n) for c in A_ix[A_ip[r]:A_ip[r + 1]]}
    free = sorted(pattern - present)
    if free:  # inserting outside the assembled pattern raises (MAT_NEW_NONZERO_ALLOCATION_ERR)
        with pytest.raises(P.Error):
            A.setValues([free[0][0]], [free[0][1]], [[1.0]], addv=True)


def test_vec_ops(pa):
    P = pa.petsc
    rng = np.random.default_rng(5)
    n = 10001
    a, b = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    x = P.Vec().createWithArray(a)
    y = P.Vec().createWithArray(b)
    assert abs(x.dot(y) - a @ b) < 1e-12
    assert abs(x.norm() - np.linalg.norm(a)) < 1e-12
    z = x + y
    np.testing.assert_allclose(z.getArray(), a + b, rtol=1e-15)
    z.axpy(2.0, x)
    np.testing.assert_allclose(z.getArray(), a + b + 2 * a, rtol=1e-14)
    z *= 0.5
    np.testing.assert_allclose(z.getArray(), 0.5 * (3 * a + b), rtol=1e-14)
    w = x * y
    np.testing.assert_allclose(w.getArray(), a * b, rtol=1e-15)
    x.setValues([3, 5], [7.0, 8.0])
    x.setValues([3], [1.0], addv=True)
    assert x.getValues([3, 5]).tolist() == [8.0, 8.0]
    r = P.Vec().createWithArray(np.array([2.0, 0.0, 4.0]))
    r.reciprocal()
    assert r.getArray().tolist() == [0.5, 0.0, 0.25]


@pytest.mark.parametrize("case", ["uniform2d", "tg2d"])
def test_preonly_lu_matches_golden(pa, case):
    """The makefile's -ksp_type preonly -pc_type lu (makefile:7): a dense device
    LU (rocSOLVER).  The golden u is the reference's KleSolver.solve with a
    direct solve standing in for PETSc's LU, so both sides are direct solves:
    agreement to roundoff, and the reference's known answers
    (test_solver.py:25,37)."""
    g = _golden(case)
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    opts = pa.petsc.Options()
    opts.update({"ksp_type": "preonly", "pc_type": "lu"})
    try:
        sol = pa.KleSolver()
        sol.setMat(mat)
        sol.setUp()
    finally:
        opts.pop("ksp_type")
        opts.pop("pc_type")
    ksp = sol.getKSP()
    vort = mat.Rw.createVecRight()
    vort.setArray(g["vort0"])
    vel = sol.getSolution()
    vel.setArray(g["vel0"])
    sol.solve(vort)
    u = vel.getArray()
    assert ksp.getIterationNumber() == 1 and ksp.getConvergedReason() == 4  # KSP_CONVERGED_ITS
    assert ksp.getTrueRelativeResidual() < 1e-13
    assert np.linalg.norm(u - g["u"]) <= 1e-12 * np.linalg.norm(g["u"])
    if case == "uniform2d":
        assert np.linalg.norm(u - g["u_exact"]) < 1e-12
    if case == "tg2d":
        assert np.linalg.norm(u - g["u_exact"]) < 1e-5


def test_gmres_lu_is_one_step_and_preonly_jacobi(pa):
    """KspSolver.createSolver's own gmres + PC lu (kle_solver.py:54-64) takes
    one step; preonly + jacobi applies D^-1 once, like PETSc."""
    g = _golden("tg2d_small")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    b = mat.K.createVecLeft()
    rng = np.random.default_rng(3)
    b.setArray(rng.uniform(-1, 1, b.getLocalSize()))
    ksp = pa.petsc.KSP().create()
    ksp.setType("gmres")
    pc = pa.petsc.PC().create()
    pc.setType("lu")
    ksp.setPC(pc)
    ksp.setOperators(mat.K)
    ksp.setUp()
    x = mat.K.createVecRight()
    ksp.solve(b, x)
    K = O.CSR.from_arrays(*mat.K.getValuesCSR(), mat.K.getSize()[1])
    assert ksp.getIterationNumber() == 1
    assert np.linalg.norm(K.mult(x.getArray()) - b.getArray()) <= 1e-13 * np.linalg.norm(b.getArray())
    ksp2 = pa.petsc.KSP().create()
    ksp2.setType("preonly")
    pc2 = pa.petsc.PC().create()
    pc2.setType("jacobi")
    ksp2.setPC(pc2)
    ksp2.setOperators(mat.K)
    ksp2.setUp()
    ksp2.solve(b, x)
    ip, ix, dv = mat.K.getValuesCSR()
    d = np.array([dv[ip[i]:ip[i + 1]][ix[ip[i]:ip[i + 1]] == i][0] for i in range(len(ip) - 1)])
    np.testing.assert_allclose(x.getArray(), b.getArray() / d, rtol=1e-15)


def test_lu_too_large_raises(pa):
    """Dense device LU is for small sequential systems; beyond that PC lu
    raises (PETSc error 56) -- no CPU fallback."""
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [8, 8, 8], "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    ksp = pa.petsc.KSP().create()
    pc = pa.petsc.PC().create()
    pc.setType("lu")
    ksp.setPC(pc)
    ksp.setOperators(mat.K)
    with pytest.raises(pa.Error) as e:
        ksp.setUp()
    assert e.value.ierr == 56


def test_larger_mesh_properties(pa):
    """Size-independent properties on a 3-D p=4 mesh (the bench config family):
    symmetry of K, linearity of SpMV, CG true residual, Dirichlet rows."""
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [6, 5, 4], "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    rng = np.random.default_rng(11)
    x = mat.K.createVecRight()
    y = mat.K.createVecRight()
    xa, ya = rng.uniform(-1, 1, x.getLocalSize()), rng.uniform(-1, 1, y.getLocalSize())
    x.setArray(xa)
    y.setArray(ya)
    Ax, Ay = mat.K * x, mat.K * y
    s = x + y
    As = mat.K * s
    np.testing.assert_allclose(As.getArray(), Ax.getArray() + Ay.getArray(), rtol=1e-12, atol=1e-9)
    assert abs(y.dot(Ax) - x.dot(Ay)) <= 1e-12 * abs(y.dot(Ax)) + 1e-9
    # Dirichlet rows are identity
    bn = sorted(dom.getNodesDirichlet())
    idx = (np.array(bn)[:, None] * 3 + np.arange(3)).ravel()
    np.testing.assert_array_equal(Ax.getArray()[idx], xa[idx])
    ksp = pa.petsc.KSP().create()
    ksp.setTolerances(rtol=1e-10, max_it=20000)
    ksp.setOperators(mat.K)
    u = mat.K.createVecRight()
    ksp.solve(Ax, u)
    assert ksp.getTrueRelativeResidual() <= 2e-10
    assert np.linalg.norm(u.getArray() - xa) <= 1e-5 * np.linalg.norm(xa)


@pytest.mark.parametrize("pad", [8, 16])
def test_row_padding_and_nt_loads_are_exact(pa, pad):
    """Padded row streams (every stream 128-B aligned) and non-temporal loads
    change only the memory layout / cache policy: export, diagonal, scaling and
    SpMV must be bit-identical to the unpadded plain-load matrix."""
    from pynama_amd.runtime import get_row_padding, get_value_layout, set_row_padding, set_value_layout
    g = _golden("tg3d_p4")
    mats = []
    old, old_lay = get_row_padding(), get_value_layout()
    set_value_layout(0)  # padding is a property of the stream layout
    try:
        for q in (1, pad):
            set_row_padding(q)
            dom = _domain(pa, g)
            mat = pa.MatFS()
            mat.setDomain(dom)
            mat.build()
            mats.append(mat)
    finally:
        set_row_padding(old)
        set_value_layout(old_lay)
    a, b = mats
    for nm in ("K", "Krhs", "Rw"):
        for u, v in zip(getattr(a, nm).getValuesCSR(), getattr(b, nm).getValuesCSR()):
            np.testing.assert_array_equal(u, v)
    rng = np.random.default_rng(3)
    x = a.K.createVecRight()
    x.setArray(rng.uniform(-1, 1, x.getLocalSize()))
    y0 = (a.K * x).getArray()
    np.testing.assert_array_equal((b.K * x).getArray(), y0)
    np.testing.assert_array_equal(b.K.getDiagonal().getArray(), a.K.getDiagonal().getArray())
    # padding is not useful traffic (only the real-length array, 4 B per row, is added)
    assert 0 <= b.K.spmvBytes() - a.K.spmvBytes() <= 4 * a.K.getSize()[0] / 3
    sc = a.K.createVecLeft()
    sc.setArray(rng.uniform(0.5, 2, sc.getLocalSize()))
    a.Rw.diagonalScale(L=sc)
    b.Rw.diagonalScale(L=sc)
    for u, v in zip(a.Rw.getValuesCSR(), b.Rw.getValuesCSR()):
        np.testing.assert_array_equal(u, v)


def test_structured_columns_are_exact(pa):
    """Row-box (computed) columns in the SpMV == the streamed column indices,
    bitwise; K / Rw / operators of a box mesh qualify, Krhs does not."""
    g = _golden("tg3d_p4")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    op = mat.getOperators()
    assert mat.K.isStructured() and mat.Rw.isStructured() and op.SrT.isStructured()
    assert not mat.Krhs.isStructured()
    rng = np.random.default_rng(4)
    for A in (mat.K, mat.Rw, op.Curl, op.SrT, op.DivSrT):
        x = A.createVecRight()
        x.setArray(rng.uniform(-1, 1, x.getLocalSize()))
        y1 = (A * x).getArray()
        A.setSpmvStructured(False)
        y0 = (A * x).getArray()
        A.setSpmvStructured(True)
        np.testing.assert_array_equal(y1, y0)
        assert A.spmvBytes() > 0


def test_chunked_value_layout_is_exact(pa):
    """Layout 1 (16-block chunks + packed tail, no per-stream padding) stores
    the same entries: CSR exports, getRow, diagonal, scaling and SpMV of the
    free-slip matrices, the operators and the no-slip matrices are bitwise equal
    to layout 0."""
    from pynama_amd.runtime import get_value_layout, set_value_layout
    old = get_value_layout()
    g = _golden("tg3d_p4")
    built = {}
    try:
        for lay in (0, 1):
            set_value_layout(lay)
            dom = _domain(pa, g)
            mat = pa.MatFS()
            mat.setDomain(dom)
            mat.build()
            cfg = {"domain": {"ngl": 4, "box-mesh": {"nelem": [3, 3], "lower": [0, 0], "upper": [1, 1]}},
                   "boundary-conditions": {"no-slip": {"up": [1, 0], "down": [0, 0], "left": [0, 0],
                                                       "right": [0, 0]}}}
            dns = pa.Domain()
            dns.configure(cfg)
            dns.setUp()
            mns = pa.MatNS()
            mns.setDomain(dns)
            mns.build()
            op = mat.getOperators()
            built[lay] = [mat.K, mat.Krhs, mat.Rw, op.Curl, op.SrT, op.DivSrT, mns.Kfs, mns.Krhsfs,
                          mns.getKplusKfs(), mns.Rdfs]
    finally:
        set_value_layout(old)
    rng = np.random.default_rng(9)
    for A0, A1 in zip(built[0], built[1]):
        for u, v in zip(A0.getValuesCSR(), A1.getValuesCSR()):
            np.testing.assert_array_equal(u, v)
        x = A0.createVecRight()
        x.setArray(rng.uniform(-1, 1, x.getLocalSize()))
        np.testing.assert_array_equal((A0 * x).getArray(), (A1 * x).getArray())
        r = A0.getOwnershipRange()[0] + 5
        for u, v in zip(A0.getRow(r), A1.getRow(r)):
            np.testing.assert_array_equal(u, v)
    K0, K1 = built[0][0], built[1][0]
    np.testing.assert_array_equal(K0.getDiagonal().getArray(), K1.getDiagonal().getArray())
    s = K0.createVecLeft()
    s.setArray(rng.uniform(0.5, 2, s.getLocalSize()))
    K0.diagonalScale(L=s)
    K1.diagonalScale(L=s)
    for u, v in zip(K0.getValuesCSR(), K1.getValuesCSR()):
        np.testing.assert_array_equal(u, v)


def test_spmv_layouts_and_column_modes_agree(pa):
    """The node-block SpMV kernel (k_nb_spmv) for both value layouts and both
    column modes (structured boxes / streamed bcol) gives bitwise the same
    product, and equals the exported CSR product to 1e-13, for K/Rw/Krhs and
    the operator shapes (3x3, 6x3, 3x6)."""
    import scipy.sparse as sp

    from pynama_amd.runtime import get_value_layout, set_value_layout
    g = _golden("tg3d_p4")
    old = get_value_layout()
    ref = {}
    try:
        for lay in (0, 1):
            set_value_layout(lay)
            dom = _domain(pa, g)
            mat = pa.MatFS()
            mat.setDomain(dom)
            mat.build()
            op = mat.getOperators()
            for nm, A in (("K", mat.K), ("Rw", mat.Rw), ("Krhs", mat.Krhs), ("SrT", op.SrT),
                          ("DivSrT", op.DivSrT), ("Curl", op.Curl)):
                rng = np.random.default_rng(len(nm))
                x = A.createVecRight()
                xa = rng.uniform(-1, 1, x.getLocalSize())
                x.setArray(xa)
                ys = []
                for st in (True, False):
                    A.setSpmvStructured(st)
                    ys.append((A * x).getArray())
                A.setSpmvStructured(True)
                np.testing.assert_array_equal(ys[0], ys[1])
                if nm in ref:
                    np.testing.assert_array_equal(ys[0], ref[nm])
                else:
                    ref[nm] = ys[0]
                ip, ix, d = A.getValuesCSR()
                yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
                np.testing.assert_allclose(ys[0], yh, rtol=0, atol=1e-13 * max(1.0, np.abs(yh).max()))
    finally:
        set_value_layout(old)


@pytest.mark.parametrize("nelem,ngl", [([3, 2, 2], 5), ([12, 10, 6], 5), ([7, 5, 4], 3), ([4, 3, 3], 7)])
def test_spmv_x_in_lds_is_bitwise(pa, nelem, ngl):
    """k_nb_spmv_xl (x staged in LDS per workgroup of 8 rows) ==
    k_nb_spmv with global x gathers (spmv_x_lds 0, 4 and 8 waves), bitwise,
    for the structured K and Rw: lattice lines of 11-49 nodes, so workgroups
    both fit one union box and wrap into the next line (global fallback)."""
    from pynama_amd.runtime import get_tuning, set_tuning
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    for A in (mat.K, mat.Rw):
        assert A.isStructured()
        x = A.createVecRight()
        x.setArray(np.random.default_rng(3).uniform(-1, 1, x.getLocalSize()))
        ys = []
        try:
            for xl, wv in ((1, 0), (0, 0), (0, 4), (0, 8)):
                set_tuning("spmv_x_lds", xl)
                set_tuning("spmv_waves", wv)
                ys.append((A * x).getArray().copy())
        finally:
            set_tuning("spmv_x_lds", 1)
            set_tuning("spmv_waves", 0)
        assert get_tuning("spmv_x_lds") == 1
        for yv in ys[1:]:
            np.testing.assert_array_equal(ys[0], yv)


@pytest.mark.parametrize("nel,ngl", [([4, 3, 3], 5), ([3, 3, 2], 3), ([2, 2, 2], 7)])
def test_spmv_column_dictionaries_are_bitwise(pa, nel, ngl, tmp_path):
    """k_nb_spmv_dict (unstructured 3x3 rows: x staged in LDS through each
    8-row group's column dictionary, 2-byte positions instead of the column
    stream) == k_nb_spmv with the bcol stream (spmv_dict 0, 4 and 8
    waves), bitwise, for K and Rw of a perturbed, rotated, shuffled Gmsh hex
    mesh; also after Mat.duplicate.  Dictionaries are built for every size
    here (spmv_dict_min_rows 0)."""
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    from pynama_amd.runtime import get_tuning, set_tuning
    V, Cc, F, T = perturbed_box(3, nel, seed=11)
    path = tmp_path / "m.msh"
    write_gmsh(path, 3, V, Cc, F, T)
    cfg = {"domain": {"ngl": ngl, "gmsh-file": str(path)},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    old = get_tuning("spmv_dict_min_rows")
    set_tuning("spmv_dict_min_rows", 0)
    try:
        dom = pa.Domain()
        dom.configure(cfg)
        dom.setUp()
        mat = pa.MatFS()
        mat.setDomain(dom)
        mat.build(buildOperators=False)
    finally:
        set_tuning("spmv_dict_min_rows", old)
    for A in (mat.K, mat.Rw, mat.K.duplicate(copy=True)):
        assert not A.isStructured()
        x = A.createVecRight()
        x.setArray(np.random.default_rng(5).uniform(-1, 1, x.getLocalSize()))
        ys = []
        try:
            for dct, wv in ((1, 8), (0, 8), (0, 4)):
                set_tuning("spmv_dict", dct)
                set_tuning("spmv_waves", wv)
                ys.append((A * x).getArray().copy())
        finally:
            set_tuning("spmv_dict", 1)
            set_tuning("spmv_waves", 0)
        for yv in ys[1:]:
            np.testing.assert_array_equal(ys[0], yv)


@pytest.mark.parametrize("lay", [0, 1])
def test_device_pattern_matches_host(pa, lay):
    """Box-mesh patterns built on the device (k_pat_count / k_pat_fill) ==
    the host enumeration (KLE_HOST_PATTERN=1), bitwise: CSR exports,
    structured-column detection, interior row range and SpMV, for the
    free-slip matrices (all-boundary and random Dirichlet sets, 2-D and 3-D,
    two slab ranks' rows), the operators and the no-slip matrices."""
    from pynama_amd.runtime import get_value_layout, set_value_layout
    old_lay = get_value_layout()
    rng = np.random.default_rng(17)
    g = _golden("tg3d_p4")

    def build_all():
        out = []
        dom = _domain(pa, g)
        mat = pa.MatFS()
        mat.setDomain(dom)
        mat.build()
        op = mat.getOperators()
        out += [mat.K, mat.Krhs, mat.Rw, op.Curl, op.SrT, op.DivSrT]
        for dim, nel, ngl in ((3, [3, 2, 4], 4), (2, [4, 3], 5)):
            cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nel, "lower": [0] * dim, "upper": [1] * dim}},
                   "boundary-conditions": {"uniform": {"velocity": [1] * dim}}}
            d = pa.Domain()
            d.configure(cfg)
            d.setUp()
            N = d.mesh.N
            sub = np.sort(np.random.default_rng(dim).choice(N, N // 5, replace=False))
            d.mesh.set_dirichlet_nodes(sub)  # arbitrary Dirichlet set: filtered rows are not boxes
            mt = pa.MatFS()
            mt.setDomain(d)
            mt.build(buildOperators=False)
            out += [mt.K, mt.Krhs, mt.Rw]
        cfg = {"domain": {"ngl": 4, "box-mesh": {"nelem": [3, 3], "lower": [0, 0], "upper": [1, 1]}},
               "boundary-conditions": {"no-slip": {"up": [1, 0], "down": [0, 0], "left": [0, 0], "right": [0, 0]}}}
        dns = pa.Domain()
        dns.configure(cfg)
        dns.setUp()
        mns = pa.MatNS()
        mns.setDomain(dns)
        mns.build()
        out += [mns.K, mns.Krhs, mns.Rw, mns.Kfs, mns.Krhsfs, mns.Rwfs, mns.getKplusKfs(), mns.Rdfs]
        return out

    built = {}
    try:
        set_value_layout(lay)
        for host in (1, 0):
            os.environ["KLE_HOST_PATTERN"] = str(host)
            built[host] = build_all()
    finally:
        os.environ.pop("KLE_HOST_PATTERN", None)
        set_value_layout(old_lay)
    for A0, A1 in zip(built[1], built[0]):
        assert A0.isStructured() == A1.isStructured()
        for u, v in zip(A0.getValuesCSR(), A1.getValuesCSR()):
            np.testing.assert_array_equal(u, v)
        x = A0.createVecRight()
        x.setArray(rng.uniform(-1, 1, x.getLocalSize()))
        np.testing.assert_array_equal((A0 * x).getArray(), (A1 * x).getArray())


@pytest.mark.parametrize("mesh", ["box3", "box2", "umesh3"])
def test_batched_element_scratch_is_bitwise(pa, mesh, tmp_path):
    """K / Krhs / Rw assembled in element batches (KLE_ASM_SCRATCH_GB tiny:
    one element per batch, every gather continuing the stored partial sums)
    == the single-batch assembly, bitwise."""
    if mesh == "umesh3":
        from pynama_amd.meshgen import perturbed_box, write_gmsh
        V, Cc, F, T = perturbed_box(3, [3, 2, 2], seed=3)
        msh = str(tmp_path / "b.msh")
        write_gmsh(msh, 3, V, Cc, F, T)
        dom_cfg = {"ngl": 4, "gmsh-file": msh}
        bc = {"custom-func": {"name": "taylor_green3d"}}
    else:
        dim = 3 if mesh == "box3" else 2
        dom_cfg = {"ngl": 5 if dim == 3 else 6, "box-mesh": {"nelem": [3, 2, 3][:dim], "lower": [0] * dim,
                                                              "upper": [1] * dim}}
        bc = {"custom-func": {"name": "taylor_green3d" if dim == 3 else "taylor_green"}}
    out = {}
    try:
        for budget in (None, "0.000001"):
            if budget:
                os.environ["KLE_ASM_SCRATCH_GB"] = budget
            d = pa.Domain()
            d.configure({"domain": dom_cfg, "boundary-conditions": bc})
            d.setUp()
            mt = pa.MatFS()
            mt.setDomain(d)
            mt.build(buildOperators=False)
            out[budget] = [A.getValuesCSR() for A in (mt.K, mt.Krhs, mt.Rw)]
    finally:
        os.environ.pop("KLE_ASM_SCRATCH_GB", None)
    for a, b in zip(out[None], out["0.000001"]):
        for u, v in zip(a, b):
            np.testing.assert_array_equal(u, v)


def test_device_pattern_matches_host_unstructured(pa, tmp_path):
    """Unstructured meshes: the per-row sort/unique pattern kernel (k_upat) ==
    the host enumeration, bitwise, for K / Krhs / Rw (boundary and random
    Dirichlet sets), the operators and the no-slip matrices (2-D wall)."""
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    V, Cc, F, T = perturbed_box(3, [3, 3, 2], seed=8)
    m3 = str(tmp_path / "u3.msh")
    write_gmsh(m3, 3, V, Cc, F, T)
    V2, C2, F2, T2 = perturbed_box(2, [4, 3], seed=9)
    m2 = str(tmp_path / "u2.msh")
    write_gmsh(m2, 2, V2, C2, F2, T2)
    rng = np.random.default_rng(21)

    def build_all():
        out = []
        d = pa.Domain()
        d.configure({"domain": {"ngl": 4, "gmsh-file": m3},
                     "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}})
        d.setUp()
        mt = pa.MatFS()
        mt.setDomain(d)
        mt.build()
        op = mt.getOperators()
        out += [mt.K, mt.Krhs, mt.Rw, op.Curl, op.SrT, op.DivSrT]
        d = pa.Domain()
        d.configure({"domain": {"ngl": 3, "gmsh-file": m3},
                     "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}})
        d.setUp()
        N = d.mesh.N
        d.mesh.set_dirichlet_nodes(np.sort(np.random.default_rng(5).choice(N, N // 4, replace=False)))
        mt = pa.MatFS()
        mt.setDomain(d)
        mt.build(buildOperators=False)
        out += [mt.K, mt.Krhs, mt.Rw]
        d = pa.Domain()
        d.configure({"domain": {"ngl": 4, "gmsh-file": m2}, "boundary-conditions": {"no-slip": {"down": [1, 0]}}})
        d.setUp()
        mn = pa.MatNS()
        mn.setDomain(d)
        mn.build()
        out += [mn.K, mn.Krhs, mn.Rw, mn.Kfs, mn.Krhsfs, mn.Rwfs, mn.getKplusKfs(), mn.Rdfs]
        return out

    built = {}
    try:
        for host in (1, 0):
            os.environ["KLE_HOST_PATTERN"] = str(host)
            built[host] = build_all()
    finally:
        os.environ.pop("KLE_HOST_PATTERN", None)
    for A0, A1 in zip(built[1], built[0]):
        for u, v in zip(A0.getValuesCSR(), A1.getValuesCSR()):
            np.testing.assert_array_equal(u, v)
        x = A0.createVecRight()
        x.setArray(rng.uniform(-1, 1, x.getLocalSize()))
        np.testing.assert_array_equal((A0 * x).getArray(), (A1 * x).getArray())


def test_fixed_iterations_continue_the_recurrence(pa):
    """kle_ksp_continue (the bench's timed region): W fixed iterations, then n
    more continuing the same recurrence == W + n iterations in one solve,
    bitwise, for single-reduction and pipelined CG (one rank); the iteration
    count of the continuation is n and the reason CONVERGED_ITS."""
    from pynama_amd.petsc import KSP, PC
    g = _golden("tg3d_p4")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    b = K.createVecLeft()
    b.setArray(np.random.default_rng(5).uniform(-1, 1, b.getLocalSize()))
    # (symmetric storage on bricks: the pipelined update gathers the split
    # product itself, k_pipe_iter_g -- a continued call starts from a complete
    # product, read by the same kernel)
    from pynama_amd.runtime import set_tuning
    # (ksp_sr_gather 2: the single-reduction update gathers the split product
    # too, k_sr_iter_g -- by default only from 2^17 node rows)
    for kt, spd, srg in (("cg", False, 1), ("pipecg", False, 1), ("pipecg", True, 1), ("cg", True, 1),
                         ("cg", True, 2)):
        set_tuning("ksp_sr_gather", srg)
        K.setOption(K.Option.SPD, spd)
        if spd:
            assert K.spmvKernel().startswith("k_nb_spmv_sym_brick<"), K.spmvKernel()
        ksp = KSP().create()
        ksp.setType(kt)
        pc = PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setCGSingleReduction(True)
        ksp.setOperators(K)
        x = K.createVecRight()
        ksp.setFixedIterations(17)
        ksp.solve(b, x)
        ref = x.getArray().copy()
        ksp.setFixedIterations(5)
        ksp.solve(b, x)
        ksp.solveContinue(b, x, 12)
        assert ksp.getIterationNumber() == 12 and ksp.getConvergedReason() == 4  # KSP_CONVERGED_ITS
        np.testing.assert_array_equal(x.getArray(), ref)
        y = K.createVecRight()
        with pytest.raises(pa.Error):
            ksp.solveContinue(b, y, 3)  # not the (b, x) of the last fixed solve
    set_tuning("ksp_sr_gather", 1)


@pytest.mark.parametrize("kt,knob,on", [("pipecg", "ksp_pipe_gather", 1), ("cg", "ksp_sr_gather", 2)])
def test_fused_gather_matches_separate(pa, kt, knob, on):
    """CG on box bricks: the split product's owned-row gather folded into the
    next update (pipelined: k_pipe_iter_g, tuning ksp_pipe_gather; single
    reduction, one rank: k_sr_iter_g with (A u, u) from the bricks' and the
    one-block rows' shares, ksp_sr_gather 2: at every size -- by default
    from 2^17 node rows) against the separate gather launch (0): the same
    iteration count within 2, solutions
    within 1e-9, both at rtol 1e-10 (true residual), and the oracle's CG
    within 1e-7."""
    from oracle import oracle as O
    from pynama_amd.petsc import KSP, PC
    from pynama_amd.runtime import set_tuning
    g = _golden("tg3d_p4")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.spmvKernel().startswith("k_nb_spmv_sym_brick<")
    b = K.createVecLeft()
    ba = np.random.default_rng(9).uniform(-1, 1, b.getLocalSize())
    b.setArray(ba)
    out = {}
    for fused in (on, 0):
        set_tuning(knob, fused)
        try:
            ksp = KSP().create()
            ksp.setType(kt)
            ksp.setCGSingleReduction(True)
            pc = PC()
            pc.setType("jacobi")
            ksp.setPC(pc)
            ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
            ksp.setOperators(K)
            x = K.createVecRight()
            ksp.solve(b, x)
            assert ksp.getConvergedReason() > 0
            assert ksp.getTrueRelativeResidual() <= 1.01e-10
            out[fused] = (ksp.getIterationNumber(), x.getArray().copy())
            # the products the solve timed: the bricks alone (with their (y, x)
            # shares for the single-reduction fold) and their own bytes, or K's
            if fused:
                assert ksp.getProductKernel() == ("k_nb_spmv_sym_brick<16,true,true>" if kt == "cg"
                                                  else "k_nb_spmv_sym_brick<16,true,false>")
                assert 0 < ksp.getProductBytes() < K.spmvBytes()
            else:
                assert ksp.getProductKernel() == K.spmvKernel() and ksp.getProductBytes() == K.spmvBytes()
        finally:
            set_tuning(knob, 1)
    assert abs(out[on][0] - out[0][0]) <= 2, (out[on][0], out[0][0])
    assert np.linalg.norm(out[on][1] - out[0][1]) <= 1e-9 * np.linalg.norm(out[0][1])
    ip, ix, d = K.getValuesCSR()
    A = O.CSR.from_arrays(ip, ix, d, int(ip.shape[0] - 1))
    xo, ito, _ = A.cg(ba, rtol=1e-10)
    assert np.linalg.norm(out[on][1] - xo) <= 1e-7 * np.linalg.norm(xo)


def test_config2_full_size_properties(pa):
    """BASELINE config 2 at full size (1,026,675 DoF, p = 4): size-independent
    properties of the device-assembled system.  PETSc's nonzero count
    (SURVEY 8), patterns from the device == the host enumeration (SpMV
    bitwise equal), symmetry and linearity of K, identity Dirichlet rows, and
    the Jacobi-CG solve to 1e-10 (true residual)."""
    cfg = {"domain": {"ngl": 5, "box-mesh": {"nelem": [20, 16, 16], "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    mats = {}
    try:
        for host in ("1", "0"):
            os.environ["KLE_HOST_PATTERN"] = host
            dom = pa.Domain()
            dom.configure(cfg)
            dom.setUp()
            mat = pa.MatFS()
            mat.setDomain(dom)
            mat.build(buildOperators=False)
            mats[host] = (dom, mat)
    finally:
        os.environ.pop("KLE_HOST_PATTERN", None)
    dom, mat = mats["0"]
    K = mat.K
    assert K.getSize()[0] == 1026675
    assert K.getInfo()["nz_used"] == 561335085
    assert K.isStructured() and mats["1"][1].K.isStructured()
    rng = np.random.default_rng(7)
    x, y = K.createVecRight(), K.createVecRight()
    xa, ya = rng.uniform(-1, 1, x.getLocalSize()), rng.uniform(-1, 1, y.getLocalSize())
    x.setArray(xa)
    y.setArray(ya)
    from pynama_amd.runtime import set_tuning
    # K keeps symmetric storage at this size; the bitwise pattern
    # comparison runs the full-storage kernel, the symmetric one to rounding
    assert K.isSymmetricStorage()
    for name in ("K", "Krhs", "Rw"):
        A0, A1 = getattr(mats["1"][1], name), getattr(mat, name)
        v = A0.createVecRight()
        v.setArray(rng.uniform(-1, 1, v.getLocalSize()))
        try:
            set_tuning("spmv_sym", 0)
            y0 = (A0 * v).getArray().copy()
            np.testing.assert_array_equal(y0, (A1 * v).getArray())
        finally:
            set_tuning("spmv_sym", 1)
        ys = (A1 * v).getArray()
        assert np.abs(ys - y0).max() <= 1e-13 * np.abs(y0).max(), name
    Ax, Ay = K * x, K * y
    s = x + y
    np.testing.assert_allclose((K * s).getArray(), Ax.getArray() + Ay.getArray(), rtol=1e-12, atol=1e-9)
    assert abs(y.dot(Ax) - x.dot(Ay)) <= 1e-12 * abs(y.dot(Ax))
    bn = np.array(sorted(dom.getNodesDirichlet()))
    idx = (bn[:, None] * 3 + np.arange(3)).ravel()
    np.testing.assert_array_equal(Ax.getArray()[idx], xa[idx])
    ksp = pa.petsc.KSP().create()
    ksp.setType("cg")
    ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=20000)
    ksp.setOperators(K)
    u = K.createVecRight()
    ksp.solve(Ax, u)
    assert ksp.getConvergedReason() > 0
    assert ksp.getTrueRelativeResidual() <= 2e-10


def test_fs_rd_is_preallocated_and_empty(pa):
    """MatFS.Rd in free slip: preallocated by preAlloc_Rd_Rw (mat_fs.py:54-94),
    never filled by buildFS, assembled with the rest (assembleAll): a
    [dim N x N] matrix named "Rd" with no stored entries, in the kle list."""
    g = _golden("tg2d_small")
    dom = _domain(pa, g)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    N = dom.getMesh().N
    Rd = mat.Rd
    assert Rd is not None and Rd.getName() == "Rd" and Rd in mat.kle
    assert Rd.getSize() == (2 * N, N)
    assert Rd.getInfo()["nz_used"] == 0
    x = Rd.createVecRight()
    x.setArray(np.random.default_rng(3).uniform(-1, 1, x.getLocalSize()))
    np.testing.assert_array_equal((Rd * x).getArray(), np.zeros(2 * N))
