"""Symmetric (SBAIJ-style upper-triangle) storage of the KLE K
(kle_mat_set_symmetric / Mat.setOption(SPD)).

The reference solves with the SPD K that MatFS.buildFS assembles
(mat_fs.py:150-192: free-free element blocks plus a unit Dirichlet diagonal;
kle_solver.py:33-37).  libkle keeps each row's blocks from its diagonal block
on and lets every stored block serve row i and, transposed, row j.
Tolerances (the products sum in another order than the full storage):
  * SpMV vs the full-storage kernel and vs the exported PETSc CSR:
    <= 1e-14 relative (2-norm), max|diff| <= 1e-13 * max|y|
  * CG: iterations within 2 of the oracle's Jacobi-CG, solution within 1e-7
  * the default kernel (spmv_sym_det 1: exact fixed-point transposed sums) is
    bitwise reproducible: repeated products and solves are identical.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def tiles():
    """The box tests here exercise the 128-row tile kernel (the brick kernel,
    default for one rank: test_gpu_brick.py); the tiles serve p = 6 and
    spmv_sym_brick 0.  Likewise the unstructured tests exercise the 64-row
    dictionary groups (graph bricks, default for one rank:
    test_gpu_gbrick.py), which serve graph partitions at N > 1."""
    import pynama_amd
    pynama_amd.load()
    from pynama_amd.runtime import set_tuning
    set_tuning("spmv_sym_brick", 0)
    set_tuning("spmv_gsym_brick", 0)
    yield
    set_tuning("spmv_sym_brick", 1)
    set_tuning("spmv_gsym_brick", 1)


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


KNOBS = ({}, {"spmv_sym_det": 0}, {"spmv_sym_waves": 16}, {"spmv_sym_waves": 16, "spmv_sym_det": 0},
         {"spmv_sym_xcd": 3}, {"spmv_sym_stpol": 1}, {"spmv_sym_stpol": 2}, {"spmv_sym_stpol": 3})
DEFAULTS = {"spmv_sym_det": 1, "spmv_sym_waves": 0, "spmv_sym_xcd": 0, "spmv_sym_stpol": 0}


@pytest.mark.parametrize("nelem,ngl", [([3, 2, 2], 5), ([12, 10, 6], 5), ([7, 5, 4], 3), ([6, 5, 3], 2),
                                       ([3, 4, 2], 6), ([1, 1, 1], 4), ([3, 3, 2], 7), ([2, 3, 3], 7)])
def test_symmetric_spmv_matches_full_storage_and_csr(pa, nelem, ngl):
    _, mat = _mat(pa, nelem, ngl)
    K = mat.K
    from pynama_amd.runtime import get_tuning
    # (assembled with symmetric storage from spmv_sym_min_rows node rows)
    assert K.isSymmetricStorage() == (K.getSize()[0] // 3 >= get_tuning("spmv_sym_min_rows"))
    K.setOption(K.Option.SPD, False)
    assert not K.isSymmetricStorage()
    x = K.createVecRight()
    xa = np.random.default_rng(11).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y0 = (K * x).getArray().copy()
    b0 = K.spmvBytes()
    K.setOption(K.Option.SPD, True)
    assert K.isSymmetricStorage()
    if ngl >= 5 and min(nelem) >= 2:  # (tiny meshes: the tile partials outweigh the halved values)
        assert K.spmvBytes() < 0.75 * b0
    ip, ix, d = K.getValuesCSR()
    yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
    from pynama_amd.runtime import set_tuning
    try:
        # the x-in-LDS tile kernel k_nb_spmv_sym_xl under every knob of KNOBS
        # (fixed-point and fp64-atomic transposed sums, 8 or 16 waves)
        for knobs in KNOBS:
            for k, v in knobs.items():
                set_tuning(k, v)
            name = K.spmvKernel()
            assert name.startswith("k_nb_spmv_sym_"), name
            y1 = (K * x).getArray().copy()
            for _ in range(2):
                y2 = (K * x).getArray().copy()
                for ref in (y0, yh):
                    assert np.linalg.norm(y2 - ref) <= 1e-14 * np.linalg.norm(ref), knobs
                    assert np.abs(y2 - ref).max() <= 1e-13 * np.abs(ref).max(), knobs
                if "true" in name:  # fixed-point transposed sums: bitwise reproducible
                    np.testing.assert_array_equal(y2, y1)
            for k, v in DEFAULTS.items():
                set_tuning(k, v)
    finally:
        for k, v in DEFAULTS.items():
            set_tuning(k, v)
    # partial slots aligned to 128-B lines and written whole (build knob
    # spmv_sym_align): the same sums in the same order, bitwise
    set_tuning("spmv_sym_align", 1)
    try:
        K.setOption(K.Option.SPD, True)
        ya = (K * x).getArray().copy()
    finally:
        set_tuning("spmv_sym_align", 0)
    K.setOption(K.Option.SPD, True)
    np.testing.assert_array_equal(ya, (K * x).getArray())
    # tile shapes: 8 x 2 x 4 (64 rows; spmv_sym_tile64 1 forces them where two
    # workgroups fit a CU, the default picks them for parts of < 640 128-row
    # tiles -- every matrix here) and never (2: 8 x 4 x 4, or 8 x 8 x 2 at
    # p >= 5): the same products to rounding, each bitwise reproducible
    shapes = {}
    for mode in (1, 2):
        set_tuning("spmv_sym_tile64", mode)
        try:
            K.setOption(K.Option.SPD, True)
            name = K.spmvKernel()
            ys = (K * x).getArray().copy()
            np.testing.assert_array_equal((K * x).getArray(), ys)
            for ref in (y0, yh):
                assert np.linalg.norm(ys - ref) <= 1e-14 * np.linalg.norm(ref), name
                assert np.abs(ys - ref).max() <= 1e-13 * np.abs(ref).max(), name
            shapes[mode] = name
        finally:
            set_tuning("spmv_sym_tile64", 0)
    assert ",8,2>" in shapes[1] or shapes[1] == "k_nb_spmv_sym_xl<8,true,2,4>+k_nb_sym_gather<8,2,4>", shapes
    assert shapes[2] in ("k_nb_spmv_sym_xl<8,true,4,4>+k_nb_sym_gather<8,4,4>",
                         "k_nb_spmv_sym_xl<8,true,8,2>+k_nb_sym_gather<8,8,2>",
                         "k_nb_spmv_sym_xl<16,true,8,2>+k_nb_sym_gather<8,8,2>"), shapes
    K.setOption(K.Option.SPD, True)
    K.setOption(K.Option.SPD, False)
    assert not K.isSymmetricStorage()
    np.testing.assert_array_equal((K * x).getArray(), y0)


def test_symmetric_spmv_edge_inputs(pa):
    """Zero x gives exactly zero; a NaN in x propagates (the fixed-point path
    must not turn it into a finite number); huge and tiny scales keep their
    relative accuracy (the per-tile scale follows max|x|)."""
    _, mat = _mat(pa, [4, 3, 3], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.isSymmetricStorage()
    x = K.createVecRight()
    x.setArray(np.zeros(x.getLocalSize()))
    assert not np.any((K * x).getArray())
    xa = np.random.default_rng(3).uniform(-1, 1, x.getLocalSize())
    ip, ix, d = K.getValuesCSR()
    A = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa)))
    for scale in (1e-200, 1e-8, 1.0, 1e150):
        x.setArray(xa * scale)
        y = (K * x).getArray()
        yh = A @ (xa * scale)
        assert np.linalg.norm(y - yh) <= 1e-14 * np.linalg.norm(yh), scale
    xb = xa.copy()
    xb[len(xb) // 2] = np.nan
    x.setArray(xb)
    y = (K * x).getArray()
    assert np.isnan(y).any()


def test_symmetric_cg_is_reproducible(pa):
    """With the fixed-point transposed sums (default) two solves of the same
    system take the same iterations and give bitwise the same solution -- the
    second with the update kernel's nontemporal variant (upd_nt 1, the
    default from 2M entries: only cache hints differ)."""
    from pynama_amd.runtime import get_tuning, set_tuning
    assert get_tuning("spmv_sym_det") == 1
    _, mat = _mat(pa, [6, 5, 4], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    b = K.createVecLeft()
    b.setArray(np.random.default_rng(7).uniform(-1, 1, b.getLocalSize()))
    out = []
    for nt in (0, 1):
        set_tuning("upd_nt", nt)
        ksp = pa.petsc.KSP().create()
        ksp.setType("cg")
        pc = pa.petsc.PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
        ksp.setCGSingleReduction(True)
        ksp.setOperators(K)
        x = K.createVecRight()
        try:
            ksp.solve(b, x)
        finally:
            set_tuning("upd_nt", 2)
        out.append((ksp.getIterationNumber(), x.getArray().copy()))
    assert out[0][0] == out[1][0]
    np.testing.assert_array_equal(out[0][1], out[1][1])


def test_duplicate_of_symmetric_matrix_owns_its_storage(pa):
    """Mat.duplicate(copy=True) of a matrix with symmetric storage gets its
    own copy (rebuilt from the copied values): axpy on the duplicate drops
    only the duplicate's, K keeps multiplying correctly, and destroying both
    frees each buffer once (the copy used to share K's buffers)."""
    _, mat = _mat(pa, [4, 3, 3], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    x = K.createVecRight()
    xa = np.random.default_rng(5).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y0 = (K * x).getArray().copy()
    B = K.duplicate(copy=True)
    assert B.isSymmetricStorage() and K.isSymmetricStorage()
    np.testing.assert_array_equal((B * x).getArray(), y0)
    B.axpy(1.0, K)  # B = 2 K (drops B's symmetric copy)
    assert not B.isSymmetricStorage() and K.isSymmetricStorage()
    np.testing.assert_array_equal((K * x).getArray(), y0)
    yb = (B * x).getArray()
    assert np.abs(yb - 2 * y0).max() <= 1e-13 * np.abs(y0).max()
    Z = K.duplicate(copy=False)  # zero values: full storage, product 0
    assert not Z.isSymmetricStorage()
    assert not np.any((Z * x).getArray())
    B.destroy()
    Z.destroy()
    np.testing.assert_array_equal((K * x).getArray(), y0)


def test_symmetric_cg_matches_oracle(pa):
    """Jacobi-CG on the symmetric storage (single-reduction and pipelined)
    against the oracle's CG on the exported CSR of the same K."""
    from pynama_amd import fields
    dom, mat = _mat(pa, [6, 5, 4], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.isSymmetricStorage()
    f = fields.get("taylor_green3d")
    alpha = f.alpha(0.02, 0.0)
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    vort = mat.Rw.createVecRight()
    vort.setArray(f.vorticity(dom.getFullCoordArray(), alpha))
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, 0.02)
    b = sol.rhs(vort).copy()
    ip, ix, d = K.getValuesCSR()
    Ko = O.CSR.from_arrays(ip, ix, d, len(ip) - 1)
    xo, it_o, _ = Ko.cg(b.getArray(), rtol=1e-10, jacobi=True)
    for typ, single in (("cg", True), ("cg", False), ("pipecg", True)):
        ksp = pa.petsc.KSP().create()
        ksp.setType(typ)
        pc = pa.petsc.PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
        ksp.setCGSingleReduction(single)
        ksp.setOperators(K)
        x = K.createVecRight()
        ksp.solve(b, x)
        assert ksp.getConvergedReason() > 0
        assert abs(ksp.getIterationNumber() - it_o) <= (4 if typ == "pipecg" else 2), (typ, single)
        assert ksp.getTrueRelativeResidual() <= 1.01e-10
        assert np.linalg.norm(x.getArray() - xo) <= 1e-7 * np.linalg.norm(xo)


def test_symmetric_storage_follows_value_changes(pa):
    """diagonalScale changes the values: the symmetric copy is dropped and the
    product follows the new values (full storage)."""
    _, mat = _mat(pa, [4, 3, 3], 5)
    K = mat.K
    K.setOption(K.Option.SYMMETRIC, True)
    assert K.isSymmetricStorage()
    s = K.createVecLeft()
    s.setArray(np.random.default_rng(2).uniform(0.5, 2.0, s.getLocalSize()))
    K.diagonalScale(s, None)
    assert not K.isSymmetricStorage()
    x = K.createVecRight()
    xa = np.random.default_rng(5).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    ip, ix, d = K.getValuesCSR()
    yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
    y = (K * x).getArray()
    assert np.abs(y - yh).max() <= 1e-13 * np.abs(yh).max()


def test_symmetric_storage_refused_where_it_does_not_apply(pa):
    """Rw (not symmetric) and a 2-D K (2x2 blocks) keep the full storage;
    setOption leaves them as they are, as PETSc ignores options a format does
    not use.  (p = 6 is supported since round 3: its 20 x 20 x 8-node tile
    regions take one 16-wave workgroup per CU.)"""
    _, mat = _mat(pa, [3, 3, 2], 4)
    for A in (mat.Rw,):
        A.setOption(A.Option.SPD, True)
        assert not A.isSymmetricStorage()
    cfg = {"domain": {"ngl": 4, "box-mesh": {"nelem": [5, 4], "lower": [0, 0], "upper": [1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    m2 = pa.MatFS()
    m2.setDomain(dom)
    m2.build(buildOperators=False)
    m2.K.setOption(m2.K.Option.SPD, True)
    assert not m2.K.isSymmetricStorage()
    _, m6 = _mat(pa, [2, 2, 2], 7)
    m6.K.setOption(m6.K.Option.SPD, True)
    assert m6.K.isSymmetricStorage()
    assert m6.K.spmvKernel().startswith("k_nb_spmv_sym_xl<")  # (P = 6: the tight tile region fits the LDS)


def test_assembly_turns_symmetric_storage_on_from_the_threshold(pa):
    from pynama_amd.runtime import get_tuning, set_tuning
    old = get_tuning("spmv_sym_min_rows")
    try:
        set_tuning("spmv_sym_min_rows", 0)
        _, mat = _mat(pa, [3, 2, 2], 5)
        assert mat.K.isSymmetricStorage()
        assert not mat.Rw.isSymmetricStorage()
        set_tuning("spmv_sym", 0)
        _, mat = _mat(pa, [3, 2, 2], 5)
        assert not mat.K.isSymmetricStorage()
    finally:
        set_tuning("spmv_sym", 1)
        set_tuning("spmv_sym_min_rows", old)


# ---- unstructured (graph-numbered) K: k_nb_spmv_gsym + k_nb_gsym_gather ----

def _umat(pa, tmp_path, nelem, ngl, seed=5):
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    dim = len(nelem)
    V, Cc, F, T = perturbed_box(dim, nelem, seed=seed)
    path = tmp_path / f"m{seed}.msh"
    write_gmsh(path, dim, V, Cc, F, T)
    cfg = {"domain": {"ngl": ngl, "gmsh-file": str(path)},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d" if dim == 3 else "taylor_green"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    return dom, mat


@pytest.mark.parametrize("nelem,ngl", [([3, 2, 2], 5), ([6, 5, 4], 5), ([4, 3, 3], 3), ([5, 4, 3], 2),
                                       ([2, 2, 2], 7), ([1, 1, 1], 4)])
def test_unstructured_symmetric_spmv_matches_full_storage_and_csr(pa, tmp_path, nelem, ngl):
    """Gmsh hexes (perturbed, rotated, shuffled; Hilbert-numbered nodes): the
    upper-triangle storage with per-group dictionaries equals the
    column-dictionary full-storage kernel and the exported PETSc CSR to
    rounding, and repeated products are bitwise equal (fixed-point sums)."""
    from pynama_amd.runtime import set_tuning
    _, mat = _umat(pa, tmp_path, nelem, ngl)
    K = mat.K
    assert not K.isStructured()
    assert not K.isSymmetricStorage()  # below spmv_sym_min_rows: full storage
    x = K.createVecRight()
    xa = np.random.default_rng(11).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y0 = (K * x).getArray().copy()
    b0 = K.spmvBytes()
    K.setOption(K.Option.SPD, True)
    assert K.isSymmetricStorage()
    if ngl >= 5 and min(nelem) >= 4:
        assert K.spmvBytes() < 0.8 * b0
    ip, ix, d = K.getValuesCSR()
    yh = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa))) @ xa
    try:
        # groups of 16 / 8 rows, one launch or the groups split over two
        # (the larger dictionaries in a second launch with more LDS)
        # (align: each group's partials from a 128-B line, written whole)
        for rows, waves, split, align in ((64, 0, 0, 0), (64, 8, 0, 0), (32, 16, 0, 0), (32, 8, 0, 0),
                                          (16, 0, 0, 0), (8, 0, 0, 0), (128, 0, 0, 0), (64, 0, 120, 0),
                                          (32, 8, 60, 0), (8, 0, 20, 0), (128, 0, 200, 0), (64, 0, 0, 1),
                                          (32, 8, 60, 1)):
            set_tuning("spmv_gsym_rows", rows)
            set_tuning("spmv_gsym_waves", waves)
            set_tuning("spmv_gsym_split", split)
            set_tuning("spmv_sym_align", align)
            K.setOption(K.Option.SPD, True)
            for det in (1, 0):
                set_tuning("spmv_sym_det", det)
                name = K.spmvKernel()
                want = f"k_nb_spmv_gsym<{'true' if det else 'false'},{rows},{waves or (16 if rows >= 64 else 8)}>"
                assert name.startswith(want), name
                y1 = (K * x).getArray().copy()
                for _ in range(2):
                    y2 = (K * x).getArray().copy()
                    for ref in (y0, yh):
                        assert np.linalg.norm(y2 - ref) <= 1e-14 * np.linalg.norm(ref), (rows, split, det)
                        assert np.abs(y2 - ref).max() <= 1e-13 * np.abs(ref).max(), (rows, split, det)
                    if det:
                        np.testing.assert_array_equal(y2, y1)
                if det and rows == 64 and not split and not align:
                    # partial-store cache policies (spmv_gsym_stpol; default 2, sc1): the same bits
                    for pol in (0, 1, 3):
                        set_tuning("spmv_gsym_stpol", pol)
                        try:
                            np.testing.assert_array_equal((K * x).getArray(), y1)
                        finally:
                            set_tuning("spmv_gsym_stpol", 2)
    finally:
        set_tuning("spmv_sym_det", 1)
        set_tuning("spmv_sym_align", 0)
        set_tuning("spmv_gsym_rows", 64)
        set_tuning("spmv_gsym_waves", 0)
        set_tuning("spmv_gsym_split", 0)
    K.setOption(K.Option.SPD, False)
    assert not K.isSymmetricStorage()
    np.testing.assert_array_equal((K * x).getArray(), y0)


def test_unstructured_symmetric_spmv_edge_inputs(pa, tmp_path):
    """Zero x gives exactly zero, a NaN propagates, and the per-group scale
    follows max|x| from 1e-200 to 1e150."""
    _, mat = _umat(pa, tmp_path, [4, 3, 3], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.isSymmetricStorage()
    x = K.createVecRight()
    x.setArray(np.zeros(x.getLocalSize()))
    assert not np.any((K * x).getArray())
    xa = np.random.default_rng(3).uniform(-1, 1, x.getLocalSize())
    ip, ix, d = K.getValuesCSR()
    A = sp.csr_matrix((d, ix, ip), shape=(len(ip) - 1, len(xa)))
    for scale in (1e-200, 1e-8, 1.0, 1e150):
        x.setArray(xa * scale)
        y = (K * x).getArray()
        yh = A @ (xa * scale)
        assert np.linalg.norm(y - yh) <= 1e-14 * np.linalg.norm(yh), scale
    xb = xa.copy()
    xb[len(xb) // 3] = np.nan
    x.setArray(xb)
    assert np.isnan((K * x).getArray()).any()


def test_unstructured_symmetric_cg_matches_oracle(pa, tmp_path):
    """Jacobi-CG through the graph symmetric storage (single-reduction with
    the gather's fused (w, u) partials, classic, pipelined) against the
    oracle's CG on the exported CSR; two solves bitwise equal."""
    from pynama_amd import fields
    dom, mat = _umat(pa, tmp_path, [6, 5, 4], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    assert K.isSymmetricStorage()
    f = fields.get("taylor_green3d")
    alpha = f.alpha(0.02, 0.0)
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    vort = mat.Rw.createVecRight()
    vort.setArray(f.vorticity(dom.getFullCoordArray(), alpha))
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, 0.02)
    b = sol.rhs(vort).copy()
    ip, ix, d = K.getValuesCSR()
    Ko = O.CSR.from_arrays(ip, ix, d, len(ip) - 1)
    xo, it_o, _ = Ko.cg(b.getArray(), rtol=1e-10, jacobi=True)
    for typ, single in (("cg", True), ("cg", True), ("cg", False), ("pipecg", True)):
        ksp = pa.petsc.KSP().create()
        ksp.setType(typ)
        pc = pa.petsc.PC()
        pc.setType("jacobi")
        ksp.setPC(pc)
        ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=10000)
        ksp.setCGSingleReduction(single)
        ksp.setOperators(K)
        x = K.createVecRight()
        ksp.solve(b, x)
        assert ksp.getConvergedReason() > 0
        assert abs(ksp.getIterationNumber() - it_o) <= (4 if typ == "pipecg" else 2), (typ, single)
        assert ksp.getTrueRelativeResidual() <= 1.01e-10
        assert np.linalg.norm(x.getArray() - xo) <= 1e-7 * np.linalg.norm(xo)
        if typ == "cg" and single:
            if "first" in locals():
                np.testing.assert_array_equal(x.getArray(), first)
            first = x.getArray().copy()


def test_unstructured_symmetric_storage_refused_where_it_does_not_apply(pa, tmp_path):
    """Rw (not symmetric) and a 2-D unstructured K (2x2 blocks) keep the full
    storage; K of the same mesh takes the graph storage."""
    _, mat = _umat(pa, tmp_path, [3, 3, 2], 4)
    mat.Rw.setOption(mat.Rw.Option.SPD, True)
    assert not mat.Rw.isSymmetricStorage()
    mat.K.setOption(mat.K.Option.SPD, True)
    assert mat.K.isSymmetricStorage()
    _, m2 = _umat(pa, tmp_path, [5, 4], 4, seed=6)
    m2.K.setOption(m2.K.Option.SPD, True)
    assert not m2.K.isSymmetricStorage()


def test_unstructured_duplicate_owns_its_symmetric_storage(pa, tmp_path):
    _, mat = _umat(pa, tmp_path, [4, 3, 3], 5)
    K = mat.K
    K.setOption(K.Option.SPD, True)
    x = K.createVecRight()
    x.setArray(np.random.default_rng(5).uniform(-1, 1, x.getLocalSize()))
    y0 = (K * x).getArray().copy()
    B = K.duplicate(copy=True)
    assert B.isSymmetricStorage()
    np.testing.assert_array_equal((B * x).getArray(), y0)
    B.axpy(1.0, K)
    assert not B.isSymmetricStorage() and K.isSymmetricStorage()
    np.testing.assert_array_equal((K * x).getArray(), y0)
    assert np.abs((B * x).getArray() - 2 * y0).max() <= 1e-13 * np.abs(y0).max()
    B.destroy()
    np.testing.assert_array_equal((K * x).getArray(), y0)
