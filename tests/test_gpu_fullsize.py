"""BASELINE config 2 at full size against the oracle.

Config 2: box [0,1]^3, nelem [20,16,16], ngl 5 (p = 4), Taylor-Green-3D
Dirichlet data on every face: 342,225 nodes, 1,026,675 DoF, K 561,335,085
nonzeros.  The device system (libkle: device patterns, MFMA element kernel,
node-block gather) is compared with `oracle/kle_oracle.c`'s assembly of the
same mesh, which restates MatFS.buildFS (mat_fs.py:131-192) cell by cell in
ascending cell order (OpenMP over elements and disjoint row ranges; bitwise the
serial loop):

  * connectivity (reference local order, via the golden loc2lat table) and the
    Dirichlet node set: bit-exact;
  * K / Krhs / Rw: indptr and indices bit-exact, values <= 1e-12 * max|ref|;
  * b = Rw w + Krhs u_bc (KleSolver.solve, kle_solver.py:33-37): <= 1e-12 *
    max|b|;
  * the device CG solution (rtol 1e-10, the north star's "same residual as
    PETSc KSP within 1e-10"): true residual with the ORACLE's K and b <=
    1.05e-10 (the device stops on its recursive residual; 5 % allows the
    recursive/true drift), and ||u - u_oracle|| / ||u_oracle|| <= 1e-7 against
    the oracle's Jacobi-CG at rtol 1e-10 (SURVEY 8(d) "Convergence").

Runs for ~2-3 minutes on the GPU box (oracle: ~35 s of element matrices on 16
host threads, ~70 s of CG); progress goes to stderr so a long step is visible.
"""
import os
import sys
import time

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
NELEM, NGL = [20, 16, 16], 5


def _log(t0, msg):
    sys.__stderr__.write(f"[config2-parity {time.perf_counter() - t0:7.1f}s] {msg}\n")
    sys.__stderr__.flush()


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


@pytest.mark.timeout(900)
def test_config2_full_size_matches_oracle(pa):
    from pynama_amd import fields
    t0 = time.perf_counter()
    cfg = {"domain": {"ngl": NGL, "box-mesh": {"nelem": NELEM, "lower": [0, 0, 0], "upper": [1, 1, 1]}},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    f = fields.get("taylor_green3d")
    nu = 0.01 / 0.5  # taylor-green3d.yaml: rho 0.5, mu 0.01
    alpha = f.alpha(nu, 0.0)
    vort = mat.Rw.createVecRight()
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, nu)
    ksp = sol.getKSP()
    ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=20000)
    _log(t0, "device system assembled")

    # ---- oracle mesh: connectivity, coordinates, Dirichlet set
    om = O.BoxMesh(3, NELEM, [0, 0, 0], [1, 1, 1], NGL)
    assert om.N == 342225
    loc2lat = np.load(os.path.join(G, "case_tg3d_p4.npz"))["loc2lat"]
    assert loc2lat.shape == (NGL ** 3, 3)
    my_idx = (loc2lat * NGL ** np.arange(3)).sum(1)
    np.testing.assert_array_equal(dom.mesh.conn()[:, my_idx], om.conn())
    xo = om.coords()
    np.testing.assert_allclose(dom.getFullCoordArray().reshape(-1, 3), xo, rtol=0, atol=1e-15)
    on_bd = ((xo == 0.0) | (xo == 1.0)).any(axis=1)
    np.testing.assert_array_equal(np.array(sorted(dom.getNodesDirichlet())), np.flatnonzero(on_bd))
    _log(t0, "connectivity bit-exact, coordinates, Dirichlet set equal")

    vort.setArray(f.vorticity(xo, alpha))
    b = sol.rhs(vort).copy()
    bd = b.getArray().copy()
    sol.solve(vort)
    assert ksp.getConvergedReason() > 0
    u_dev = vel.getArray().copy()
    its_dev = ksp.getIterationNumber()
    _log(t0, f"device CG: {its_dev} iterations, device true residual {ksp.getTrueRelativeResidual():.3e}")

    # ---- the box symmetric SpMV on bricks (default, one rank): its plan, and
    # the 128-row tile kernel on the same K and u to 1e-14 (both exact
    # fixed-point transposed sums, other scales and summation orders)
    from pynama_amd.runtime import set_tuning
    K = mat.K
    assert K.isSymmetricStorage() and K.spmvKernel().startswith("k_nb_spmv_sym_brick"), K.spmvKernel()
    bk = K.getSymmetricBricks()
    assert 0 < bk["bricks"] <= 256 and min(bk["dims"]) >= 1 and bk["region_entries_per_row"] < 2.5, bk
    _log(t0, f"bricks: {bk}")
    y1 = (K * vel).getArray().copy()
    np.testing.assert_array_equal((K * vel).getArray(), y1)
    set_tuning("spmv_sym_brick", 0)
    try:
        K.setOption(K.Option.SPD, True)
        assert K.spmvKernel().startswith("k_nb_spmv_sym_xl"), K.spmvKernel()
        yt = (K * vel).getArray()
        assert np.linalg.norm(yt - y1) <= 1e-14 * np.linalg.norm(y1)
    finally:
        set_tuning("spmv_sym_brick", 1)
        K.setOption(K.Option.SPD, True)
    np.testing.assert_array_equal((K * vel).getArray(), y1)
    del yt
    # ---- where the value array lies does not set the speed (VERDICT r04
    # item 1: the 128-row tiles' mid-stream partial stores made the product
    # bimodal over placements, 424-491 us, profiles/r04/ab/values_placement.jsonl).
    # The same offsets, twice each in turn; each placement's faster pass of 100
    # products (windows of 20 carry +-2.5 % of timing noise on one unmoved
    # array, of 200 +-0.2 %: profiles/r05/placement_noise.jsonl); <= 3 % spread.
    # All offsets within ONE allocation (moveValues(fresh=False): the same
    # physical pages); a fresh allocation of the same size moves every
    # offset together by up to 4 % (its pages: 406-424 us over allocations,
    # profiles/r05/placement_*.jsonl), which no layout of the values changes.
    # (Offsets are multiples of the 128-B cache line, as every allocation is:
    # a base 64 B off the line splits each 16-block chunk load over two lines
    # and cost 16 %, 479 vs 413 us, in the r05 run of this test.)
    from pynama_amd.runtime import get_ctx
    ctx = get_ctx()
    yv = K.createVecLeft()
    offsets = [0, 256, 4096, 65536, 1 << 20, 2101248, 0, (3 << 20) + 384]
    times = {}
    for _ in range(2):
        for k, off in enumerate(offsets):
            K.moveValues(off, fresh=False)
            K.mult(vel, yv)
            np.testing.assert_array_equal(yv.getArray(), y1)
            for _ in range(5):
                K.mult(vel, yv)
            ctx.synchronize()
            ctx.set_profiling(True, only="spmv")
            ctx.reset_stats()
            for _ in range(100):
                K.mult(vel, yv)
            ctx.synchronize()
            c, ms = ctx.kernel_stats("spmv")
            ctx.set_profiling(False)
            times.setdefault(k, []).append(1e3 * ms / c)
    best = [min(v) for v in times.values()]
    spread = (max(best) - min(best)) / min(best)
    _log(t0, f"value placements {offsets}: SpMV {[round(b, 1) for b in best]} us, spread {spread:.3f}")
    assert spread <= 0.03, (best, spread)
    del y1, yv

    # ---- oracle assembly (mat_fs.py:131-192)
    Ko, Kro, Rwo = om.assemble_fs(on_bd.astype(np.uint8))
    _log(t0, f"oracle assembly: K {Ko.nnz} nnz, Krhs {Kro.nnz}, Rw {Rwo.nnz}")
    assert Ko.nnz == 561335085
    for name, ref in (("K", Ko), ("Krhs", Kro), ("Rw", Rwo)):
        ip, ix, d = getattr(mat, name).getValuesCSR()
        np.testing.assert_array_equal(ip, ref.indptr, err_msg=name)
        np.testing.assert_array_equal(ix, ref.indices, err_msg=name)
        err = float(np.abs(d - ref.data).max())
        assert err <= 1e-12 * float(np.abs(ref.data).max()), (name, err)
        del ip, ix, d
        _log(t0, f"{name}: pattern bit-exact, max|diff| {err:.3e}")

    # ---- b = Rw w + Krhs u (KleSolver.solve, kle_solver.py:33-37)
    ubc = np.zeros(om.N * 3)
    bn = np.flatnonzero(on_bd)
    ubc[(bn[:, None] * 3 + np.arange(3)).ravel()] = f.velocity(xo[bn], alpha)
    bo = Rwo.mult(f.vorticity(xo, alpha)) + Kro.mult(ubc)
    del Kro, Rwo, ref
    berr = float(np.abs(bd - bo).max())
    assert berr <= 1e-12 * float(np.abs(bo).max()), berr

    # ---- solution: true residual with the oracle's operator, and the oracle's CG
    res = float(np.linalg.norm(bo - Ko.mult(u_dev)) / np.linalg.norm(bo))
    _log(t0, f"b max|diff| {berr:.3e}; true residual of the device solution with the oracle's K, b: {res:.3e}")
    assert res <= 1.05e-10
    uo, its_o, rr_o = Ko.cg(bo, rtol=1e-10, jacobi=True)
    rel = float(np.linalg.norm(u_dev - uo) / np.linalg.norm(uo))
    _log(t0, f"oracle CG: {its_o} iterations (true residual {rr_o:.3e}); ||u - u_oracle||/||u_oracle|| {rel:.3e}")
    assert rr_o <= 1.05e-10
    assert rel <= 1e-7
    assert abs(its_dev - its_o) <= 4


@pytest.mark.timeout(600)
def test_unstructured_full_size_dictionary_spmv_is_bitwise(pa, tmp_path):
    """The 1M-DoF unstructured bench mesh (config 5's path at config 2's size:
    [20,16,16] perturbed / rotated / shuffled hexes through Gmsh, p = 4): the
    column-dictionary SpMV that runs by default there (k_nb_spmv_dict; groups
    of up to ~1,050 distinct nodes, built at matrix creation) equals the
    bcol-stream kernel bitwise for K, Rw and Krhs, and the solve converges as
    the bench records (891 iterations at rtol 1e-10)."""
    from pynama_amd import fields
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    from pynama_amd.runtime import set_tuning
    t0 = time.perf_counter()
    V, Cc, F, T = perturbed_box(3, NELEM, seed=5)
    path = tmp_path / "mesh.msh"
    write_gmsh(path, 3, V, Cc, F, T)
    cfg = {"domain": {"ngl": NGL, "gmsh-file": str(path)},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    _log(t0, "unstructured system assembled")
    # (K's default product is the symmetric storage on graph bricks, which
    # spmv_dict does not touch: its full storage is compared with spmv_sym 0,
    # and the graph bricks with that to rounding)
    assert mat.K.isSymmetricStorage() and mat.K.spmvKernel().startswith("k_nb_spmv_gsym_brick<")
    for name in ("K", "Rw", "Krhs"):
        A = getattr(mat, name)
        assert not A.isStructured()
        x = A.createVecRight()
        x.setArray(np.random.default_rng(7).uniform(-1, 1, x.getLocalSize()))
        try:
            ys = (A * x).getArray().copy()
            set_tuning("spmv_sym", 0)
            y1 = (A * x).getArray().copy()
            set_tuning("spmv_dict", 0)
            y0 = (A * x).getArray().copy()
        finally:
            set_tuning("spmv_dict", 1)
            set_tuning("spmv_sym", 1)
        np.testing.assert_array_equal(y1, y0, err_msg=name)
        if name == "K":
            assert np.linalg.norm(ys - y1) <= 1e-14 * np.linalg.norm(y1)
        else:
            np.testing.assert_array_equal(ys, y1, err_msg=name)
    _log(t0, "K / Rw / Krhs: dictionary SpMV == column-stream SpMV, bitwise; K's graph bricks == both to rounding")
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    f = fields.get("taylor_green3d")
    nu = 0.01 / 0.5
    vort = mat.Rw.createVecRight()
    vort.setArray(f.vorticity(dom.getFullCoordArray(), f.alpha(nu, 0.0)))
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, nu)
    ksp = sol.getKSP()
    ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=20000)
    sol.solve(vort)
    assert ksp.getConvergedReason() > 0
    assert ksp.getTrueRelativeResidual() <= 1.05e-10
    assert abs(ksp.getIterationNumber() - 891) <= 4
    _log(t0, f"solve: {ksp.getIterationNumber()} iterations")


@pytest.mark.timeout(900)
def test_unstructured_full_size_matches_oracle(pa, tmp_path):
    """Config 5's path at config 2's size against the oracle: the bench's
    1M-DoF unstructured mesh ([20,16,16] perturbed / rotated / shuffled hexes
    through Gmsh, p = 4) assembled on the device (kle_umesh.cpp numbering,
    Hilbert order; column-dictionary SpMV) and by `oracle.UMesh` (nodes
    identified by coordinates, C assembly of mat_fs.py:131-192 in ascending
    cell order).  Under the node map: the Dirichlet set equal; K, Krhs and Rw
    equal as operators (products with two random vectors <= 1e-12 of scale);
    b <= 1e-12; the device solution's true residual with the oracle's K and b
    <= 1.05e-10 and within 1e-7 of the oracle's Jacobi-CG solution."""
    from pynama_amd import fields
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    t0 = time.perf_counter()
    V, Cc, F, T = perturbed_box(3, NELEM, seed=5)
    path = tmp_path / "mesh.msh"
    write_gmsh(path, 3, V, Cc, F, T)
    cfg = {"domain": {"ngl": NGL, "gmsh-file": str(path)},
           "boundary-conditions": {"custom-func": {"name": "taylor_green3d"}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build(buildOperators=False)
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    ksp = sol.getKSP()
    ksp.setTolerances(rtol=1e-10, atol=0.0, max_it=20000)
    f = fields.get("taylor_green3d")
    alpha = f.alpha(0.01 / 0.5, 0.0)
    xd = dom.getFullCoordArray().reshape(-1, 3)
    vort = mat.Rw.createVecRight()
    vort.setArray(f.vorticity(xd, alpha))
    vel = sol.getSolution()
    dom.applyBoundaryConditions(vel, "velocity", 0.0, 0.02)
    b = sol.rhs(vort).copy()
    bd = b.getArray().copy()
    sol.solve(vort)
    assert ksp.getConvergedReason() > 0
    u_dev = vel.getArray().copy()
    _log(t0, f"device: {ksp.getIterationNumber()} iterations")

    um = O.UMesh(3, NGL, V, Cc, F, T)
    assert um.N == 342225
    mp = O.node_map(xd, um.coords())              # device node -> oracle node
    xo = um.coords()
    flag = ((um.tags_ & 0x3f) != 0).astype(np.uint8)
    np.testing.assert_array_equal(np.sort(mp[np.array(sorted(dom.getNodesDirichlet()))]), np.flatnonzero(flag))
    _log(t0, "oracle mesh, node map, Dirichlet set equal")
    Ko, Kro, Rwo = um.assemble_fs(flag)
    _log(t0, f"oracle assembly: K {Ko.nnz} nnz")
    dof = (mp[:, None] * 3 + np.arange(3)).ravel()  # device DoF -> oracle DoF
    rng = np.random.default_rng(3)
    for name, ref in (("K", Ko), ("Krhs", Kro), ("Rw", Rwo)):
        A = getattr(mat, name)
        for _ in range(2):
            xo_v = rng.uniform(-1, 1, ref.n if hasattr(ref, "n") else um.N * 3)
            x = A.createVecRight()
            x.setArray(xo_v[dof])
            yd = (A * x).getArray()
            yo = ref.mult(xo_v)[dof]
            assert np.abs(yd - yo).max() <= 1e-12 * max(1.0, np.abs(yo).max()), name
        _log(t0, f"{name}: equal as operators under the node map")
    ubc = np.zeros(um.N * 3)
    bn = np.flatnonzero(flag)
    ubc[(bn[:, None] * 3 + np.arange(3)).ravel()] = f.velocity(xo[bn], alpha)
    bo = Rwo.mult(f.vorticity(xo, alpha)) + Kro.mult(ubc)
    assert np.abs(bd - bo[dof]).max() <= 1e-12 * np.abs(bo).max()
    u_o = np.empty_like(u_dev)
    u_o[dof] = u_dev                                # device solution in oracle numbering
    res = float(np.linalg.norm(bo - Ko.mult(u_o)) / np.linalg.norm(bo))
    assert res <= 1.05e-10, res
    uo, its_o, rr_o = Ko.cg(bo, rtol=1e-10, jacobi=True)
    rel = float(np.linalg.norm(u_o - uo) / np.linalg.norm(uo))
    _log(t0, f"true residual {res:.3e}; oracle CG {its_o} iterations; ||u - u_oracle|| / ||u_oracle|| {rel:.3e}")
    assert rel <= 1e-7
