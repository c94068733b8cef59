"""GPU parity of the unstructured-mesh row: device assembly,
KLE solve and evalRHS on Gmsh meshes vs the reference's own code (golden
fixtures: the reference's test.msh, a rotated / shuffled / perturbed hex
mesh, a no-slip wall on test.msh) and vs the CPU oracle on larger meshes.

Numbering.  The reference numbers nodes by PETSc section offsets, ours by
topological entity (kle_umesh.cpp), the fixtures by coordinates; matrices
and vectors are compared after relabelling through node coordinates
(oracle.node_map), so the check is pattern-exact and value-tight but
blind to the labels themselves (pinned in tests/test_umesh.py).

Tolerances (fp64): patterns bit-exact after relabelling; values <=
1e-12 * max|ref| (the element integrals are summed in a different but
equivalent order); CG (rtol 1e-13) vs the reference's direct solve <= 1e-9
relative; evalRHS <= 1e-6 of its scale, as for the box meshes."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
MSH = os.path.join(G, "test.msh")
TG = {2: {"custom-func": {"name": "taylor_green"}}, 3: {"custom-func": {"name": "taylor_green3d"}}}


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _msh(g, tmp_path):
    if "mesh_cells" not in g:
        return MSH
    from pynama_amd.meshgen import write_gmsh
    p = str(tmp_path / "mesh.msh")
    write_gmsh(p, int(g["dim"]), g["mesh_vertices"], g["mesh_cells"], g["mesh_facets"], g["mesh_tags"])
    return p


def _domain(pa, path, ngl, bc):
    dom = pa.Domain()
    dom.configure({"domain": {"ngl": ngl, "gmsh-file": path}, "boundary-conditions": bc})
    dom.setUp()
    assert dom.getMeshType() == "gmsh"
    return dom


def _relabel(A, mp, R, C, shape):
    """Our CSR in the fixture's numbering, as sorted (keys, values)."""
    ip, ix, d = A.getValuesCSR()
    rows = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    gr = mp[rows // R] * R + rows % R
    gc = mp[ix // C] * C + ix % C
    key = gr * shape[1] + gc
    o = np.argsort(key, kind="stable")
    return key[o], d[o]


def _check(A, g, name, mp, R, C):
    shape = tuple(int(v) for v in g[name + "_shape"])
    key, d = _relabel(A, mp, R, C, shape)
    ip = g[name + "_indptr"]
    rows = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    rkey = rows * shape[1] + g[name + "_indices"]
    np.testing.assert_array_equal(key, rkey, err_msg=name)
    ref = g[name + "_data"]
    assert np.abs(d - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max()), name


def _vec_to_ours(v, mp, bs):
    return np.asarray(v).reshape(-1, bs)[mp].ravel()


@pytest.mark.parametrize("case", ["gmsh2d", "umesh3d"])
def test_umesh_matrices_match_golden(pa, case, tmp_path):
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim, ngl = int(g["dim"]), int(g["ngl"])
    dom = _domain(pa, _msh(g, tmp_path), ngl, TG[dim])
    mp = O.node_map(dom.getFullCoordArray().reshape(-1, dim), g["coords"])
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    dw, ds = (1, 3) if dim == 2 else (3, 6)
    for name, R, C in (("K", dim, dim), ("Krhs", dim, dim), ("Rw", dim, dw)):
        _check(getattr(mat, name), g, name, mp, R, C)
    op = mat.getOperators()
    for name, R, C in (("Curl", dw, dim), ("SrT", ds, dim), ("DivSrT", dim, ds)):
        _check(getattr(op, name), g, name, mp, R, C)


@pytest.mark.parametrize("case", ["gmsh2d", "umesh3d"])
def test_umesh_solve_and_eval_rhs_match_golden(pa, case, tmp_path):
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim, ngl = int(g["dim"]), int(g["ngl"])
    dw = 1 if dim == 2 else 3
    cfg = {"name": case, "material-properties": {"rho": float(g["rho"]), "mu": float(g["mu"])},
           "domain": {"ngl": ngl, "gmsh-file": _msh(g, tmp_path)}, "boundary-conditions": TG[dim],
           "initial-conditions": TG[dim]}
    prob = pa.BaseProblem(cfg)
    prob.setUp()
    prob.setUpSolver()
    mp = O.node_map(prob.dom.getFullCoordArray().reshape(-1, dim), g["coords"])
    sol = prob.solverKLE
    sol.getKSP().setTolerances(rtol=1e-13)
    vort = prob.vort.duplicate()
    vort.setArray(_vec_to_ours(g["vort0"], mp, dw))
    vel = sol.getSolution()
    vel.setArray(_vec_to_ours(g["vel0"], mp, dim))
    b = sol.rhs(vort)
    np.testing.assert_allclose(b.getArray(), _vec_to_ours(g["b"], mp, dim), rtol=0,
                               atol=1e-12 * np.abs(g["b"]).max())
    sol.solve(vort)
    u = vel.getArray()
    ref = _vec_to_ours(g["u"], mp, dim)
    assert np.linalg.norm(u - ref) <= 1e-9 * np.linalg.norm(ref)
    # the discretisation error of the reference (exact TG field) is reproduced
    ex = _vec_to_ours(g["u_exact"], mp, dim)
    assert abs(np.linalg.norm(u - ex) - float(g["err_l2"])) <= 1e-8 * max(1.0, float(g["err_l2"]))
    # evalRHS (base_problem.py:111-154) at t = 0.25
    prob.vort.setArray(_vec_to_ours(g["rhs_vort_in"], mp, dw))
    f = prob.operator.Curl.createVecLeft()
    prob.evalRHS(None, float(g["rhs_t"]), prob.vort, f)
    np.testing.assert_allclose(prob.vort.getArray(), _vec_to_ours(g["rhs_vort_bc"], mp, dw), rtol=0,
                               atol=1e-12 * max(1.0, np.abs(g["rhs_vort_bc"]).max()))
    uu = sol.getSolution().getArray()
    rv = _vec_to_ours(g["rhs_vel"], mp, dim)
    assert np.linalg.norm(uu - rv) <= 1e-9 * max(1.0, np.linalg.norm(rv))
    rf = _vec_to_ours(g["rhs_f"], mp, dw)
    assert np.abs(f.getArray() - rf).max() <= 1e-6 * max(1.0, np.abs(rf).max())


NS3 = {"up": [1, 0, 0.5], "down": [0, 0, 0], "left": [0, 0, 0], "right": [0, 0, 0], "front": [0, 0, 0],
       "back": [0, 0, 0]}


@pytest.mark.parametrize("case,walls", [("gmsh2d_ns", {"down": [1, 0]}), ("umesh3d_ns", NS3)])
def test_umesh_noslip_matches_golden(pa, case, walls, tmp_path):
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    dim = int(g["dim"])
    dw = 1 if dim == 2 else 3
    dom = _domain(pa, _msh(g, tmp_path), int(g["ngl"]), {"no-slip": walls})
    mp = O.node_map(dom.getFullCoordArray().reshape(-1, dim), g["coords"])
    # the DoF classes (incl. the corner rule) equal the reference's sets
    inv = np.empty_like(mp)
    inv[mp] = np.arange(len(mp))
    for ours, ref in ((dom.getTangDofs(collect=True), g["tang_dofs"]),
                      (dom.getNormalDofs(collect=True), g["normal_dofs"])):
        o = np.array(sorted(ours), dtype=np.int64)
        np.testing.assert_array_equal(np.sort(mp[o // dim] * dim + o % dim), ref)
    mat = pa.MatNS()
    mat.setDomain(dom)
    mat.build()
    for name, R, C in (("K", dim, dim), ("Krhs", dim, dim), ("Rw", dim, dw), ("Rd", dim, 1), ("Kfs", dim, dim),
                       ("Krhsfs", dim, dim), ("Rwfs", dim, dw), ("Rdfs", dim, 1)):
        _check(getattr(mat, name), g, name, mp, R, C)
    sol = pa.KleSolver()
    sol.setMat(mat)
    sol.setUp()
    sol.getKSP().setTolerances(rtol=1e-13)
    sol.solverFS.setTolerances(rtol=1e-13)
    vort = mat.Rw.createVecRight()
    vort.setArray(_vec_to_ours(g["vort0"], mp, dw))
    vel = sol.getSolution()
    vel.setArray(_vec_to_ours(g["vel0"], mp, dim))
    sol.solveFS(vort)
    vfs = sol.getFreeSlipSolution().getArray()
    rfs = _vec_to_ours(g["velFS"], mp, dim)
    assert np.linalg.norm(vfs - rfs) <= 1e-9 * np.linalg.norm(rfs)
    sol.solve(vort)
    ru = _vec_to_ours(g["u"], mp, dim)
    assert np.linalg.norm(vel.getArray() - ru) <= 1e-9 * max(1.0, np.linalg.norm(ru))


@pytest.mark.parametrize("nelem,ngl,seed", [([4, 3, 3], 3, 21), ([3, 2, 3], 5, 22)])
def test_umesh_matches_oracle_3d(pa, nelem, ngl, seed, tmp_path):
    """Larger rotated hex meshes vs the C oracle (coordinate numbering)."""
    from pynama_amd.meshgen import perturbed_box, write_gmsh
    V, Cc, F, T = perturbed_box(3, nelem, seed=seed)
    p = str(tmp_path / "m.msh")
    write_gmsh(p, 3, V, Cc, F, T)
    dom = _domain(pa, p, ngl, TG[3])
    um = O.UMesh(3, ngl, V, Cc, F, T)
    mp = O.node_map(dom.getFullCoordArray().reshape(-1, 3), um.coords())
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    dirf = (um.tags_ & 0x3f) != 0
    K, Kr, Rw = um.assemble_fs(dirf.astype(np.uint8))
    Cu, S, D, _ = um.assemble_ops()

    def asg(prefix, A):
        return {prefix + "_indptr": A.indptr, prefix + "_indices": A.indices, prefix + "_data": A.data,
                prefix + "_shape": np.array([A.m, A.n])}

    g = {}
    for nm, A in (("K", K), ("Krhs", Kr), ("Rw", Rw), ("Curl", Cu), ("SrT", S), ("DivSrT", D)):
        g.update(asg(nm, A))
    for name, R, C in (("K", 3, 3), ("Krhs", 3, 3), ("Rw", 3, 3)):
        _check(getattr(mat, name), g, name, mp, R, C)
    op = mat.getOperators()
    for name, R, C in (("Curl", 3, 3), ("SrT", 6, 3), ("DivSrT", 3, 6)):
        _check(getattr(op, name), g, name, mp, R, C)
    # the node-block SpMV on an irregular pattern (bcol stream, no lattice boxes)
    assert not mat.K.isStructured()
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, K.m)
    xv = mat.K.createVecRight()
    xv.setArray(_vec_to_ours(x, mp, 3))
    y = (mat.K * xv).getArray()
    yr = _vec_to_ours(K.mult(x), mp, 3)
    assert np.linalg.norm(y - yr) <= 1e-13 * np.linalg.norm(yr)
