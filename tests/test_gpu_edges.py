"""Edge cases of the device path against the CPU oracle: the smallest meshes
(one element, p = 1), anisotropic / offset boxes, high order (p = 6, 7),
Dirichlet sets that leave a single free node, and the solver on them.
Same tolerances as test_gpu.py (patterns bit-exact, values <= 1e-12 rel.)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def _check(pa, dim, nelem, lower, upper, ngl, faces=None):
    cfg = {"domain": {"ngl": ngl, "box-mesh": {"nelem": nelem, "lower": lower, "upper": upper}},
           "boundary-conditions": {"uniform": {"velocity": [1.0, -0.5, 0.25][:dim]}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    if faces is not None:
        dom.mesh.set_dirichlet_faces(faces)
    mat = pa.MatFS()
    mat.setDomain(dom)
    mat.build()
    om = O.BoxMesh(dim, nelem, lower, upper, ngl)
    flag = np.zeros(om.N, np.uint8)
    bn = dom.mesh.face_nodes(faces if faces is not None else pa.mesh.FACES[dim])
    flag[bn] = 1
    refs = dict(zip(("K", "Krhs", "Rw"), om.assemble_fs(flag)))
    for nm, R in refs.items():
        ip, ix, d = getattr(mat, nm).getValuesCSR()
        np.testing.assert_array_equal(ip, R.indptr, err_msg=nm)
        np.testing.assert_array_equal(ix, R.indices, err_msg=nm)
        if R.nnz:
            assert np.abs(d - R.data).max() <= 1e-12 * max(1.0, np.abs(R.data).max()), nm
    # SpMV and a solve on the assembled system
    K = refs["K"]
    x = mat.K.createVecRight()
    xa = np.random.default_rng(1).uniform(-1, 1, x.getLocalSize())
    x.setArray(xa)
    y = (mat.K * x).getArray()
    yr = K.mult(xa)
    assert np.linalg.norm(y - yr) <= 1e-13 * max(1.0, np.linalg.norm(yr))
    ksp = pa.petsc.KSP().create()
    ksp.setTolerances(rtol=1e-12, max_it=20000)
    ksp.setOperators(mat.K)
    u = mat.K.createVecRight()
    ksp.solve(mat.K * x, u)
    assert ksp.getConvergedReason() > 0
    assert np.linalg.norm(u.getArray() - xa) <= 1e-7 * np.linalg.norm(xa)


@pytest.mark.parametrize("dim,nelem,ngl", [(2, [1, 1], 2), (3, [1, 1, 1], 2), (2, [1, 1], 8), (3, [1, 1, 1], 5),
                                           (3, [2, 1, 1], 7)])
def test_smallest_and_high_order_meshes(pa, dim, nelem, ngl):
    _check(pa, dim, nelem, [0.0] * dim, [1.0] * dim, ngl)


@pytest.mark.parametrize("dim", [2, 3])
def test_anisotropic_offset_box(pa, dim):
    _check(pa, dim, [5, 2, 3][:dim], [-1.5, 0.25, 10.0][:dim], [2.0, 0.3, 13.0][:dim], 4)


def test_partial_dirichlet_faces(pa):
    """Dirichlet on two faces only (the rest free): patterns with free boundary rows."""
    _check(pa, 3, [2, 3, 2], [0, 0, 0], [1, 1, 1], 3, faces=["left", "down"])


def test_more_ranks_than_layers_is_an_error(pa):
    with pytest.raises(pa.Error):
        pa.BoxMesh(3, [2, 2, 2], [0, 0, 0], [1, 1, 1], 3, rank=0, nranks=3)
