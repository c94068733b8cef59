"""The reference's petsc4py calls, made the reference's way, on pynama_amd.petsc
(the surface is tests/golden/petsc4py_surface.json,
scanned from mat_fs.py, mat_ns.py, kle_solver.py, base_problem.py:111-222 and
boundary_conditions.py:1,191-278).  Every result is checked against numpy on
the same small matrices: a chain of 1-D elements (the assembly pattern of
MatFS.buildFS, mat_fs.py:175-189), a rectangular Rw-like operator, and the
KSP subclass pattern of kle_solver.py:49-64 (a KSP subclass whose __init__
does not chain up)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P():
    import pynama_amd
    pynama_amd.load()
    import pynama_amd.petsc as PETSc
    return PETSc


def _chain(P, n, shift, name):
    """n x n: per element (i, i+1) the local [[1, -1], [-1, 1]] added with
    np.ix_ blocks, then `shift` on the diagonal with the scalar form."""
    K = P.Mat().createAIJ(((n, None), (n, None)), nnz=(np.full(n, 3, np.int32), np.zeros(n, np.int32)),
                          comm=P.COMM_WORLD)                                    # mat_fs.py:103-104
    K.setUp()
    K.setName(name)
    loc = np.array([[1.0, -1.0], [-1.0, 1.0]])
    free = [0, 1]
    for e in range(n - 1):
        gl = [e, e + 1]
        K.setValues(gl, gl, loc[np.ix_(free, free)], addv=True)                  # mat_fs.py:179
    for i in range(n):
        K.setValues(i, i, shift, addv=True)                                       # mat_fs.py:117
    K.assemble()
    dense = np.diag(np.full(n, float(shift)))
    for e in range(n - 1):
        dense[e:e + 2, e:e + 2] += loc
    return K, dense


def test_mat_vec_ksp_is_comm_as_the_reference_calls_them(P):
    n, m = 9, 5
    K, Kd = _chain(P, n, 2, "K")
    Kfs, Kfsd = _chain(P, n, 1, "Kfs")
    assert K.getName() == "K"
    info = K.getInfo()                                                            # mat_fs.py:127
    assert info["nz_used"] >= n
    assert K.isSymmetric()                                                        # mat_fs.py:129
    # rectangular Rw (n x m) with positional addv (mat_fs.py:245-247 form)
    rng = np.random.default_rng(2)
    Rwd = np.zeros((n, m))
    Rw = P.Mat().createAIJ(((n, None), (m, None)), nnz=(np.full(n, m, np.int32), np.zeros(n, np.int32)),
                           comm=P.COMM_WORLD)
    Rw.setUp()
    for blk in range(3):
        rows = [blk * 3 + k for k in range(3)]
        cols = [(blk + k) % m for k in range(2)]
        v = rng.uniform(-1, 1, (3, 2))
        Rw.setValues(rows, cols, v, True)
        Rwd[np.ix_(rows, cols)] += v
    Rw.assemble()
    assert not Rw.isSymmetric()
    # weights: Vec.createMPI(((k, None)), comm=), setValues(list, ndarray, True), reciprocal, diagonalScale(L=)
    weig = P.Vec().createMPI(((n, None)), comm=P.COMM_WORLD)                      # mat_fs.py:228
    w = rng.uniform(1, 2, n)
    weig.setValues(list(range(n)), np.repeat(w[:, None], 1, axis=1).ravel(), True)  # mat_fs.py:249-251
    weig.assemble()
    weig.reciprocal()
    Rw.diagonalScale(L=weig)                                                      # mat_fs.py:257
    Rwd = Rwd / w[:, None]
    weig.destroy()
    # vectors and the KLE right-hand side: Rw * vort + Krhs * vel (kle_solver.py:35)
    vort = Rw.createVecRight()
    vort.setName("vorticity")
    va = rng.uniform(-1, 1, m)
    vort.setValues(list(range(m)), va, addv=False)                                # base_problem.py:209
    vort.assemble()
    vel = K.createVecRight()
    ua = rng.uniform(-1, 1, n)
    ind = np.arange(*K.getOwnershipRange(), dtype=np.int32)                       # base_problem.py:141-142
    vel.setValues(ind[::1], ua, False)                                            # base_problem.py:146
    vel.assemble()
    rhs = Rw * vort + Kfs * vel
    np.testing.assert_allclose(rhs.getArray(), Rwd @ va + Kfsd @ ua, rtol=1e-13, atol=1e-14)
    # Mat.mult, duplicate, *=, axpy, scale (base_problem.py:123-136)
    aux = vel.duplicate()
    K.mult(vel, aux)
    aux *= (2.0 * 0.5)
    other = vel.duplicate()
    other.setValues(ind, np.full(n, 0.25), False)
    other.assemble()
    aux.axpy(-1.0 * 2.0, other)
    out = vel.duplicate()
    Kfs.mult(aux, out)
    out.scale(1 / 2.0)
    np.testing.assert_allclose(out.getArray(), Kfsd @ (Kd @ ua - 0.5) / 2.0, rtol=1e-13, atol=1e-14)
    # Mat + Mat (kle_solver.py:25) and the KSP subclass of kle_solver.py:49-64
    S = K + Kfs
    np.testing.assert_allclose((S * vel).getArray(), (Kd + Kfsd) @ ua, rtol=1e-13, atol=1e-14)

    class KspSolver(P.KSP):
        comm = P.COMM_WORLD

        def __init__(self):  # (does not chain up, as the reference's does not)
            self.logger = None

        def createSolver(self, mat):
            self.create(self.comm)
            self.setType('gmres')
            pc = P.PC().create()
            pc.setType('lu')
            self.setPC(pc)
            self.setFromOptions()
            self.setOperators(mat)
            self.setUp()

    solver = KspSolver()
    solver.createSolver(S)
    x = S.createVecRight()
    solver(rhs, x)                                                                # kle_solver.py:35
    np.testing.assert_allclose(x.getArray(), np.linalg.solve(Kd + Kfsd, Rwd @ va + Kfsd @ ua), rtol=1e-10)
    assert solver.getConvergedReason() > 0
    # IS unions and the allgather of boundary_conditions.py:199-214 on this rank
    inds = P.IS().createGeneral([])
    for b in (P.IS().createBlock(3, [2, 0]), P.IS().createBlock(3, [1])):
        inds = b.union(inds)
    assert set(inds.getIndices()) == set(range(9))
    loc = set(P.IS().createBlock(3, [2, 0]).getBlockIndices())
    for remote in P.COMM_WORLD.tompi4py().allgather([loc]):
        loc |= remote[0]
    assert loc == {0, 2}
    assert P.COMM_WORLD.rank == 0
