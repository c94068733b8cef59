"""Boundary conditions (pynama_amd.boundaries) against the facts of the
reference's own tests: src/tests/test_boundary_conditions.py (Boundary,
BoundaryConditions set-up per YAML form, DoF sets by type, Taylor-Green
boundary values) and src/tests/test_boundary_ns.py (normal / tangential DoFs
of no-slip walls), restated -- host-only."""
from math import cos, exp, pi, sin

import numpy as np
import pytest

from pynama_amd.boundaries import Boundary, BoundaryConditions, FunctionBoundary


# ---------------------------------------------------- test_boundary_conditions.py:9-65
@pytest.mark.parametrize("dim,vel,vort", [(2, [1, 4], [0]), (3, [1, 6, 8], [32, 12, 124])])
def test_basic_boundary(dim, vel, vort):
    b = Boundary("left", "free-slip", dim)
    b.setValues("velocity", vel)
    b.setValues("vorticity", vort)
    assert b.getName() == "left" and b.getType() == "free-slip"
    nodes = [0, 11, 24, 78]
    b.setNodes(nodes)
    np.testing.assert_array_equal(b.getDofsConstrained(), [i * dim + d for i in nodes for d in range(dim)])
    np.testing.assert_array_almost_equal(b.getValues("velocity"), np.tile(vel, len(nodes)), decimal=14)
    b.setNodes([123, 12415, 1566, 121])
    np.testing.assert_array_equal(b.getNodes(), [123, 12415, 1566, 121])
    with pytest.raises(Exception):
        b.getValues("pressure")


# --------------------------------------------------- test_boundary_conditions.py:67-172
SIDES = ["up", "down", "right", "left"]


def test_set_up_only_fs():
    v = {"velocity": [1, 0], "vorticity": [0]}
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"free-slip": {s: v for s in ("down", "right", "left", "up")}})
    assert bcs.getType() == "FS"
    assert len(bcs.getNamesByType("free-slip")) == 4 and bcs.getNamesByType("no-slip") == []


def test_set_up_custom_func():
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"custom-func": {"name": "taylor_green", "attributes": ["velocity", "vorticity"]}})
    assert bcs.getType() == "FS"
    assert len(bcs.getNamesByType("free-slip")) == 4 and bcs.getNamesByType("no-slip") == []
    assert all(s in bcs.getBordersNeedsCoords() for s in SIDES)


def test_set_up_custom_and_uniform():
    v = {"velocity": [1, 0], "vorticity": [0]}
    cf = {"custom-func": {"name": "taylor_green", "attributes": ["velocity", "vorticity"]}}
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"free-slip": {"down": v, "right": cf, "left": cf, "up": v}})
    assert bcs.getType() == "FS"
    assert len(bcs.getNamesByType("free-slip")) == 4 and bcs.getNamesByType("no-slip") == []
    assert "right" in bcs.getBordersNeedsCoords() and "left" in bcs.getBordersNeedsCoords()
    assert "up" not in bcs.getBordersNeedsCoords()


def test_set_up_only_ns():
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"no-slip": {s: {"velocity": [1, 0]} for s in ("down", "right", "left", "up")}})
    assert bcs.getType() == "NS"
    assert len(bcs.getNamesByType("no-slip")) == 4 and bcs.getNamesByType("free-slip") == []


def test_set_up_fs_ns():
    v = {"velocity": [1, 0], "vorticity": [0]}
    cf = {"custom-func": {"name": "taylor_green", "attributes": ["velocity", "vorticity"]}}
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"free-slip": {"down": v, "right": cf},
                               "no-slip": {"left": {"velocity": [1, 0]}, "up": {"velocity": [1, 0]}}})
    assert bcs.getType() == "FS-NS"
    assert {"down", "right"} <= set(bcs.getNamesByType("free-slip"))
    assert {"up", "left"} <= set(bcs.getNamesByType("no-slip"))
    assert "right" in bcs.getBordersNeedsCoords()


def test_get_indices():
    nodes = {"down": [0, 1, 2, 3], "right": [3, 4, 5, 6], "up": [6, 7, 8], "left": [8, 9, 10, 11, 0]}
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"free-slip": {"down": {"velocity": [1, 0], "vorticity": [0]},
                                             "right": {"velocity": [1, 0], "vorticity": [0]}},
                               "no-slip": {"left": {"velocity": [2, 0]}, "up": {"velocity": [2, 0]}}})
    for name, n in nodes.items():
        bcs.setBoundaryNodes(name, n)
    dim = 2
    ns = {n * dim + d for n in nodes["left"] + nodes["up"] for d in range(dim)}
    fs = {n * dim + d for n in nodes["down"] + nodes["right"] for d in range(dim)}
    assert bcs.getNoSlipIndices() == ns and bcs.getFreeSlipIndices() == fs
    assert bcs.getIndicesByType("no-slip") == ns and bcs.getIndicesByType("free-slip") == fs
    with pytest.raises(Exception):
        bcs.setBoundaryNodes("front", [1])


def test_uniform_forms():
    """uniform velocity (vorticity defaults to 0) and the Reynolds-number form
    (boundary_conditions.py:87-114): |v| = re * (mu / rho) / Lref along `direction` degrees."""
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"uniform": {"velocity": [4, 0]}})
    assert bcs.getType() == "FS" and len(bcs.getNamesByType("free-slip")) == 4
    b = bcs.getBoundary("up")
    np.testing.assert_array_equal(b.getVelocitySetted(), [4, 0])
    np.testing.assert_array_equal(b._vals["vorticity"], [0])
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"uniform": {"re": 100, "mu": 0.01, "rho": 0.5, "Lref": "1/2", "direction": 30}})
    vref = 100 * 0.02 / 0.5
    np.testing.assert_allclose(bcs.getBoundary("left").getVelocitySetted(),
                               [cos(pi / 6) * vref, sin(pi / 6) * vref], rtol=1e-15)
    with pytest.raises(Exception):
        BoundaryConditions(SIDES).setBoundaryConditions({"uniform": {"re": 100, "mu": 0.01}})
    with pytest.raises(Exception):
        BoundaryConditions(SIDES).setBoundaryConditions({})


# -------------------------------------------------- test_boundary_conditions.py:193-255
def _tg_velocity(coord, t, nu):   # functions/taylor_green.py velocity_test, restated
    x, y = 2 * pi * coord[0], 2 * pi * coord[1]
    e = exp(-4 * pi ** 2 * nu * t * 2.0)
    return [cos(x) * sin(y) * e, -sin(x) * cos(y) * e]


def _tg_vorticity(coord, t, nu):  # functions/taylor_green.py vorticity, restated
    x, y = 2 * pi * coord[0], 2 * pi * coord[1]
    return -2 * pi * 2.0 * cos(x) * cos(y) * exp(-4 * pi ** 2 * nu * t * 2.0)


@pytest.mark.parametrize("t,nu", [(0.0, 100.0), (0.3, 0.02)])
def test_function_boundary_taylor_green_2d(t, nu):
    coords = np.array([0, 0, 0.1, 0.1, 0.3, 0.3, 0.6, 0.6, 0.8, 0.8], dtype=float)
    b = FunctionBoundary("up", "taylor_green", ["velocity", "vorticity", "alpha"], dim=2)
    b.setNodes([0, 1, 2, 3, 4])
    b.setNodesCoordinates(coords)
    np.testing.assert_array_almost_equal(b.getNodesCoordinates().ravel(), coords, decimal=14)
    c = coords.reshape(5, 2)
    np.testing.assert_array_almost_equal(b.getValues("velocity", t, nu),
                                         np.concatenate([_tg_velocity(p, t, nu) for p in c]), decimal=14)
    np.testing.assert_array_almost_equal(b.getValues("vorticity", t, nu),
                                         [_tg_vorticity(p, t, nu) for p in c], decimal=14)


# ------------------------------------------------------------- test_boundary_ns.py
@pytest.mark.parametrize("dim,nodes", [(2, [0, 11, 24, 78]), (3, [0, 11, 24])])
def test_no_slip_normals_and_tangentials(dim, nodes):
    normal = {"down": 1, "left": 0, "front": 2}
    for name in ("down", "left") + (("front",) if dim == 3 else ()):
        b = Boundary(name, "no-slip", dim)
        b.setValues("velocity", [1, 4, 11][:dim])
        b.setNodes(nodes)
        assert b.getNormalDofs() == {n * dim + normal[name] for n in nodes}
        tangs = [a for a in range(dim) if a != normal[name]]
        assert b.getTangDofs() == {n * dim + a for a in tangs for n in nodes}
        assert b.getTangDirections() == tangs
        for a in tangs:
            assert b.getTangDofs(a) == {n * dim + a for n in nodes}
        np.testing.assert_array_equal(b.getVelocitySettedTangential(), np.array([1, 4, 11][:dim])[tangs])


def test_no_slip_normal_corner_rule():
    """getNoSlipNormalDofs(allGather=True): a left / right wall drops its normal
    (x) DoF where the node's y DoF is already the normal DoF of an up / down
    wall listed before it (boundary_conditions.py:227-243); without allGather
    every wall keeps its normal DoFs."""
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"no-slip": {"up": {"velocity": [1, 0]}, "down": {"velocity": [0, 0]},
                                           "left": {"velocity": [0, 0]}, "right": {"velocity": [0, 0]}}})
    nodes = {"down": [0, 1, 2], "right": [2, 5, 8], "up": [6, 7, 8], "left": [0, 3, 6]}
    for name, n in nodes.items():
        bcs.setBoundaryNodes(name, n)
    every = {n * 2 + 1 for n in nodes["up"] + nodes["down"]} | {n * 2 for n in nodes["left"] + nodes["right"]}
    assert bcs.getNoSlipNormalDofs() == every
    corners = {0 * 2, 2 * 2, 6 * 2, 8 * 2}  # x DoFs of the corner nodes
    assert bcs.getNoSlipNormalDofs(allGather=True) == every - corners
    assert bcs.getNoSlipTangDofs() == {n * 2 for n in nodes["up"] + nodes["down"]} | \
        {n * 2 + 1 for n in nodes["left"] + nodes["right"]}
    assert bcs.getNodesByType("no-slip") == set(range(9)) - {4}


class _Vec:
    def __init__(self, n):
        self.a = np.full(n, np.nan)
        self.assembled = False

    def setValues(self, idx, vals, addv=False):
        assert addv is False
        self.a[np.asarray(list(idx))] = vals

    def assemble(self):
        self.assembled = True


def test_set_values_to_vec():
    """setValuesToVec / setTangentialValuesToVec (boundary_conditions.py:252-278):
    INSERT of the boundary values, 2-D vorticity one value per node."""
    bcs = BoundaryConditions(SIDES)
    bcs.setBoundaryConditions({"no-slip": {"up": {"velocity": [2, 0]}, "down": {"velocity": [0, 0]}}})
    bcs.setBoundaryNodes("up", [6, 7, 8])
    bcs.setBoundaryNodes("down", [0, 1, 2])
    v = _Vec(18)
    bcs.setValuesToVec(v, "velocity", 0.0, 0.01)
    assert v.assembled
    np.testing.assert_array_equal(v.a[[12, 13, 14, 15, 16, 17]], [2, 0, 2, 0, 2, 0])
    np.testing.assert_array_equal(v.a[:6], 0)
    w = _Vec(9)
    bcs.setValuesToVec(w, "vorticity", 0.0, 0.01)
    np.testing.assert_array_equal(w.a[[0, 1, 2, 6, 7, 8]], 0)
    t = _Vec(18)
    bcs.setTangentialValuesToVec(t, "velocity", 0.0, 0.01)
    np.testing.assert_array_equal(t.a[[12, 14, 16]], 2)       # x is tangential to "up"
    assert np.isnan(t.a[[13, 15, 17]]).all()                   # normal DoFs untouched
