"""Boundary conditions: the reference's Boundary / FunctionBoundary /
BoundaryConditions surface (boundaries/boundary.py,
boundaries/boundary_conditions.py:8-278), host-side.

They decide which nodes are Dirichlet (free-slip: every velocity DoF fixed;
no-slip: normal DoFs fixed, tangential DoFs freed by the K + Kfs pre-solve),
and write the boundary values into device vectors before each KLE solve
(`setValuesToVec`, the `u` of `b = Rw w + Krhs u`, kle_solver.py:33-37).
petsc4py IS objects are replaced by node arrays: a boundary of `dim`
components owns DoFs `node * dim + c`, node-major, as PETSc's block IS.
"""
import ast
import operator
from math import cos, radians, sin

import numpy as np

from . import fields
from .runtime import world

# normal axis of each named face; the other axes are tangential (boundary.py Directions)
NORMAL_AXIS = {"left": 0, "right": 0, "up": 1, "down": 1, "front": 2, "back": 2}


def _gather_sets(s):
    """Union over ranks (the reference's comm.allgather of index sets)."""
    _, size = world()
    if size == 1:
        return [s]
    import torch.distributed as dist
    parts = [None] * size
    dist.all_gather_object(parts, s)
    return parts


class Boundary:
    """One named face with constant values (boundary.py:6-125)."""

    needsCoords = False

    def __init__(self, name, typ, dim):
        if name not in NORMAL_AXIS:
            raise KeyError(f"unknown boundary name '{name}'")
        self._name, self._type, self._dim = name, typ, int(dim)
        self._normal = NORMAL_AXIS[name]
        self._tangs = [a for a in range(self._dim) if a != self._normal]
        self._nodes = None
        self._vals = {}

    # -- identity / type
    def getName(self):
        return self._name

    def setType(self, t):
        self._type = t

    def getType(self):
        return self._type

    def __repr__(self):
        return f"Boundary Name:{self._name}:: Type: {self._type}  :: DOFS Constrained {self._dim}\n"

    # -- values
    def setValues(self, attrName, vals):
        self._vals[attrName] = np.array(vals)

    def getValues(self, attrName, t=None, nu=None):
        if attrName not in self._vals:
            raise Exception(f"{attrName} Not defined")
        return np.tile(self._vals[attrName], len(self.getNodes()))

    def getVelocitySetted(self):
        return self._vals["velocity"]

    def getVelocitySettedTangential(self):
        return self._vals["velocity"][self._tangs]

    def getDirectionsConstrained(self):
        return str(np.array(("x", "y", "z"))[self._dim])

    # -- nodes and DoFs
    def setNodes(self, nodes):
        self._nodes = np.asarray(nodes, dtype=np.int64).ravel()

    def getNodes(self):
        if self._nodes is None:
            raise Exception(f"Nodes not defined in boundary {self._name}")
        return self._nodes

    def getNumOfNodes(self):
        return len(self.getNodes())

    def getDofsConstrained(self):
        n = self.getNodes()
        return (n[:, None] * self._dim + np.arange(self._dim)[None, :]).ravel()

    def getSize(self):
        return len(self.getNodes()) * self._dim

    def getNormalDofs(self):
        return set((self.getNodes() * self._dim + self._normal).tolist())

    def getTangDofs(self, tangDir=None):
        axes = self._tangs if tangDir is None else [tangDir]
        n = self.getNodes()
        out = set()
        for a in axes:
            out |= set((n * self._dim + a).tolist())
        return out

    def getTangDirections(self):
        return list(self._tangs)

    def destroy(self):
        self._nodes = None


class FunctionBoundary(Boundary):
    """Free-slip face whose values come from an analytic field
    (boundary.py:127-156; functions/taylor_green*.py)."""

    needsCoords = True

    def __init__(self, name, func_name, attrs, dim):
        super().__init__(name, "free-slip", dim)
        self.funcName = func_name
        self._func = fields.get(func_name)
        for a in attrs:
            if a not in ("velocity", "vorticity", "alpha", "convective", "diffusive"):
                raise AttributeError(f"{func_name} has no attribute {a}")
        self._coords = None

    def setNodesCoordinates(self, arr):
        a = np.asarray(arr, dtype=np.float64)
        self._coords = a.reshape(len(self.getNodes()), self._dim)

    def getNodesCoordinates(self):
        return self._coords

    def getValues(self, attrName, t, nu):
        alpha = self._func.alpha(0.0 if nu is None else nu, 0.0 if t is None else t)
        f = getattr(self._func, attrName)
        return np.asarray(f(self._coords, alpha), dtype=np.float64).ravel()


_OPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv,
        ast.Pow: operator.pow, ast.USub: operator.neg}


def _arith(expr):
    """Numeric value of a YAML `Lref` entry: a number or a plain arithmetic
    expression (the reference eval()s it, boundary_conditions.py:101)."""
    if isinstance(expr, (int, float)):
        return float(expr)

    def ev(node):
        if isinstance(node, ast.Expression):
            return ev(node.body)
        if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)):
            return float(node.value)
        if isinstance(node, ast.BinOp) and type(node.op) in _OPS:
            return _OPS[type(node.op)](ev(node.left), ev(node.right))
        if isinstance(node, ast.UnaryOp) and type(node.op) in _OPS:
            return _OPS[type(node.op)](ev(node.operand))
        raise ValueError(f"Lref must be a number or an arithmetic expression, got {expr!r}")
    return ev(ast.parse(str(expr), mode="eval"))


class BoundaryConditions:
    """Boundary conditions of a domain (boundary_conditions.py:8-278).  Types:
    "FS" (every face free-slip / uniform / custom-func), "NS" (no-slip walls),
    "FS-NS" (mixed: parsed; the KLE matrices for it do not exist in the
    reference either, base_problem.py:161-162)."""

    types = ["FS", "NS", "FS-NS"]
    bcTypesAvailable = ("uniform", "custom-func", "free-slip", "no-slip")

    def __init__(self, sides):
        self._sides = list(sides)
        self._dim = 2 if len(self._sides) == 4 else 3
        self._all = []
        self._by_name = {}
        self._by_type = {"free-slip": [], "no-slip": []}
        self._needs_coords = []
        self._type = None

    def __repr__(self):
        rows = [" --== Boundary Conditions ==--", "   Name   |   Type   |   Values   |   Nodes   "]
        for b in self._all:
            try:
                val = str(b.getVelocitySetted())
            except KeyError:
                val = "Not defined"
            nodes = str(b._nodes) if b._nodes is not None else "Not Defined"
            rows.append(f"{b.getName():10}|{b.getType():10}|{val:12}|{nodes:12}")
        return "\n".join(rows) + "\n"

    # ------------------------------------------------------------ setup
    def setBoundaryConditions(self, data):
        """`data` is the case's 'boundary-conditions' dictionary."""
        if "uniform" in data:
            self._type = "FS"
            vals = self._uniform(data["uniform"])
            for side in self._sides:
                self._add(side, "free-slip", vals)
        elif "custom-func" in data:
            self._type = "FS"
            cf = data["custom-func"]
            for side in self._sides:
                self._add_func(side, cf["name"], cf.get("attributes", ["velocity", "vorticity", "alpha"]))
        elif "free-slip" in data and "no-slip" in data:
            self._type = "FS-NS"
            self._per_side("free-slip", data["free-slip"])
            self._per_side("no-slip", data["no-slip"])
        elif "free-slip" in data:
            self._type = "FS"
            self._per_side("free-slip", data["free-slip"])
        elif "no-slip" in data:
            self._type = "NS"
            self._per_side("no-slip", data["no-slip"])
        else:
            raise Exception("Boundary Conditions not defined")

    def getType(self):
        return self._type

    def _zero_vort(self):
        # the reference writes [0] here, one value per node, which only fits
        # the 2-D vorticity; in 3-D it is [0, 0, 0] so setValuesToVec can write it
        return [0] if self._dim == 2 else [0, 0, 0]

    def _uniform(self, d):
        if "velocity" in d and "vorticity" not in d:
            return {"velocity": d["velocity"], "vorticity": self._zero_vort()}
        if "re" in d:
            for k in ("mu", "rho", "Lref", "direction"):
                if k not in d:
                    raise Exception("mu, rho, Lref AND/OR direction not defined")
            vref = d["re"] * (d["mu"] / d["rho"]) / _arith(d["Lref"])
            ang = radians(d["direction"])
            return {"velocity": [cos(ang) * vref, sin(ang) * vref], "vorticity": self._zero_vort()}
        return d

    def _per_side(self, typ, sides):
        for name, vals in sides.items():
            if isinstance(vals, dict) and "custom-func" in vals:
                cf = vals["custom-func"]
                self._add_func(name, cf["name"], cf.get("attributes", ["velocity", "vorticity", "alpha"]))
            else:
                self._add(name, typ, vals)

    def _register(self, b, typ):
        if typ not in self._by_type:
            raise Exception("Wrong boundary type")
        self._all.append(b)
        self._by_type[typ].append(b)
        self._by_name[b.getName()] = b

    def _add(self, name, typ, vals):
        b = Boundary(name, typ, self._dim)
        if isinstance(vals, (list, tuple)):
            b.setValues("velocity", vals)
            b.setValues("vorticity", self._zero_vort())
        else:
            for k, v in vals.items():
                b.setValues(k, v)
            if "vorticity" not in vals:  # a wall given only its velocity (no-slip)
                b.setValues("vorticity", self._zero_vort())
        self._register(b, typ)

    def _add_func(self, name, func_name, attrs):
        self._register(FunctionBoundary(name, func_name, attrs, self._dim), "free-slip")
        self._needs_coords.append(name)

    # ------------------------------------------------------------ queries
    def getNames(self, bcs=None):
        return [b.getName() for b in (self._all if bcs is None else bcs)]

    def getNamesByType(self, bcType):
        return self.getNames(self._by_type[bcType])

    def getBordersNeedsCoords(self):
        return self._needs_coords

    def getBoundary(self, name):
        return self._by_name[name]

    def getIndicesByName(self, name):
        return self._by_name[name].getDofsConstrained()

    def setBoundaryNodes(self, bName, nodes):
        if bName not in self._by_name:
            raise Exception("Boundary Not found")
        self._by_name[bName].setNodes(nodes)

    def setBoundaryCoords(self, bName, coords):
        self._by_name[bName].setNodesCoordinates(coords)

    def _dof_union(self, bcs):
        out = set()
        for b in bcs:
            out |= set(b.getDofsConstrained().tolist())
        return out

    def getIndicesByType(self, bcType):
        return self._dof_union(self._by_type[bcType])

    def getNodesByType(self, bcType, allGather=False):
        out = set()
        for b in self._by_type[bcType]:
            loc = set(b.getNodes().tolist())
            if allGather:
                for remote in _gather_sets(set(loc)):
                    loc |= remote
            out |= loc
        return out

    def getNoSlipIndices(self, allGather=False):
        return self._dof_union(self._by_type["no-slip"])

    def getFreeSlipIndices(self):
        return self._dof_union(self._by_type["free-slip"])

    def getNoSlipTangDofs(self, allGather=False):
        out = set()
        for b in self._by_type["no-slip"]:
            loc = b.getTangDofs()
            if allGather:
                for remote in _gather_sets(set(loc)):
                    loc |= remote
            out |= loc
        return out

    def getNoSlipNormalDofs(self, allGather=False):
        """Normal DoFs of the no-slip walls.  With allGather, a left / right
        wall's normal (x) DoF is dropped where the node's y DoF is already a
        normal DoF of an earlier up / down wall: a corner keeps the normal of
        the wall listed first (boundary_conditions.py:227-243)."""
        out, drop = set(), set()
        for b in self._by_type["no-slip"]:
            loc = b.getNormalDofs()
            if allGather:
                for remote in _gather_sets(set(loc)):
                    if b.getName() in ("left", "right"):
                        drop |= {i for i in remote if i + 1 in out}
                    loc |= remote
            out |= loc
        return out - drop

    # ------------------------------------------------------------ writers
    def setValuesToVec(self, vec, name, t, nu):
        """Boundary values of `name` into `vec` (INSERT), then assemble
        (boundary_conditions.py:252-260).  2-D vorticity is one value per node."""
        for b in self._all:
            if b._nodes is None or len(b._nodes) == 0:
                continue
            vals = b.getValues(name, t, nu)
            inds = b.getNodes() if (self._dim == 2 and name == "vorticity") else b.getDofsConstrained()
            vec.setValues(inds, vals, addv=False)
        vec.assemble()

    def setTangentialValuesToVec(self, vec, name, t, nu):
        """The walls' tangential velocity on their tangential DoFs: the no-slip
        condition (boundary_conditions.py:262-278)."""
        for b in self._by_type["no-slip"]:
            if b._nodes is None or len(b._nodes) == 0:
                continue
            vel = np.asarray(b.getVelocitySetted(), dtype=np.float64)
            n = b.getNumOfNodes()
            for a in b.getTangDirections():
                vec.setValues(b.getNodes() * self._dim + a, np.repeat(vel[a], n), addv=False)
        vec.assemble()
