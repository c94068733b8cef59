"""Domain facade: structured box mesh + boundary conditions.

Host-side mirror of the subset of the reference's Domain
(domain/domain.py:16-318) and BoundaryConditions
(boundaries/boundary_conditions.py:44-278) that the KLE hot path calls:
configure / setOptions / setUp, getDimension(s), getNodesRange,
getLocalCellRange, getNodesDirichlet, getFullCoordArray, getAllNodes,
applyBoundaryConditions.  Same config schema as src/cases/*.yaml.
Meshes: "box-mesh" (BoxDom) and "gmsh-file" (GmshDom, MSH 4.1 quads/hexes,
dmplex.py:390-395); on a Gmsh mesh the boundary names are the Face Sets
values of the facets' physical tags in the reference's name order (tag 1 ->
"down" in 2-D, "back" in 3-D; dmplex.py:27-30,175-178).
"""
import copy

import numpy as np

from . import fields
from .mesh import FACES, BoxMesh, UnstructuredMesh
from .runtime import world


class _Boundary:
    """One named face with constant values or an analytic function."""

    def __init__(self, name, kind, values=None, func=None):
        self.name, self.kind, self.values, self.func = name, kind, values or {}, func
        self.nodes = np.zeros(0, dtype=np.int64)
        self.coords = None

    def get_values(self, var, dim, t, nu):
        n = len(self.nodes)
        if self.func is not None:
            alpha = self.func.alpha(nu if nu is not None else 0.0, t if t is not None else 0.0)
            f = self.func.velocity if var == "velocity" else self.func.vorticity
            return np.asarray(f(self.coords, alpha), dtype=np.float64).ravel()
        val = self.values.get(var)
        if val is None:
            val = [0.0] * (dim if var == "velocity" else (1 if dim == 2 else 3))
        return np.tile(np.asarray(val, dtype=np.float64), n)


class Domain:
    def __init__(self):
        self.domData = None
        self.bcData = None
        self.mesh = None
        self._bcs = []
        self._type = None
        self._type_mesh = None

    # ------------------------------------------------------------ config
    def configure(self, inp):
        data = copy.deepcopy(inp)
        if "domain" in data:
            self.domData = data["domain"]
        if "boundary-conditions" in data:
            self.bcData = data["boundary-conditions"]

    def setOptions(self, **kwargs):
        for key, val in kwargs.items():
            if key == "ngl":
                self.domData["ngl"] = val
            elif key in ("lower", "upper", "nelem"):
                self.domData["box-mesh"][key] = val
            elif key == "fileName":
                self.domData["gmsh-file"] = val
            elif key in ("freeSlip", "noSlip", "constant"):
                k = {"freeSlip": "free-slip", "noSlip": "no-slip"}.get(key, key)
                self.bcData[k] = val
            # other keys (e.g. keepCoords) are accepted and ignored, as the reference warns

    # ------------------------------------------------------------- setup
    def setUp(self):
        self.create()
        self.dim = self.mesh.dim
        self._coords = self.mesh.coords()
        self._setup_bcs()

    def create(self):
        """Domain.create (domain.py:25-43): the mesh of the 'box-mesh' or
        'gmsh-file' entry, partitioned over the ranks."""
        if not self.domData:
            raise ValueError("Domain not defined")
        rank, size = world()
        if "box-mesh" in self.domData:
            box = self.domData["box-mesh"]
            self._type_mesh = "box"
            self.mesh = BoxMesh(len(box["nelem"]), box["nelem"], box["lower"], box["upper"],
                                self.domData["ngl"], rank, size)
        elif "gmsh-file" in self.domData:
            self._type_mesh = "gmsh"
            self.mesh = UnstructuredMesh.from_gmsh(self.domData["gmsh-file"], self.domData["ngl"], rank, size,
                                                   partitioner=self.domData.get("partitioner", "inertial"))
        else:
            raise ValueError("Mesh Type not defined")

    def getMeshType(self):
        return self._type_mesh

    def _setup_bcs(self):
        if not self.bcData:
            raise ValueError("Boundary Conditions Not defined")
        names = FACES[self.dim]
        bc = self.bcData
        self._bcs = []
        if "uniform" in bc:
            self._type = "FS"
            vals = dict(bc["uniform"])
            vals.setdefault("vorticity", [0] if self.dim == 2 else [0, 0, 0])
            for n in names:
                self._bcs.append(_Boundary(n, "free-slip", vals))
        elif "custom-func" in bc:
            self._type = "FS"
            f = fields.get(bc["custom-func"]["name"])
            for n in names:
                self._bcs.append(_Boundary(n, "free-slip", func=f))
        elif "free-slip" in bc and "no-slip" not in bc:
            self._type = "FS"
            for n, v in bc["free-slip"].items():
                if isinstance(v, dict) and "custom-func" in v:
                    self._bcs.append(_Boundary(n, "free-slip", func=fields.get(v["custom-func"]["name"])))
                elif isinstance(v, dict):
                    self._bcs.append(_Boundary(n, "free-slip", dict(v)))
                else:
                    self._bcs.append(_Boundary(n, "free-slip", {"velocity": v}))
        elif "no-slip" in bc and "free-slip" not in bc:
            # walls with constant velocity (BoundaryConditions.__setBoundary,
            # boundary_conditions.py:115-136); dict order = processing order
            self._type = "NS"
            zero_w = [0] if self.dim == 2 else [0, 0, 0]
            for n, v in bc["no-slip"].items():
                vals = dict(v) if isinstance(v, dict) else {"velocity": v}
                vals.setdefault("vorticity", zero_w)
                self._bcs.append(_Boundary(n, "no-slip", vals))
        else:
            # mixed free-slip + no-slip: the reference has no matrix for it either
            # (base_problem.py:161-162, "FSNS Mat not implemented")
            raise NotImplementedError("mixed free-slip / no-slip boundaries (FS-NS)")
        for b in self._bcs:
            b.nodes = self.mesh.face_nodes([b.name])
            lo = self.mesh.node_range[0]
            b.coords = self._coords[b.nodes - lo] if len(b.nodes) else np.zeros((0, self.dim))
        if self._type == "NS":
            self.mesh.set_noslip_faces([b.name for b in self._bcs])
        else:
            self.mesh.set_dirichlet_faces([b.name for b in self._bcs])

    # ------------------------------------------------------------ queries
    def getMesh(self):
        return self.mesh

    def getDimension(self):
        return self.dim

    def getDimensions(self):
        return self.dim, 1 if self.dim == 2 else 3, 3 if self.dim == 2 else 6

    def getNGL(self):
        return self.mesh.ngl

    def getNumOfElements(self):
        return self.mesh.E

    def getNumOfNodes(self):
        return self.mesh.N

    def getNodesRange(self):
        return self.mesh.node_range

    def getLocalCellRange(self):
        return self.mesh.elem_range

    def getBoundaryType(self):
        return self._type

    def getFullCoordArray(self):
        return self._coords

    def getAllNodes(self):
        lo, hi = self.mesh.node_range
        return np.arange(lo, hi, dtype=np.int64)

    def getBorderNodes(self, name):
        return self.mesh.face_nodes([name])

    # no-slip DoF sets (BoundaryConditions.getNoSlip*, boundary_conditions.py:205-238)
    _AXIS = {"left": 0, "right": 0, "up": 1, "down": 1, "front": 2, "back": 2}

    def _ns(self):
        return [b for b in self._bcs if b.kind == "no-slip"]

    def getNodesNoSlip(self, collect=False):
        nodes = set()
        for b in self._ns():
            nodes |= set(b.nodes.tolist())
        return nodes

    def getTangDofs(self, collect=False):
        dofs = set()
        for b in self._ns():
            ax = self._AXIS[b.name]
            for t in range(self.dim):
                if t != ax:
                    dofs |= set((b.nodes * self.dim + t).tolist())
        return dofs

    def getNormalDofs(self, collect=False):
        dofs, remove = set(), set()
        for b in self._ns():
            ax = self._AXIS[b.name]
            loc = set((b.nodes * self.dim + ax).tolist())
            if collect and b.name in ("left", "right"):
                remove |= {i for i in loc if i + 1 in dofs}
            dofs |= loc
        return dofs - remove

    def getNodesDirichlet(self, collect=False):
        nodes = set()
        for b in self._bcs:
            if b.kind == "free-slip":
                nodes |= set(b.nodes.tolist())
        return nodes

    # -------------------------------------------------------------- BCs
    def applyBoundaryConditions(self, vec, varName, t=None, nu=None):
        """BoundaryConditions.setValuesToVec (boundary_conditions.py:252-260)."""
        for b in self._bcs:
            if len(b.nodes) == 0:
                continue
            vals = b.get_values(varName, self.dim, t, nu)
            if self.dim == 2 and varName == "vorticity":
                inds = b.nodes
            else:
                comps = self.dim
                inds = (b.nodes[:, None] * comps + np.arange(comps)[None, :]).ravel()
            vec.setValues(inds, vals, addv=False)
        vec.assemble()

    def applyBoundaryConditionsNS(self, vec, varName, t=None, nu=None):
        """BoundaryConditions.setTangentialValuesToVec (boundary_conditions.py:262-278):
        the tangential wall velocity on every no-slip wall."""
        for b in self._ns():
            if len(b.nodes) == 0:
                continue
            vel = np.asarray(b.values["velocity"], dtype=np.float64)
            ax = self._AXIS[b.name]
            for t_ in range(self.dim):
                if t_ != ax:
                    vec.setValues(b.nodes * self.dim + t_, np.repeat(vel[t_], len(b.nodes)), addv=False)
        vec.assemble()
