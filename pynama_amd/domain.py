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

from .boundaries import NORMAL_AXIS, BoundaryConditions
from .mesh import FACES, BoxMesh, UnstructuredMesh
from .runtime import world


class Domain:
    def __init__(self):
        self.domData = None
        self.bcData = None
        self.mesh = None
        self.bcs = None
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
        """BoundaryConditions on the mesh's named faces (domain.py:77-96:
        setBoundaryConditions, then each face's nodes and, for analytic
        fields, their coordinates)."""
        if not self.bcData:
            raise ValueError("Boundary Conditions Not defined")
        self.bcs = BoundaryConditions(FACES[self.dim])
        self.bcs.setBoundaryConditions(self.bcData)
        self._type = self.bcs.getType()
        if self._type == "FS-NS":
            # mixed free-slip + no-slip: the reference has no matrix for it either
            # (base_problem.py:161-162, "FSNS Mat not implemented")
            raise NotImplementedError("mixed free-slip / no-slip boundaries (FS-NS)")
        lo = self.mesh.node_range[0]
        needs = set(self.bcs.getBordersNeedsCoords())
        for name in self.bcs.getNames():
            nodes = self.mesh.face_nodes([name])
            self.bcs.setBoundaryNodes(name, nodes)
            if name in needs:
                self.bcs.setBoundaryCoords(name, self._coords[nodes - lo] if len(nodes)
                                           else np.zeros((0, self.dim)))
        if self._type == "NS":
            self.mesh.set_noslip_faces(self.bcs.getNamesByType("no-slip"))
        else:
            self.mesh.set_dirichlet_faces(self.bcs.getNamesByType("free-slip"))

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

    # no-slip DoF sets (BoundaryConditions.getNoSlip*, boundary_conditions.py:205-238),
    # this rank's nodes
    _AXIS = NORMAL_AXIS

    def getBoundaryConditions(self):
        return self.bcs

    def _ns(self):
        return [self.bcs.getBoundary(n) for n in self.bcs.getNamesByType("no-slip")]

    def getNodesNoSlip(self, collect=False):
        return self.bcs.getNodesByType("no-slip")

    def getTangDofs(self, collect=False):
        return self.bcs.getNoSlipTangDofs()

    def getNormalDofs(self, collect=False):
        """collect: the corner rule of getNoSlipNormalDofs(allGather=True) --
        a left / right wall drops its normal DoF where an earlier up / down
        wall already fixed the node's y DoF -- on this rank's nodes."""
        dofs, remove = set(), set()
        for b in self._ns():
            loc = b.getNormalDofs()
            if collect and b.getName() in ("left", "right"):
                remove |= {i for i in loc if i + 1 in dofs}
            dofs |= loc
        return dofs - remove

    def getNodesDirichlet(self, collect=False):
        return self.bcs.getNodesByType("free-slip")

    # -------------------------------------------------------------- BCs
    def applyBoundaryConditions(self, vec, varName, t=None, nu=None):
        """BoundaryConditions.setValuesToVec (boundary_conditions.py:252-260)."""
        self.bcs.setValuesToVec(vec, varName, t, nu)

    def applyBoundaryConditionsNS(self, vec, varName, t=None, nu=None):
        """BoundaryConditions.setTangentialValuesToVec (boundary_conditions.py:262-278):
        the tangential wall velocity on every no-slip wall."""
        self.bcs.setTangentialValuesToVec(vec, varName, t, nu)
