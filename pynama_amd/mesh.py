"""Meshes + slab partition (host side of libkle, no GPU needed).

BoxMesh replaces for the hot path the reference's DMPlex box mesh and FEM
section numbering (domain/dmplex.py:18-49,193-196,352-372,382-388).  Canonical
numbering: node id = ix + Lx*(iy + Ly*iz) on the GLL lattice, cells
x-fastest, element-local nodes in tensor order; ranks own slabs of whole
element layers along the slowest axis (z in 3-D, y in 2-D).

UnstructuredMesh replaces GmshDom (dmplex.py:390-395) + DMPlexDistribute:
quads / hexes from a Gmsh 4.1 file or from arrays; GLL nodes numbered by
topological entity (kle_umesh.cpp).  Cells are partitioned by inertial
recursive bisection (Chaco's inertial method; any number of neighbours per
rank, index-list halos) or, with partitioner="slab", into slabs along the
longest axis whose nodes are ordered [lower interface | interior | upper
interface] so the halo keeps the box mesh's two-range form.  Boundary faces
carry the Gmsh physical tag of their facet as the Face Sets value: tag t is
face name FACES[dim][t-1] (dmplex.py:27-30,175-178).
"""
import ctypes as C

import numpy as np

from ._lib import MeshInfo, call, load

PARTITIONERS = {"inertial": 0, "chaco": 0, "slab": 1}


def set_partitioner(name):
    """Partitioner of unstructured meshes created afterwards
    (PetscPartitioner type of DMPlexDistribute, dmplex.py:21)."""
    call("kle_set_partitioner", PARTITIONERS[name] if isinstance(name, str) else int(name))


def get_partitioner():
    return {0: "inertial", 1: "slab"}[int(load().kle_get_partitioner())]


class _partitioner:
    """Use `name` for one mesh creation (None: the current setting)."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = get_partitioner()
        if self.name is not None:
            set_partitioner(self.name)

    def __exit__(self, *exc):
        set_partitioner(self.prev)

# face names in the reference's order (dmplex.py:27-30): bit i of a face mask
FACES = {2: ["down", "right", "up", "left"],
         3: ["back", "front", "down", "up", "right", "left"]}


class _Mesh:
    def _load(self, h):
        self._h = h
        info = MeshInfo()
        call("kle_mesh_get_info", h, C.byref(info))
        self.info = info
        self.dim, self.ngl = info.dim, info.ngl
        dim = self.dim
        self.kind = "box" if info.kind == 0 else "unstructured"
        self.rank, self.nranks = info.rank, info.nranks
        self.N = info.n_nodes
        self.E = info.n_elems
        self.node_range = (info.node_begin, info.node_end)
        self.ext_range = (info.ext_begin, info.ext_end)
        self.elem_range = (info.elem_begin, info.elem_end)
        self.lattice = tuple(info.lattice[:dim])
        self.nelem = tuple(info.nelem[:dim])
        self.nn = self.ngl ** self.dim
        self.dim_w = 1 if dim == 2 else 3
        self.dim_s = 3 if dim == 2 else 6

    def __del__(self):
        try:
            if self._h:
                call("kle_mesh_destroy", self._h)
                self._h = None
        except Exception:
            pass

    @property
    def n_owned(self):
        return self.node_range[1] - self.node_range[0]

    def conn(self):
        ne = self.elem_range[1] - self.elem_range[0]
        out = np.zeros(ne * self.nn, dtype=np.int64)
        call("kle_mesh_get_conn", self._h, out)
        return out.reshape(ne, self.nn)

    def corners(self):
        ne = self.elem_range[1] - self.elem_range[0]
        out = np.zeros(ne * 2 ** self.dim * self.dim)
        call("kle_mesh_get_corners", self._h, out)
        return out.reshape(ne, 2 ** self.dim, self.dim)

    def coords(self):
        out = np.zeros(self.n_owned * self.dim)
        call("kle_mesh_get_coords", self._h, out)
        return out.reshape(self.n_owned, self.dim)

    def face_mask(self, names):
        faces = FACES[self.dim]
        m = 0
        for n in names:
            m |= 1 << faces.index(n)
        return m

    def face_nodes(self, names):
        """Owned nodes on the named faces, sorted (getBorderNodes, dmplex.py:160-166)."""
        mask = self.face_mask(names) if not isinstance(names, int) else names
        n = C.c_int64()
        call("kle_mesh_face_nodes", self._h, mask, None, C.byref(n))
        out = np.zeros(max(n.value, 1), dtype=np.int64)
        call("kle_mesh_face_nodes", self._h, mask, out.ctypes.data, C.byref(n))
        return out[: n.value]

    def set_dirichlet_faces(self, names):
        call("kle_mesh_set_dirichlet_faces", self._h, self.face_mask(names))

    def set_noslip_faces(self, names):
        """No-slip walls, in configuration order (fixes the corner DoF classes)."""
        faces = np.array([FACES[self.dim].index(n) for n in names], dtype=np.int32)
        call("kle_mesh_set_noslip_faces", self._h, faces if len(faces) else np.zeros(1, np.int32), len(faces))

    def set_dirichlet_nodes(self, nodes):
        nodes = np.ascontiguousarray(np.asarray(sorted(nodes), dtype=np.int64))
        call("kle_mesh_set_dirichlet_nodes", self._h, nodes if len(nodes) else np.zeros(1, np.int64),
             len(nodes))

    def pattern(self, which):
        """Symbolic node-block pattern: 0 K, 1 Krhs, 2 Rw -> (row_ptr, global cols)."""
        nb = C.c_int64()
        call("kle_mesh_pattern_size", self._h, int(which), C.byref(nb))
        rp = np.zeros(self.n_owned + 1, dtype=np.int64)
        cols = np.zeros(max(nb.value, 1), dtype=np.int64)
        call("kle_mesh_pattern", self._h, int(which), rp, cols.ctypes.data)
        return rp, cols[: nb.value]

    def halo(self):
        lo, hi, sl, sh = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        lr, hr = C.c_int(), C.c_int()
        call("kle_mesh_halo", self._h, C.byref(lo), C.byref(hi), C.byref(sl), C.byref(sh), C.byref(lr),
             C.byref(hr))
        return {"lo_nodes": lo.value, "hi_nodes": hi.value, "send_lo_nodes": sl.value,
                "send_hi_nodes": sh.value, "lo_rank": lr.value, "hi_rank": hr.value}

    def peers(self):
        """Halo neighbours: {rank: (ghost nodes received, owned-local node ids sent)}."""
        n = C.c_int()
        call("kle_mesh_get_peers", self._h, C.byref(n), None, None, None, None)
        k = n.value
        ranks = np.zeros(max(k, 1), np.int32)
        rn = np.zeros(max(k, 1), np.int64)
        sn = np.zeros(max(k, 1), np.int64)
        call("kle_mesh_get_peers", self._h, C.byref(n), ranks.ctypes.data, rn.ctypes.data, sn.ctypes.data, None)
        sl = np.zeros(max(int(sn[:k].sum()), 1), np.int64)
        call("kle_mesh_get_peers", self._h, C.byref(n), ranks.ctypes.data, rn.ctypes.data, sn.ctypes.data,
             sl.ctypes.data)
        out, o = {}, 0
        for j in range(k):
            out[int(ranks[j])] = (int(rn[j]), sl[o:o + sn[j]].copy())
            o += int(sn[j])
        return out

    def ext_gids(self):
        """Global node id of every owned + ghost node, in the vector layout's order."""
        out = np.zeros(max(self.ext_range[1] - self.ext_range[0], 1), np.int64)
        call("kle_mesh_get_ext_gids", self._h, out)
        return out[: self.ext_range[1] - self.ext_range[0]]


class BoxMesh(_Mesh):
    def __init__(self, dim, nelem, lower, upper, ngl, rank=0, nranks=1):
        dim = int(dim)
        ne = np.array(list(nelem) + [1] * (3 - dim), dtype=np.int64)
        lo = np.array(list(lower) + [0.0] * (3 - dim), dtype=np.float64)
        hi = np.array(list(upper) + [1.0] * (3 - dim), dtype=np.float64)
        h = C.c_void_p()
        call("kle_mesh_create_box", dim, ne, lo, hi, int(ngl), int(rank), int(nranks), C.byref(h))
        self._load(h)


class UnstructuredMesh(_Mesh):
    """Quad / hex mesh: UnstructuredMesh.from_gmsh(path, ngl) (GmshDom.create)
    or UnstructuredMesh(dim, ngl, vertices, cells, facets, facet_tags)."""

    def __init__(self, dim, ngl, vertices, cells, facets=None, facet_tags=None, rank=0, nranks=1, _handle=None,
                 partitioner=None):
        if _handle is not None:
            self._load(_handle)
            return
        dim = int(dim)
        v = np.zeros((len(vertices), 3))
        v[:, :dim] = np.asarray(vertices, dtype=np.float64)[:, :dim]
        cells = np.ascontiguousarray(cells, dtype=np.int64)
        assert cells.ndim == 2 and cells.shape[1] == 2 ** dim
        nf = 0 if facets is None else len(facets)
        fa = np.ascontiguousarray(facets if nf else np.zeros((1, 2 ** (dim - 1))), dtype=np.int64)
        ft = np.ascontiguousarray(facet_tags if nf else np.zeros(1), dtype=np.int32)
        h = C.c_void_p()
        with _partitioner(partitioner):
            call("kle_mesh_create_unstructured", dim, int(ngl), len(v), np.ascontiguousarray(v.ravel()), len(cells),
                 cells.ravel(), nf, fa.ctypes.data, ft.ctypes.data, int(rank), int(nranks), C.byref(h))
        self._load(h)

    @classmethod
    def from_gmsh(cls, path, ngl, rank=0, nranks=1, partitioner=None):
        h = C.c_void_p()
        with _partitioner(partitioner):
            call("kle_mesh_create_gmsh", str(path).encode(), int(ngl), int(rank), int(nranks), C.byref(h))
        return cls(None, None, None, None, _handle=h)

    def elements(self):
        """Global cell ids of the local (owned + ghost) elements, ascending."""
        out = np.zeros(max(self.elem_range[1] - self.elem_range[0], 1), dtype=np.int64)
        call("kle_mesh_get_elements", self._h, out)
        return out[: self.elem_range[1] - self.elem_range[0]]
