"""ParaView output: XDMF 2.0 time series over HDF5 (or raw binary) node data.

Mirror of the reference's Paraviewer / XmlGenerator (viewer/paraviewer.py:9-80,
viewer/xml_generator.py:4-120): the mesh coordinates once (mesh.h5:/fields/mesh),
then per saved step one file vec-data-<step>.h5 with the named vectors under
/fields, and a <case>.xmf that ParaView reads as a temporal collection of
Polyvertex grids -- vectors as JOINs of the component hyperslabs, scalars
(one value per node) directly, exactly the reference's XML layout.

HDF5 is written through ctypes on the system libhdf5 (the reference uses
PETSc's HDF5 viewer); where no libhdf5 can be loaded the same XDMF points at
raw little-endian float64 files (Format="Binary"), which ParaView also reads.
On several ranks the owned pieces are gathered to rank 0, which writes.
"""
import ctypes as C
import ctypes.util
import glob
import os
from xml.dom import minidom
from xml.etree.ElementTree import Element, SubElement, tostring

import numpy as np

from .runtime import _dist, world


class _H5:
    """The six HDF5 calls a 1-D float64 dataset needs (HDF5 >= 1.8 API)."""

    def __init__(self, path):
        L = C.CDLL(path)
        hid = C.c_int64
        L.H5open.restype = C.c_int
        if L.H5open() < 0:
            raise OSError("H5open failed")
        L.H5Fcreate.restype = hid
        L.H5Fcreate.argtypes = [C.c_char_p, C.c_uint, hid, hid]
        L.H5Gcreate2.restype = hid
        L.H5Gcreate2.argtypes = [hid, C.c_char_p, hid, hid, hid]
        L.H5Screate_simple.restype = hid
        L.H5Screate_simple.argtypes = [C.c_int, C.POINTER(C.c_uint64), C.c_void_p]
        L.H5Dcreate2.restype = hid
        L.H5Dcreate2.argtypes = [hid, C.c_char_p, hid, hid, hid, hid, hid]
        L.H5Dwrite.restype = C.c_int
        L.H5Dwrite.argtypes = [hid, hid, hid, hid, hid, C.c_void_p]
        L.H5Fopen.restype = hid
        L.H5Fopen.argtypes = [C.c_char_p, C.c_uint, hid]
        L.H5Dopen2.restype = hid
        L.H5Dopen2.argtypes = [hid, C.c_char_p, hid]
        L.H5Dget_space.restype = hid
        L.H5Dget_space.argtypes = [hid]
        L.H5Sget_simple_extent_npoints.restype = C.c_int64
        L.H5Sget_simple_extent_npoints.argtypes = [hid]
        L.H5Dread.restype = C.c_int
        L.H5Dread.argtypes = [hid, hid, hid, hid, hid, C.c_void_p]
        for f in ("H5Dclose", "H5Sclose", "H5Gclose", "H5Fclose"):
            getattr(L, f).argtypes = [hid]
            getattr(L, f).restype = C.c_int
        self.L = L
        self.f64 = hid.in_dll(L, "H5T_IEEE_F64LE_g").value
        self.native = hid.in_dll(L, "H5T_NATIVE_DOUBLE_g").value

    def write(self, path, group, arrays):
        L = self.L
        f = L.H5Fcreate(path.encode(), 2, 0, 0)  # H5F_ACC_TRUNC, default property lists
        if f < 0:
            raise OSError(f"cannot create {path}")
        g = L.H5Gcreate2(f, group.encode(), 0, 0, 0)
        try:
            for name, a in arrays:
                a = np.ascontiguousarray(a, dtype=np.float64).ravel()
                dims = (C.c_uint64 * 1)(len(a))
                s = L.H5Screate_simple(1, dims, None)
                d = L.H5Dcreate2(g, name.encode(), self.f64, s, 0, 0, 0)
                rc = L.H5Dwrite(d, self.native, 0, 0, 0, a.ctypes.data)
                L.H5Dclose(d)
                L.H5Sclose(s)
                if rc < 0:
                    raise OSError(f"H5Dwrite {name} failed")
        finally:
            L.H5Gclose(g)
            L.H5Fclose(f)

    def read(self, path, name):
        """Dataset `name` (full path, e.g. /fields/mesh) as float64 (tests)."""
        L = self.L
        f = L.H5Fopen(path.encode(), 0, 0)  # H5F_ACC_RDONLY
        if f < 0:
            raise OSError(f"cannot open {path}")
        try:
            d = L.H5Dopen2(f, name.encode(), 0)
            if d < 0:
                raise KeyError(name)
            s = L.H5Dget_space(d)
            out = np.zeros(L.H5Sget_simple_extent_npoints(s))
            L.H5Sclose(s)
            rc = L.H5Dread(d, self.native, 0, 0, 0, out.ctypes.data)
            L.H5Dclose(d)
            if rc < 0:
                raise OSError(f"H5Dread {name} failed")
            return out
        finally:
            L.H5Fclose(f)


def _find_hdf5():
    cands = [ctypes.util.find_library("hdf5")] + sorted(glob.glob("/opt/conda/lib/libhdf5.so*"))
    for c in cands:
        if not c or "hl" in os.path.basename(c):
            continue
        try:
            return _H5(c)
        except (OSError, ValueError, AttributeError):
            continue
    return None


class XmlGenerator:
    """xml_generator.py:4-120 (same element tree)."""

    def __init__(self, dim, h5name, fmt="HDF"):
        self.root = Element("Xdmf")
        self.root.set("Version", "2.0")
        self.dim = dim
        self.h5name = h5name
        self.fmt = fmt
        self.ext = "h5" if fmt == "HDF" else "bin"

    def setUpDomainNodes(self, totalNodes=None, nodesPerDim=None):
        self.dimensions = int(totalNodes if totalNodes is not None else np.prod(nodesPerDim))

    def generateXMLTemplate(self):
        self.domain = SubElement(self.root, "Domain")
        self.grid = SubElement(self.domain, "Grid")
        self.grid.set("Name", "TimeSeries")
        self.grid.set("GridType", "Collection")
        self.grid.set("CollectionType", "Temporal")

    def _data(self, parent, dims, ref):
        d = SubElement(parent, "DataItem")
        d.set("Dimensions", str(dims))
        d.set("NumberType", "Float")
        if self.fmt == "HDF":
            d.set("Format", "HDF")
            d.text = ref
        else:
            d.set("Format", "Binary")
            d.set("Precision", "8")
            d.set("Endian", "Little")
            d.text = ref.replace(":/fields/", "-").replace(".h5", "") + ".bin"
        return d

    def generateMeshData(self, name):
        g = SubElement(self.grid, "Grid")
        g.set("Name", name)
        g.set("GridType", "uniform")
        t = SubElement(g, "Topology")
        t.set("TopologyType", "Polyvertex")
        t.set("Dimensions", str(self.dimensions))
        geo = SubElement(g, "Geometry")
        geo.set("GeometryType", "XY" if self.dim == 2 else "XYZ")
        self._data(geo, self.dimensions * self.dim, "mesh.h5:/fields/mesh")
        return g

    def setTimeStamp(self, t, meshElem):
        SubElement(meshElem, "Time").set("Value", str(t))

    def setVectorAttribute(self, name, step, meshGrid):
        attr = SubElement(meshGrid, "Attribute")
        attr.set("Name", name)
        attr.set("AttributeType", "Vector")
        attr.set("Center", "Node")
        fn = SubElement(attr, "DataItem")
        fn.set("ItemType", "Function")
        fn.set("Dimensions", f"{self.dimensions} {self.dim}")
        fn.set("Function", "JOIN(" + ", ".join(f"${i}" for i in range(self.dim)) + ")")
        for i in range(self.dim):
            hs = SubElement(fn, "DataItem")
            hs.set("ItemType", "HyperSlab")
            hs.set("Dimensions", str(self.dimensions))
            hs.set("Name", f"{name}-{'XYZ'[i]}")
            sel = SubElement(hs, "DataItem")
            sel.set("Dimensions", "3 1")
            sel.set("Format", "XML")
            sel.text = f"{i} {self.dim} {self.dimensions}"
            self._data(hs, self.dimensions * self.dim, f"{self.h5name}-{step:05d}.h5:/fields/{name}")

    def setScalarAttribute(self, name, step, meshGrid):
        attr = SubElement(meshGrid, "Attribute")
        attr.set("Name", name)
        attr.set("AttributeType", "Scalar")
        attr.set("Center", "Node")
        self._data(attr, self.dimensions, f"{self.h5name}-{step:05d}.h5:/fields/{name}")

    def tostring(self):
        return minidom.parseString(tostring(self.root, "utf-8")).toprettyxml(indent=" ")

    def writeFile(self, nameFile):
        with open(f"{nameFile}.xmf", "w") as f:
            f.write(self.tostring())


class Paraviewer:
    """paraviewer.py:9-80: configure / saveMesh / saveData / writeXmf."""

    def __init__(self, fmt=None):
        self._h5 = None if fmt == "Binary" else _find_hdf5()
        self.fmt = "HDF" if self._h5 is not None else "Binary"

    def configure(self, dim, saveDir=None):
        self.saveDir = "." if not saveDir else saveDir
        rank, _ = world()
        if rank == 0:
            os.makedirs(self.saveDir, exist_ok=True)
        self.h5name = "vec-data"
        self.dim = dim
        self.xmlWriter = XmlGenerator(dim, self.h5name, self.fmt)

    @staticmethod
    def _gather(a):
        """Owned pieces of a distributed vector, concatenated in rank order on rank 0."""
        d = _dist()
        a = np.asarray(a, dtype=np.float64)
        if d is None or d.get_world_size() == 1:
            return a
        parts = [None] * d.get_world_size()
        d.all_gather_object(parts, a)
        return np.concatenate(parts)

    def _write(self, fname, arrays):
        rank, _ = world()
        if rank != 0:
            return
        path = os.path.join(self.saveDir, fname)
        if self.fmt == "HDF":
            self._h5.write(path, "/fields", arrays)
        else:
            base = path[:-3] if path.endswith(".h5") else path
            for name, a in arrays:
                np.ascontiguousarray(a, dtype="<f8").tofile(f"{base}-{name}.bin")

    def saveMesh(self, coords, name="mesh"):
        arr = coords.getArray() if hasattr(coords, "getArray") else coords
        full = self._gather(np.asarray(arr).ravel())
        self.xmlWriter.setUpDomainNodes(totalNodes=len(full) // self.dim)
        self.xmlWriter.generateXMLTemplate()
        self._write("mesh.h5", [(name, full)])

    def saveData(self, step, time, *vecs):
        arrays = [(v.getName(), self._gather(v.getArray())) for v in vecs]
        self._write(f"{self.h5name}-{step:05d}.h5", arrays)
        grid = self.xmlWriter.generateMeshData("mesh1")
        self.xmlWriter.setTimeStamp(time, grid)
        for (name, a) in arrays:
            if len(a) == self.xmlWriter.dimensions:
                self.xmlWriter.setScalarAttribute(name, step, grid)
            else:
                self.xmlWriter.setVectorAttribute(name, step, grid)

    def writeXmf(self, name):
        rank, _ = world()
        if rank == 0:
            self.xmlWriter.writeFile(os.path.join(self.saveDir, name))
