"""ParaView output: the reference's XDMF layout
(viewer/xml_generator.py:4-120) over HDF5 written through libhdf5, or raw
binary where no libhdf5 loads -- host-only."""
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from pynama_amd.viewer import Paraviewer, _find_hdf5


class _V:
    def __init__(self, name, a):
        self.name, self.a = name, np.asarray(a, float)

    def getName(self):
        return self.name

    def getArray(self):
        return self.a


@pytest.mark.parametrize("fmt", ["HDF", "Binary"])
def test_xdmf_time_series(tmp_path, fmt):
    if fmt == "HDF" and _find_hdf5() is None:
        pytest.skip("no libhdf5 in this image")
    rng = np.random.default_rng(0)
    n, dim = 17, 3
    v = Paraviewer(fmt="Binary" if fmt == "Binary" else None)
    assert v.fmt == fmt
    v.configure(dim, str(tmp_path / "out"))
    coords = rng.uniform(size=n * dim)
    v.saveMesh(coords)
    steps = []
    for step in (1, 2):
        vel, vort = _V("velocity", rng.uniform(size=n * dim)), _V("vorticity", rng.uniform(size=n * 3))
        scal = _V("num proc", np.arange(n))
        v.saveData(step, 0.1 * step, vel, vort, scal)
        steps.append((vel, vort, scal))
    v.writeXmf("case")
    root = ET.parse(tmp_path / "out" / "case.xmf").getroot()
    assert root.tag == "Xdmf" and root.get("Version") == "2.0"
    grids = root.find("Domain").find("Grid").findall("Grid")
    assert [g.find("Time").get("Value") for g in grids] == ["0.1", "0.2"]
    attrs = grids[0].findall("Attribute")
    assert [(a.get("Name"), a.get("AttributeType")) for a in attrs] == \
        [("velocity", "Vector"), ("vorticity", "Vector"), ("num proc", "Scalar")]
    assert attrs[0].find("DataItem").get("Function") == "JOIN($0, $1, $2)"
    # the data the XDMF points at
    out = tmp_path / "out"
    if fmt == "HDF":
        h5 = _find_hdf5()
        np.testing.assert_array_equal(h5.read(str(out / "mesh.h5"), "/fields/mesh"), coords)
        for step, (vel, vort, scal) in zip((1, 2), steps):
            f = str(out / f"vec-data-{step:05d}.h5")
            np.testing.assert_array_equal(h5.read(f, "/fields/velocity"), vel.a)
            np.testing.assert_array_equal(h5.read(f, "/fields/num proc"), scal.a)
        assert grids[0].find("Geometry").find("DataItem").text == "mesh.h5:/fields/mesh"
    else:
        ref = grids[1].find("Geometry").find("DataItem").text
        np.testing.assert_array_equal(np.fromfile(out / ref, "<f8"), coords)
        hs = attrs[0].find("DataItem").findall("DataItem")[1].findall("DataItem")[1].text
        np.testing.assert_array_equal(np.fromfile(out / hs, "<f8"), steps[0][0].a)
    assert os.path.exists(out / "case.xmf")


G = os.path.join(os.path.dirname(__file__), "golden")
_VEC_SIZES = {2: (2, 1), 3: (3, 3)}  # velocity, vorticity components


@pytest.mark.parametrize("dim,n", [(2, 13), (3, 17)])
def test_xdmf_tree_matches_reference_generator(dim, n):
    """Our XmlGenerator, driven in Paraviewer's sequence, writes the same
    document as the reference's own XmlGenerator (golden xdmf_<dim>d.xmf from
    tests/golden/make_golden.py: viewer/xml_generator.py:4-120 in the call
    order of viewer/paraviewer.py:21-70) -- text-identical."""
    from pynama_amd.viewer import XmlGenerator
    gen = XmlGenerator(dim, "vec-data", "HDF")
    gen.setUpDomainNodes(totalNodes=n)
    gen.generateXMLTemplate()
    cv, cw = _VEC_SIZES[dim]
    for step, t in ((1, 0.1), (2, 0.2), (10, 1.25)):
        grid = gen.generateMeshData("mesh1")
        gen.setTimeStamp(t, grid)
        for name, size in (("velocity", cv * n), ("vorticity", cw * n), ("num proc", n)):
            if size == gen.dimensions:
                gen.setScalarAttribute(name, step, grid)
            else:
                gen.setVectorAttribute(name, step, grid)
    with open(os.path.join(G, f"xdmf_{dim}d.xmf")) as f:
        assert gen.tostring() == f.read()


@pytest.mark.parametrize("dim,n", [(2, 13), (3, 17)])
def test_paraviewer_xmf_matches_reference_generator(tmp_path, dim, n):
    """End to end through Paraviewer (saveMesh, saveData per step, writeXmf)
    with HDF5 output: the .xmf equals the reference generator's document,
    element for element and attribute for attribute."""
    if _find_hdf5() is None:
        pytest.skip("no libhdf5 in this image")
    rng = np.random.default_rng(1)
    cv, cw = _VEC_SIZES[dim]
    v = Paraviewer()
    v.configure(dim, str(tmp_path / "out"))
    v.saveMesh(rng.uniform(size=n * dim))
    for step, t in ((1, 0.1), (2, 0.2), (10, 1.25)):
        v.saveData(step, t, _V("velocity", rng.uniform(size=cv * n)), _V("vorticity", rng.uniform(size=cw * n)),
                   _V("num proc", np.zeros(n)))
    v.writeXmf("case")
    got = ET.parse(tmp_path / "out" / "case.xmf").getroot()
    ref = ET.parse(os.path.join(G, f"xdmf_{dim}d.xmf")).getroot()

    def walk(a, b):
        assert a.tag == b.tag and a.attrib == b.attrib and (a.text or "").strip() == (b.text or "").strip()
        assert list(a.attrib) == list(b.attrib)
        assert len(a) == len(b)
        for x, y in zip(a, b):
            walk(x, y)
    walk(got, ref)
    with open(tmp_path / "out" / "case.xmf") as f, open(os.path.join(G, f"xdmf_{dim}d.xmf")) as g:
        assert f.read() == g.read()
