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
