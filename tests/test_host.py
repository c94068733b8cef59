"""CPU-only tests of libkle's host side: the C ABI exports, the structured
mesh / numbering / symbolic patterns against the golden fixtures (bit-exact),
the reference's domain facts, and the slab partition + halo plan."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
CASES = ["uniform2d", "tg2d", "tg2d_small", "tg3d", "tg3d_p4", "cavity2d"]


@pytest.fixture(scope="module")
def pa():
    import pynama_amd
    pynama_amd.load()
    return pynama_amd


def test_library_exports_every_header_symbol(pa):
    hdr = open(os.path.join(ROOT, "include", "kle.h")).read()
    names = sorted(set(re.findall(r"\b(kle_[a-z0-9_]+)\s*\(", hdr)))
    assert len(names) > 60
    lib = C.CDLL(pa._lib.LIBPATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes binding declares all of them
    bound = set(pa._lib.exported_symbols())
    assert not (set(names) - bound), sorted(set(names) - bound)


def _mesh(pa, g):
    return pa.BoxMesh(int(g["dim"]), list(g["nelem"]), list(g["lower"]), list(g["upper"]), int(g["ngl"]))


def _tensor_index(loc2lat, ngl):
    idx = np.zeros(len(loc2lat), dtype=np.int64)
    for d in range(loc2lat.shape[1]):
        idx += loc2lat[:, d] * ngl ** d
    return idx


def _expand(rp, cols, R, C, dir_rows=None):
    """node-block pattern -> scalar CSR pattern in PETSc layout"""
    ip, ix = [0], []
    for i in range(len(rp) - 1):
        c = cols[rp[i]:rp[i + 1]]
        for a in range(R):
            if dir_rows is not None and dir_rows[i]:
                ix.append(c[0] * C + a)
            else:
                ix.extend((c[:, None] * C + np.arange(C)[None, :]).ravel().tolist())
            ip.append(len(ix))
    return np.array(ip), np.array(ix, dtype=np.int64)


@pytest.mark.parametrize("case", CASES)
def test_mesh_conn_coords_patterns(pa, case):
    g = np.load(os.path.join(G, f"case_{case}.npz"))
    m = _mesh(pa, g)
    ngl, dim = int(g["ngl"]), int(g["dim"])
    conn = m.conn()
    np.testing.assert_array_equal(conn[:, _tensor_index(g["loc2lat"], ngl)], g["conn"])
    np.testing.assert_allclose(m.coords(), g["coords"], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(m.corners(), g["corners"])
    if case == "cavity2d":
        return  # no-slip sets differ (next row); conn/coords still pinned
    m.set_dirichlet_nodes(g["dir_nodes"])
    dirf = np.zeros(m.N, bool)
    dirf[g["dir_nodes"]] = True
    dw = 1 if dim == 2 else 3
    for which, nm, C_ in ((0, "K", dim), (1, "Krhs", dim), (2, "Rw", dw)):
        rp, cols = m.pattern(which)
        ip, ix = _expand(rp, cols, dim, C_, dirf if which < 2 else None)
        np.testing.assert_array_equal(ip, g[nm + "_indptr"])
        np.testing.assert_array_equal(ix, g[nm + "_indices"])


def test_domain_facts_from_reference_tests(pa):
    # test_domain.py:30-39: 2x2 box, ngl=3 -> 25 nodes, 4 cells
    m = pa.BoxMesh(2, [2, 2], [0, 0], [1, 1], 3)
    assert (m.N, m.E) == (25, 4)
    # test_domain.py:52-62: ngl=7 -> (7*2-1)^2 nodes
    assert pa.BoxMesh(2, [2, 2], [0, 0], [1, 1], 7).N == 13 * 13
    # test_domain.py:223-227 / ngl=2: x-fastest lexicographic numbering
    m = pa.BoxMesh(2, [2, 2], [0, 0], [1, 1], 2)
    xy = m.coords()
    np.testing.assert_array_equal(xy[:, 0], np.tile([0, 0.5, 1], 3))
    np.testing.assert_array_equal(xy[:, 1], np.repeat([0, 0.5, 1], 3))
    # test_dmplex_wrapper.py:24-27 cell-0 corners (2-D), closure order
    m = pa.BoxMesh(2, [3, 4], [0, 0], [0.6, 0.8], 3)
    np.testing.assert_allclose(m.corners()[0].ravel(), [0, 0, 0.2, 0, 0.2, 0.2, 0, 0.2], atol=1e-13)
    # test_dmplex_wrapper.py:29-47 border node counts (2-D [3,4], ngl=3)
    assert len(m.face_nodes(["down", "right", "up", "left"])) == 28
    for b in ("up", "down"):
        assert len(m.face_nodes([b])) == 7
    for b in ("left", "right"):
        assert len(m.face_nodes([b])) == 9
    # test_dmplex_wrapper.py:100-115 (3-D [3,4,5], ngl=3)
    m3 = pa.BoxMesh(3, [3, 4, 5], [0, 0, 0], [0.6, 0.8, 1], 3)
    np.testing.assert_allclose(m3.corners()[0].ravel(),
                               np.array([[0, 0, 0], [0, .2, 0], [.2, .2, 0], [.2, 0, 0], [0, 0, .2], [.2, 0, .2],
                                         [.2, .2, .2], [0, .2, .2]]).ravel(), atol=1e-13)
    assert m3.E == 60
    assert len(m3.face_nodes(["back", "front", "down", "up", "right", "left"])) == 28 * 11 + 35 * 2
    # TestNglIndexing2D (test_dmplex_wrapper.py:61-88)
    for ngl in range(2, 10, 2):
        if ngl > 8:
            continue
        mm = pa.BoxMesh(2, [2, 3], [0, 0], [0.6, 0.8], ngl)
        assert len(mm.face_nodes(["down", "right", "up", "left"])) == 10 + 10 * (ngl - 2)
        for b in ("up", "down"):
            assert len(mm.face_nodes([b])) == 3 + 2 * (ngl - 2)
        for b in ("left", "right"):
            assert len(mm.face_nodes([b])) == 4 + 3 * (ngl - 2)


def test_bench_config_counts(pa):
    """Config 2 of BASELINE.json: n = 1,026,675, nnz(K) = 561,335,085."""
    m = pa.BoxMesh(3, [20, 16, 16], [0, 0, 0], [1, 1, 1], 5)
    m.set_dirichlet_faces(["back", "front", "down", "up", "right", "left"])
    assert m.N * 3 == 1026675
    rp, cols = m.pattern(0)
    ndir = len(m.face_nodes(["back", "front", "down", "up", "right", "left"]))
    assert len(cols) * 9 - 6 * ndir == 561335085


@pytest.mark.parametrize("nranks", [2, 3, 4, 8])
def test_slab_partition_and_halo_plan(pa, nranks):
    dims = ([20, 16, 16], 5)
    ms = [pa.BoxMesh(3, dims[0], [0, 0, 0], [1, 1, 1], dims[1], r, nranks) for r in range(nranks)]
    for m in ms:
        m.set_dirichlet_faces(["back", "front", "down", "up", "right", "left"])
    # owned ranges tile [0, N) in rank order
    assert ms[0].node_range[0] == 0 and ms[-1].node_range[1] == ms[0].N
    for a, b in zip(ms, ms[1:]):
        assert a.node_range[1] == b.node_range[0]
    serial = pa.BoxMesh(3, dims[0], [0, 0, 0], [1, 1, 1], dims[1])
    serial.set_dirichlet_faces(["back", "front", "down", "up", "right", "left"])
    for which in (0, 1, 2):
        rp_s, cols_s = serial.pattern(which)
        for m in ms:
            rp, cols = m.pattern(which)
            lo, hi = m.node_range
            # the partitioned rows are exactly the serial rows
            np.testing.assert_array_equal(cols, cols_s[rp_s[lo]:rp_s[hi]])
            # every column lies in the ghosted ext range
            if len(cols):
                assert cols.min() >= m.ext_range[0] and cols.max() < m.ext_range[1]
    # halo plan: what r sends down is what r-1 receives from above, and v.v.
    plane = ms[0].lattice[0] * ms[0].lattice[1]
    for r in range(nranks):
        h = ms[r].halo()
        if r > 0:
            assert h["lo_rank"] == r - 1
            assert h["lo_nodes"] == ms[r].node_range[0] - ms[r].ext_range[0]
            assert ms[r - 1].halo()["hi_nodes"] == plane  # one ghost plane above
        if r < nranks - 1:
            assert h["hi_rank"] == r + 1
    # local elements cover every element touching an owned row
    for m in ms:
        lo, hi = m.node_range
        sconn = serial.conn()
        need = np.nonzero(((sconn >= lo) & (sconn < hi)).any(1))[0]
        assert need.min() >= m.elem_range[0] and need.max() < m.elem_range[1]


def test_noslip_dof_sets_match_reference():
    """Domain no-slip DoF sets (getTangDofs / getNormalDofs(collect=True)) equal
    the reference BoundaryConditions' sets on the cavity fixture."""
    import pynama_amd as pa
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "case_cavity2d.npz"))
    cfg = {"domain": {"ngl": 3, "box-mesh": {"nelem": [4, 4], "lower": [0, 0], "upper": [1, 1]}},
           "boundary-conditions": {"no-slip": {"up": [2, 0], "down": [0, 0], "left": [0, 0], "right": [0, 0]}}}
    dom = pa.Domain()
    dom.configure(cfg)
    dom.setUp()
    assert dom.getBoundaryType() == "NS"
    assert sorted(dom.getTangDofs(collect=True)) == sorted(g["tang_dofs"].tolist())
    assert sorted(dom.getNormalDofs(collect=True)) == sorted(g["normal_dofs"].tolist())
    assert dom.getNodesNoSlip() == set(int(d) // 2 for d in g["tang_dofs"])


def test_bench_launcher_failure_path():
    """`bench.py --gpus 2` without torchrun starts its own ranks; when they
    fail (no GPU in this container) the launcher exits non-zero, prints no
    JSON line, and does not hang; a launch past its deadline is killed (124)."""
    import subprocess
    import sys
    env = dict(os.environ, KLE_COMM_TIMEOUT_S="20")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--nelem", "2,2,2",
                          "--ngl", "3", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode != 0
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert "2-rank launch failed" in out.stderr
    sys.path.insert(0, ROOT)
    import bench
    assert bench.launch_ranks(2, ["--nelem", "2,2,2", "--no-cpu-baseline"], deadline_s=0.5) == 124


def test_bench_refuses_a_stale_pmc_record(tmp_path):
    """bench.py's roofline.traffic comes from a PMC record only when that
    record was measured on the kernel now running: same launch names and the
    same algorithmic bytes per launch (tools/pmc_traffic.py stores both);
    otherwise traffic is null and traffic_status says why."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    k = "k_nb_spmv_sym_xl<8,true,4,4>+k_nb_sym_gather<8,4,4>"
    db = {"cur": {"kernel": k, "hbm_bytes_per_launch": 2.5e9, "algorithmic_bytes_per_launch": 2354103576.0},
          "old": {"kernel": k, "hbm_bytes_per_launch": 2.6e9},
          "other": {"kernel": "k_nb_spmv_xl<8>", "hbm_bytes_per_launch": 4.6e9,
                    "algorithmic_bytes_per_launch": 2354103576.0}}
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps(db))
    assert bench.lookup_traffic(str(p), "cur", k, 2354103576.0)[0] == 2.5e9
    for key, alg in (("cur", 2461811976.0), ("old", 2354103576.0), ("other", 2354103576.0), ("none", 1.0)):
        t, why = bench.lookup_traffic(str(p), key, k, alg)
        assert t is None and why
    assert bench.lookup_traffic(str(tmp_path / "absent.json"), "cur", k, 1.0)[0] is None
    # every record of the committed file that bench.py can return names its
    # algorithmic bytes (older records without them are never used)
    for key, rec in json.load(open(os.path.join(ROOT, "profiles", "traffic.json"))).items():
        if "algorithmic_bytes_per_launch" in rec:
            t, _ = bench.lookup_traffic(os.path.join(ROOT, "profiles", "traffic.json"), key, rec["kernel"],
                                        rec["algorithmic_bytes_per_launch"])
            assert t == rec["hbm_bytes_per_launch"]


def test_petsc4py_surface_of_the_reference_host_files():
    """Every petsc4py class, method, operator and import the reference's host
    files on the path use (mat_fs.py, mat_ns.py, kle_solver.py,
    base_problem.py:111-222, boundary_conditions.py:1,191-278; scanned from
    their source by tools/scan_petsc4py_surface.py into
    tests/golden/petsc4py_surface.json) exists in pynama_amd.petsc / its
    COMM_WORLD.  tests/test_gpu_petsc_surface.py calls them the reference's way."""
    import json
    import pynama_amd.petsc as P
    from pynama_amd.runtime import COMM_WORLD
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "petsc4py_surface.json")))
    assert d["unclassified"] == []
    assert len(d["entries"]) >= 50
    dunder = {"__mul__", "__add__", "__sub__", "__imul__", "__call__"}
    missing = []
    for e in d["entries"]:
        c, m = e["class"], e["member"]
        if c == "module":
            ok = m == "PETSc" or hasattr(P, m)
        elif c == "Comm":
            ok = hasattr(COMM_WORLD, m)
        elif c == "mpi4py.Comm":
            ok = hasattr(COMM_WORLD.tompi4py(), m)
        elif m in ("__init__", "__subclass__"):
            ok = isinstance(getattr(P, c, None), type)
        else:
            ok = callable(getattr(getattr(P, c, None), m, None)) or (m in dunder and hasattr(getattr(P, c), m))
        if not ok:
            missing.append(f"{c}.{m} ({e['sites'][0]})")
    assert not missing, missing
    # the keyword / argument forms the shim's signatures must take
    import inspect
    forms = {f"{e['class']}.{e['member']}": e["forms"] for e in d["entries"]}
    for key, kw in (("Mat.createAIJ", {"nnz", "comm"}), ("Mat.diagonalScale", {"L"}), ("Vec.createMPI", {"comm"}),
                    ("Vec.setValues", {"addv"}), ("Mat.setValues", {"addv"})):
        cls, meth = key.split(".")
        params = set(inspect.signature(getattr(getattr(P, cls), meth)).parameters)
        used = {k for f in forms[key] for k in f["kwargs"]}
        assert used <= kw and kw <= params, (key, used, params)


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference sources not present")
def test_petsc4py_surface_fixture_is_current(tmp_path):
    """The committed surface is what the scanner reads from the reference now."""
    import json
    import subprocess
    import sys
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scan_petsc4py_surface.py"), "--out", str(out)],
                   check=True, capture_output=True)
    assert json.load(open(out)) == json.load(open(os.path.join(ROOT, "tests", "golden", "petsc4py_surface.json")))


def test_index_sets_and_allgather_as_the_boundary_code_uses_them():
    """IS and COMM_WORLD.tompi4py().allgather the way boundary_conditions.py
    does (187-250): unions of boundary index sets from an empty general IS,
    block indices of a block IS, allgather of Python sets on one rank."""
    from pynama_amd.petsc import IS
    from pynama_amd.runtime import COMM_WORLD
    a = IS().createBlock(3, [4, 1, 7])
    assert list(a.getBlockIndices()) == [4, 1, 7]
    assert list(a.getIndices()) == [12, 13, 14, 3, 4, 5, 21, 22, 23]
    inds = IS().createGeneral([])
    for bc in (IS().createGeneral([5, 2, 9]), IS().createGeneral([2, 11]), IS().createGeneral({9, 0})):
        inds = bc.union(inds)
    assert set(inds.getIndices()) == {0, 2, 5, 9, 11} and list(inds.getIndices()) == [0, 2, 5, 9, 11]
    assert list(IS().createBlock(3, [1]).union(IS().createBlock(3, [0])).getBlockIndices()) == [0, 1]
    assert list(IS().createBlock(2, [1]).union(IS().createGeneral([0])).getIndices()) == [0, 2, 3]
    loc = {3, 4}
    coll = COMM_WORLD.tompi4py().allgather([loc])
    assert coll == [[{3, 4}]]
    assert COMM_WORLD.tompi4py().bcast("x") == "x"


def _allgather_worker(rank, size, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from pynama_amd.runtime import COMM_WORLD
        out = COMM_WORLD.tompi4py().allgather({rank * 10, rank * 10 + 1})
        b = COMM_WORLD.tompi4py().bcast({"from": rank}, root=1)
        q.put((rank, out, b))
    finally:
        dist.destroy_process_group()


def test_allgather_over_gloo_two_ranks():
    """getNodesByType(allGather=True) on two ranks: each rank's set, in rank order."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_allgather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for rank, out, b in res:
        assert out == [{0, 1}, {10, 11}] and b == {"from": 1}, (rank, out, b)


@pytest.mark.parametrize("lat,p,ncu,rounds,must", [((81, 65, 65), 4, 256, 1, True), ((81, 65, 65), 4, 128, 1, None),
                                                  ((41, 33, 9), 4, 256, 1, True), ((13, 9, 7), 2, 256, 1, True),
                                                  ((41, 33, 33), 4, 128, 1, True), ((25, 21, 13), 6, 64, 1, None),
                                                  ((5, 5, 5), 4, 256, 1, True), ((109, 109, 109), 6, 256, 1, False),
                                                  ((109, 109, 109), 6, 256, 4, True)])
def test_brick_planner_covers_the_lattice_and_balances(pa, lat, p, ncu, rounds, must):
    """The box brick planner (kle_brick_plan.cpp, host only): every plan
    covers the lattice exactly (the planner refuses otherwise), at most
    rounds x ncu bricks, regions within the LDS.  Config 4 (p = 6, 109^3
    nodes) has no one-round plan whose regions fit the LDS; with 4 rounds per
    CU it has (brick_setup raises the rounds until one fits: round 6)."""
    lib = pa.load()
    info = (C.c_int * 8)()
    st = (C.c_double * 8)()
    rc = lib.kle_brick_plan_box(lat[0], lat[1], lat[2], p, 1, ncu, rounds, 0, info, st)
    if rc != 0:
        # (bricks of more rows than one CU-share of config 2, or p = 6 in one
        # round: the regions may not fit the LDS; must: True succeeds, False
        # fails, None either)
        assert must is not True, (lat, p, ncu)
        return
    assert must is not False, (lat, p, ncu, rounds)
    assert 1 <= info[0] <= rounds * ncu
    assert info[4] <= 163840
    if lat == (81, 65, 65) and ncu == 256:
        assert st[0] < 1.11, st[0]  # (the heaviest brick / the mean: 1.098, 256 bricks)
        assert st[5] > 0.95, st[5]  # (paired tails: 97.5 % of the item lanes carry a block, 502k items; unpaired 76.6 %, 640k)
        assert st[1] < 2.2, st[1]  # (region entries per row)
    if lat == (109, 109, 109):
        assert info[0] > ncu, info[0]  # (whole rounds per CU)
