"""Synthetic unstructured quad/hex meshes (the stand-in for a Gmsh file).

`perturbed_box` builds a structured box of cells and then makes it
unstructured in every way the ingest path must handle: interior vertices are
moved randomly (curved-free but non-affine cells), vertex ids and cell order
are shuffled, and every cell gets a random orientation-preserving rotation of
its local frame, so neighbouring cells see shared edges and faces in every
relative orientation (the case the reference's orientation rules,
indices.py:77-85, exist for).  Boundary facets carry the Face Sets tag of
the box side they lie on (tag = 1 + index in FACES, the reference's names).
`write_gmsh` saves such a mesh as MSH 4.1 ASCII.
"""
import itertools

import numpy as np

from .mesh import FACES

# box side -> (axis, side), the reference's naming (dmplex.py:27-30)
_SIDE = {"left": (0, 0), "right": (0, 1), "down": (1, 0), "up": (1, 1), "back": (2, 0), "front": (2, 1)}
# tensor corner t = x + 2y (+4z) -> Gmsh vertex slot
_T2G = {2: [0, 1, 3, 2], 3: [0, 1, 3, 2, 4, 5, 7, 6]}


def _rotations(dim):
    """Orientation-preserving symmetries of the square / cube as corner maps
    new tensor corner -> old tensor corner."""
    out = []
    for perm in itertools.permutations(range(dim)):
        for signs in itertools.product((1, -1), repeat=dim):
            R = np.zeros((dim, dim), int)
            for i, j in enumerate(perm):
                R[i, j] = signs[i]
            if round(np.linalg.det(R)) != 1:
                continue
            m = []
            for t in range(2 ** dim):
                b = np.array([(t >> k) & 1 for k in range(dim)]) * 2 - 1
                o = (R @ b + 1) // 2
                m.append(int(sum(int(o[k]) << k for k in range(dim))))
            out.append(m)
    return out


def perturbed_box(dim, nelem, lower=None, upper=None, jitter=0.15, seed=0, rotate=True, shuffle=True):
    """-> (vertices [nv, 3], cells [nc, 2^dim] Gmsh order, facets, facet_tags)."""
    rng = np.random.default_rng(seed)
    nelem = [int(n) for n in nelem]
    lower = np.zeros(dim) if lower is None else np.asarray(lower, float)
    upper = np.ones(dim) if upper is None else np.asarray(upper, float)
    h = (upper - lower) / np.array(nelem)
    nv_ax = [n + 1 for n in nelem]
    grid = np.stack(np.meshgrid(*[np.arange(n) for n in nv_ax[::-1]], indexing="ij")[::-1], -1).reshape(-1, dim)
    X = lower + grid * h
    interior = np.all((grid > 0) & (grid < np.array(nv_ax) - 1), axis=1)
    X[interior] += rng.uniform(-jitter, jitter, (interior.sum(), dim)) * h
    vid = lambda g: int(sum(int(g[k]) * int(np.prod(nv_ax[:k])) for k in range(dim)))  # noqa: E731
    cells = []
    rots = _rotations(dim)
    for c in itertools.product(*[range(n) for n in nelem[::-1]]):
        c = c[::-1]
        tv = [vid([c[k] + ((t >> k) & 1) for k in range(dim)]) for t in range(2 ** dim)]
        if rotate:
            r = rots[rng.integers(len(rots))]
            tv = [tv[r[t]] for t in range(2 ** dim)]
        g = [0] * (2 ** dim)
        for t in range(2 ** dim):
            g[_T2G[dim][t]] = tv[t]
        cells.append(g)
    cells = np.array(cells, np.int64)
    # boundary facets with the side's tag
    facets, tags = [], []
    for name in FACES[dim]:
        ax, side = _SIDE[name]
        other = [k for k in range(dim) if k != ax]
        for c in itertools.product(*[range(nelem[k]) for k in other]):
            base = [0] * dim
            base[ax] = nv_ax[ax] - 1 if side else 0
            quad = []
            for bits in ([0], [1]) if dim == 2 else ([0, 0], [1, 0], [1, 1], [0, 1]):
                g = list(base)
                for k, b in zip(other, bits):
                    g[k] = c[other.index(k)] + b
                quad.append(vid(g))
            facets.append(quad)
            tags.append(FACES[dim].index(name) + 1)
    facets = np.array(facets, np.int64)
    tags = np.array(tags, np.int64)
    if shuffle:
        pv = rng.permutation(len(X))  # new id of old vertex
        Xn = np.empty_like(X)
        Xn[pv] = X
        X, cells, facets = Xn, pv[cells], pv[facets]
        cells = cells[rng.permutation(len(cells))]
    V = np.zeros((len(X), 3))
    V[:, :dim] = X
    return V, cells, facets, tags


def write_gmsh(path, dim, vertices, cells, facets, tags):
    """MSH 4.1 ASCII: one entity per facet tag (with that physical tag) and one
    for the cells."""
    utags = sorted(set(int(t) for t in tags))
    lines = ["$MeshFormat", "4.1 0 8", "$EndMeshFormat", "$Entities"]
    cnt = [0, 0, 0, 0]
    cnt[dim - 1] = len(utags)
    cnt[dim] = 1
    lines.append(" ".join(map(str, cnt)))
    for t in utags:  # facet entities: tag, bbox, 1 physical tag, 0 bounding entities
        lines.append(f"{t} 0 0 0 0 0 0 1 {t} 0")
    lines.append("1 0 0 0 0 0 0 0 0")
    lines.append("$EndEntities")
    nv = len(vertices)
    lines += ["$Nodes", f"1 {nv} 1 {nv}", f"{dim} 1 0 {nv}"]
    lines += [str(i + 1) for i in range(nv)]
    lines += ["%.17g %.17g %.17g" % tuple(v) for v in vertices]
    lines.append("$EndNodes")
    ftype, ctype = (3, 5) if dim == 3 else (1, 3)
    nel = len(facets) + len(cells)
    blocks = [(t, np.asarray(facets)[np.asarray(tags) == t]) for t in utags]
    lines += ["$Elements", f"{len(blocks) + 1} {nel} 1 {nel}"]
    k = 1
    for t, fs in blocks:
        lines.append(f"{dim - 1} {t} {ftype} {len(fs)}")
        for f in fs:
            lines.append(" ".join([str(k)] + [str(int(v) + 1) for v in f]))
            k += 1
    lines.append(f"{dim} 1 {ctype} {len(cells)}")
    for c in cells:
        lines.append(" ".join([str(k)] + [str(int(v) + 1) for v in c]))
        k += 1
    lines.append("$EndElements")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
