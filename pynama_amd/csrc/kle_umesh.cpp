// kle_umesh.cpp -- unstructured quad/hex meshes: Gmsh 4.1 ingest, entity
// numbering of the GLL nodes, slab partition with interface-ordered numbering.
// Host-only (no HIP calls).
//
// Replaces, for unstructured meshes, the reference's DMPlex path:
//   GmshDom.create -> DMPlexCreateFromFile       dmplex.py:390-395
//   DMPlexDistribute (Chaco partition)            dmplex.py:21
//   setFemIndexing / PetscSection offsets         dmplex.py:31-49, indices.py:22-30
//   mapEntitiesToNodes (edge/face orientations)   indices.py:70-96
//   computeFullCoordinates                        dmplex.py:62-91
//   Face Sets labels -> getBorderNodes            dmplex.py:109-166
//
// Element frame.  A cell's tensor corner (x, y[, z]) bits map to the Gmsh
// vertex order (quad 0-1-2-3 counter-clockwise; hex 0-3 bottom, 4-7 above
// them).  In DMPlex closure order (the slots of CORN2/CORN3) this is
// [g0 g1 g2 g3] for quads and [g0 g3 g2 g1 g4 g5 g6 g7] for hexes -- the
// order PETSc gives a Gmsh hex after its cell inversion -- so the element
// matrices see the same reference frame as the reference's.
//
// Node numbering.  GLL nodes are identified by the topological entity they
// lie on (vertex; edge by its vertex pair, position counted from the smaller
// vertex id; face by its vertex set, position in a frame anchored at the
// smallest vertex id; cell interior), so shared nodes coincide whatever the
// cells' relative orientation (the role of the reference's orientation rules,
// indices.py:77-85).  The reference's global numbering is PETSc's section
// order, which is not reproducible without PETSc; ours is (owner rank,
// interface segment, Hilbert order of the coordinates).  Parity tests compare
// through node coordinates.
//
// Partition (DMPlexDistribute with the Chaco partitioner, dmplex.py:21).
// Default: inertial recursive bisection of the cells -- Chaco's "inertial"
// method: split the cell centroids at the weighted median of their principal
// axis of inertia, recursively, rank counts proportional to the halves.  A
// node belongs to the highest rank among its cells.  Owned nodes are ordered
// [interior | rows that read ghosts] (Hilbert inside each), so the SpMV's
// ghost-free rows are one range that runs while the halo is in flight.  A
// rank's ghosts are grouped by owner rank in ascending global id, lower ranks
// before the owned range and higher ranks after it, so the vector layout
// [ghost_lo | owned | ghost_hi] and in-place receives are unchanged; sends are
// index lists (HaloPlan), any number of neighbours.  Ghost nodes get pseudo
// ids ext_begin + (ext position) inside the mesh (ext_gid holds their global
// ids), so every ext-indexed array and kernel works on either layout.
// Alternative (kle_set_partitioner(1)): slabs -- cells sorted by centroid
// along the axis with the most cell layers and cut into equal slabs, owned
// nodes ordered [read by the lower neighbour | interior | read by the upper],
// two contiguous halo ranges; slabs must be thick enough that no node touches
// cells of ranks two apart (checked; the error names the remedy).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <numeric>
#include <sstream>
#include <unordered_map>

#include "kle_basis.hpp"
#include "kle_internal.hpp"

using namespace kle;

namespace {

// tensor corner index t = x + 2y (+ 4z) -> Gmsh vertex slot
const int T2G2[4] = {0, 1, 3, 2};
const int T2G3[8] = {0, 1, 3, 2, 4, 5, 7, 6};
// DMPlex closure slot -> tensor corner index (CORN2 / CORN3 of kle_mesh.cpp)
const int C2T2[4] = {0, 1, 3, 2};          // (0,0) (1,0) (1,1) (0,1)
const int C2T3[8] = {0, 2, 3, 1, 4, 5, 7, 6};  // (000)(010)(110)(100)(001)(101)(111)(011)

struct KeyHash {
    size_t operator()(const std::array<int64_t, 4> &k) const
    {
        uint64_t h = 1469598103934665603ull;
        for (int64_t v : k) h = (h ^ (uint64_t)v) * 1099511628211ull;
        return (size_t)h;
    }
};
using Key = std::array<int64_t, 4>;

inline uint64_t spread3(uint64_t v)  // 21 bits -> every third bit
{
    v &= 0x1fffff;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
}

inline uint64_t spread2(uint64_t v)  // 32 bits -> every second bit
{
    v &= 0xffffffffull;
    v = (v | v << 16) & 0x0000ffff0000ffffull;
    v = (v | v << 8) & 0x00ff00ff00ff00ffull;
    v = (v | v << 4) & 0x0f0f0f0f0f0f0f0full;
    v = (v | v << 2) & 0x3333333333333333ull;
    v = (v | v << 1) & 0x5555555555555555ull;
    return v;
}

// Hilbert index of a point with b-bit coordinates q[0..n) (n = 2, 3):
// Skilling's transform of the axes to the "transposed" index, then the bits
// interleaved with axis 0 most significant.  Unlike the Morton (Z) order the
// curve never jumps, so consecutive node rows stay spatially adjacent.
inline uint64_t hilbert_key(uint32_t q[3], int n, int b)
{
    const uint32_t M = 1u << (b - 1);
    for (uint32_t Q = M; Q > 1; Q >>= 1) {
        const uint32_t P = Q - 1;
        for (int i = 0; i < n; ++i) {
            if (q[i] & Q) {
                q[0] ^= P;
            } else {
                const uint32_t t = (q[0] ^ q[i]) & P;
                q[0] ^= t;
                q[i] ^= t;
            }
        }
    }
    for (int i = 1; i < n; ++i) q[i] ^= q[i - 1];
    uint32_t t = 0;
    for (uint32_t Q = M; Q > 1; Q >>= 1)
        if (q[n - 1] & Q) t ^= Q - 1;
    for (int i = 0; i < n; ++i) q[i] ^= t;
    if (n == 2) return spread2(q[0]) << 1 | spread2(q[1]);
    return spread3(q[0]) << 2 | spread3(q[1]) << 1 | spread3(q[2]);
}

struct Build {
    int dim, ngl, p, nn, nc;
    int64_t nv, ncell;
    const double *vx;     // [nv][3]
    const int64_t *cells; // [ncell][nc] Gmsh order
    std::vector<int64_t> tv;   // [cell][nc] vertex id by tensor corner
    std::vector<int64_t> tmp;  // [cell][nn] temporary node id
    int64_t ntmp = 0;
};

// temporary node ids: vertices [0, nv), then edges, faces, cell interiors
int number_entities(Build &B)
{
    const int dim = B.dim, p = B.p, ngl = B.ngl, nn = B.nn, nc = B.nc;
    const int pm = p - 1;
    std::unordered_map<Key, int64_t, KeyHash> edges, faces;
    edges.reserve(B.ncell * (dim == 3 ? 4 : 2));
    if (dim == 3) faces.reserve(B.ncell * 4);
    // enumerate entities in cell order (deterministic ids)
    auto edge_id = [&](int64_t a, int64_t b) {
        Key k{std::min(a, b), std::max(a, b), -1, -1};
        auto it = edges.find(k);
        if (it != edges.end()) return it->second;
        int64_t id = (int64_t)edges.size();
        edges.emplace(k, id);
        return id;
    };
    auto face_id = [&](Key k) {
        std::sort(k.begin(), k.end());
        auto it = faces.find(k);
        if (it != faces.end()) return it->second;
        int64_t id = (int64_t)faces.size();
        faces.emplace(k, id);
        return id;
    };
    // pass 1: ids; pass 2: temp node ids need the totals, so store per-node (kind, entity, pos)
    struct Loc {
        uint8_t kind;  // 0 vertex, 1 edge, 2 face, 3 interior
        int64_t ent;
        int32_t pos;
    };
    std::vector<Loc> loc((size_t)B.ncell * nn);
    B.tv.resize((size_t)B.ncell * nc);
    for (int64_t c = 0; c < B.ncell; ++c)
        for (int t = 0; t < nc; ++t)
            B.tv[c * nc + t] = B.cells[c * nc + (dim == 2 ? T2G2[t] : T2G3[t])];
    for (int64_t c = 0; c < B.ncell; ++c) {
        const int64_t *V = &B.tv[c * nc];
        for (int l = 0; l < nn; ++l) {
            int q[3] = {l % ngl, (l / ngl) % ngl, dim == 3 ? l / (ngl * ngl) : 0};
            int freeax[3], nf = 0, bits = 0;
            for (int d = 0; d < dim; ++d) {
                if (q[d] == 0) continue;
                if (q[d] == p) bits |= 1 << d;
                else freeax[nf++] = d;
            }
            Loc &L = loc[c * nn + l];
            if (nf == 0) {
                L = {0, V[bits], 0};
            } else if (nf == dim) {
                int a = q[0] - 1, b = q[1] - 1, cc = dim == 3 ? q[2] - 1 : 0;
                L = {3, c, (int32_t)(a + pm * (b + pm * cc))};
            } else if (nf == 1) {
                const int d = freeax[0];
                const int64_t v0 = V[bits], v1 = V[bits | (1 << d)];
                const int s = v0 < v1 ? q[d] : p - q[d];
                L = {1, edge_id(v0, v1), s - 1};
            } else {  // 3-D face node: free axes d1 < d2
                const int d1 = freeax[0], d2 = freeax[1];
                // face corners in cyclic order (0,0) (1,0) (1,1) (0,1) of (d1, d2)
                const int cb[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
                int64_t F[4];
                for (int k = 0; k < 4; ++k) F[k] = V[bits | (cb[k][0] << d1) | (cb[k][1] << d2)];
                int o = 0;
                for (int k = 1; k < 4; ++k)
                    if (F[k] < F[o]) o = k;
                const int n1 = (o + 1) & 3, n3 = (o + 3) & 3;
                const int u = F[n1] < F[n3] ? n1 : n3;  // first axis towards the smaller neighbour
                // local coordinates of the node measured from corner o
                const int s1 = cb[o][0] ? p - q[d1] : q[d1];
                const int s2 = cb[o][1] ? p - q[d2] : q[d2];
                // does the u axis run along d1?
                const bool u_d1 = cb[u][0] != cb[o][0];
                const int su = u_d1 ? s1 : s2, sv = u_d1 ? s2 : s1;
                L = {2, face_id(Key{F[0], F[1], F[2], F[3]}), (int32_t)((su - 1) + pm * (sv - 1))};
            }
        }
    }
    const int64_t ne_ = (int64_t)edges.size(), nf_ = (int64_t)faces.size();
    const int64_t off_e = B.nv, off_f = off_e + ne_ * pm, off_c = off_f + nf_ * pm * pm;
    const int64_t per_cell = dim == 3 ? (int64_t)pm * pm * pm : (int64_t)pm * pm;
    B.ntmp = off_c + B.ncell * per_cell;
    B.tmp.resize((size_t)B.ncell * nn);
    for (size_t k = 0; k < loc.size(); ++k) {
        const Loc &L = loc[k];
        int64_t id;
        switch (L.kind) {
        case 0: id = L.ent; break;
        case 1: id = off_e + L.ent * pm + L.pos; break;
        case 2: id = off_f + L.ent * pm * pm + L.pos; break;
        default: id = off_c + L.ent * per_cell + L.pos;
        }
        B.tmp[k] = id;
    }
    return 0;
}

// principal axis (largest eigenvalue) of a symmetric dim x dim matrix, cyclic Jacobi
void principal_axis(int dim, double A[3][3], double v[3])
{
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0;
        for (int i = 0; i < dim; ++i)
            for (int j = i + 1; j < dim; ++j) off += A[i][j] * A[i][j];
        if (off < 1e-30) break;
        for (int pi = 0; pi < dim; ++pi)
            for (int q = pi + 1; q < dim; ++q) {
                if (std::fabs(A[pi][q]) < 1e-300) continue;
                const double th = (A[q][q] - A[pi][pi]) / (2 * A[pi][q]);
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1));
                const double c = 1 / std::sqrt(t * t + 1), sn = t * c;
                for (int k = 0; k < dim; ++k) {  // A <- A J
                    const double a = A[k][pi], b = A[k][q];
                    A[k][pi] = c * a - sn * b;
                    A[k][q] = sn * a + c * b;
                }
                for (int k = 0; k < dim; ++k) {  // A <- J^T A
                    const double a = A[pi][k], b = A[q][k];
                    A[pi][k] = c * a - sn * b;
                    A[q][k] = sn * a + c * b;
                }
                for (int k = 0; k < dim; ++k) {
                    const double a = V[k][pi], b = V[k][q];
                    V[k][pi] = c * a - sn * b;
                    V[k][q] = sn * a + c * b;
                }
            }
    }
    int best = 0;
    for (int i = 1; i < dim; ++i)
        if (A[i][i] > A[best][best] * (1 + 1e-12)) best = i;
    // sign convention: largest |component| positive (identical on every rank)
    int big = 0;
    for (int k = 1; k < dim; ++k)
        if (std::fabs(V[k][best]) > std::fabs(V[big][best])) big = k;
    const double sg = V[big][best] < 0 ? -1.0 : 1.0;
    for (int k = 0; k < 3; ++k) v[k] = k < dim ? sg * V[k][best] : 0.0;
}

// Chaco-style inertial recursive bisection of the cells idx[lo, hi) into
// ranks [r0, r0 + nr): split at the centroid count proportional to the rank
// counts of the two halves along the principal axis of inertia.
void inertial_bisect(int dim, const std::vector<double> &cen, std::vector<int64_t> &idx, int64_t lo, int64_t hi,
                     int r0, int nr, std::vector<int> &crank)
{
    if (nr == 1) {
        for (int64_t k = lo; k < hi; ++k) crank[idx[k]] = r0;
        return;
    }
    const int64_t n = hi - lo;
    double mu[3] = {0, 0, 0}, A[3][3] = {{0}};
    for (int64_t k = lo; k < hi; ++k)
        for (int d = 0; d < dim; ++d) mu[d] += cen[idx[k] * dim + d];
    for (int d = 0; d < dim; ++d) mu[d] /= (double)n;
    for (int64_t k = lo; k < hi; ++k) {
        const double *c = &cen[idx[k] * dim];
        for (int a = 0; a < dim; ++a)
            for (int b = 0; b < dim; ++b) A[a][b] += (c[a] - mu[a]) * (c[b] - mu[b]);
    }
    double ax[3];
    principal_axis(dim, A, ax);
    std::vector<std::pair<double, int64_t>> key(n);
    for (int64_t k = lo; k < hi; ++k) {
        double s = 0;
        for (int d = 0; d < dim; ++d) s += (cen[idx[k] * dim + d] - mu[d]) * ax[d];
        // quantised so that round-off cannot reorder cells on a symmetric mesh
        key[k - lo] = {std::nearbyint(s * 1e9) / 1e9, idx[k]};
    }
    std::sort(key.begin(), key.end());
    for (int64_t k = 0; k < n; ++k) idx[lo + k] = key[k].second;
    const int n1 = nr / 2;
    const int64_t cut = lo + (n * n1 + nr / 2) / nr;
    inertial_bisect(dim, cen, idx, lo, cut, r0, n1, crank);
    inertial_bisect(dim, cen, idx, cut, hi, r0 + n1, nr - n1, crank);
}

}  // namespace

namespace kle {

int g_partitioner = 0;  // 0 inertial bisection, 1 slabs

void umesh_row_nodes(const kle_mesh *m, int64_t i, std::vector<int64_t> &out)
{
    out.clear();
    const int nn = m->nn();
    for (int64_t k = m->u_incp[i]; k < m->u_incp[i + 1]; ++k) {
        const int64_t e = m->u_inc[k] / nn;
        out.insert(out.end(), m->u_conn.begin() + e * nn, m->u_conn.begin() + (e + 1) * nn);
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
}

}  // namespace kle

extern "C" {

int kle_mesh_create_unstructured(int dim, int ngl, int64_t nverts, const double *vxyz, int64_t ncells,
                                 const int64_t *cells, int64_t nfacets, const int64_t *facets,
                                 const int *facet_tags, int rank, int nranks, kle_mesh **out)
{
    KLE_ARG(out && vxyz && cells, "null arg");
    KLE_ARG(dim == 2 || dim == 3, "dim must be 2 or 3");
    KLE_ARG(ngl >= 2 && ngl <= 8, "ngl must be in [2,8] (got %d)", ngl);
    KLE_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank");
    KLE_ARG(ncells >= 1 && nverts >= 1, "empty mesh");
    KLE_ARG(nfacets == 0 || (facets && facet_tags), "null facet arrays");
    KLE_ARG(ncells >= nranks, "%d ranks > %lld cells", nranks, (long long)ncells);
    const int nc = 1 << dim, nfv = nc / 2;
    for (int64_t k = 0; k < ncells * nc; ++k)
        if (cells[k] < 0 || cells[k] >= nverts)
            return fail(KLE_ERR_ARG, "cell %lld references vertex %lld of %lld", (long long)(k / nc),
                        (long long)cells[k], (long long)nverts);
    Build B;
    B.dim = dim;
    B.ngl = ngl;
    B.p = ngl - 1;
    B.nn = dim == 2 ? ngl * ngl : ngl * ngl * ngl;
    B.nc = nc;
    B.nv = nverts;
    B.ncell = ncells;
    B.vx = vxyz;
    B.cells = cells;
    KLE_TRY(number_entities(B));
    const int nn = B.nn, p = B.p;
    // GLL points on [0,1]
    std::vector<double> gx, gw;
    gauss_lobatto(ngl, gx, gw);
    std::vector<double> xi(ngl);
    for (int i = 0; i < ngl; ++i) xi[i] = (1.0 + gx[i]) / 2.0;
    // orientation: Jacobian determinant at the cell centre must be positive
    auto corner = [&](int64_t c, int t, int d) { return vxyz[B.tv[c * nc + t] * 3 + d]; };
    for (int64_t c = 0; c < ncells; ++c) {
        double J[3][3] = {{0}};
        for (int t = 0; t < nc; ++t)
            for (int k = 0; k < dim; ++k) {
                // d N_t / d xi_k at the centre: +-1/2^(dim-1)
                const double s = ((t >> k) & 1 ? 1.0 : -1.0) / (1 << (dim - 1));
                for (int d = 0; d < dim; ++d) J[d][k] += s * corner(c, t, d);
            }
        const double det = dim == 2 ? J[0][0] * J[1][1] - J[0][1] * J[1][0]
                                    : J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                                          J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                                          J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
        if (!(det > 0))
            return fail(KLE_ERR_ARG, "cell %lld is inverted or degenerate (det J = %g at its centre)", (long long)c, det);
    }
    const int64_t NT = B.ntmp;
    // which temporary ids are used (a vertex not referenced by any cell is dropped)
    std::vector<uint8_t> used(NT, 0);
    for (int64_t v : B.tmp) used[v] = 1;
    // coordinates: the element map at the GLL point, last cell wins (the
    // reference's INSERT order in computeFullCoordinates)
    std::vector<double> X((size_t)NT * dim, 0.0);
    for (int64_t c = 0; c < ncells; ++c)
        for (int l = 0; l < nn; ++l) {
            const int q[3] = {l % ngl, (l / ngl) % ngl, dim == 3 ? l / (ngl * ngl) : 0};
            double xv[3] = {0, 0, 0};
            for (int t = 0; t < nc; ++t) {
                double w = 1.0;
                for (int k = 0; k < dim; ++k) w *= (t >> k) & 1 ? xi[q[k]] : 1.0 - xi[q[k]];
                for (int d = 0; d < dim; ++d) xv[d] += w * corner(c, t, d);
            }
            const int64_t id = B.tmp[c * nn + l];
            for (int d = 0; d < dim; ++d) X[id * dim + d] = xv[d];
        }
    // bounding box
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int64_t c = 0; c < ncells; ++c)
        for (int t = 0; t < nc; ++t)
            for (int d = 0; d < dim; ++d) {
                lo[d] = std::min(lo[d], corner(c, t, d));
                hi[d] = std::max(hi[d], corner(c, t, d));
            }
    // partition axis: the most cell layers (box extent / mean cell extent)
    double cext[3] = {0, 0, 0};
    for (int64_t c = 0; c < ncells; ++c)
        for (int d = 0; d < dim; ++d) {
            double a = 1e300, b = -1e300;
            for (int t = 0; t < nc; ++t) {
                a = std::min(a, corner(c, t, d));
                b = std::max(b, corner(c, t, d));
            }
            cext[d] += b - a;
        }
    int ax = 0;
    double best = -1;
    for (int d = 0; d < dim; ++d) {
        const double layers = cext[d] > 0 ? (hi[d] - lo[d]) * ncells / cext[d] : 0;
        if (layers > best * (1 + 1e-9)) {
            best = layers;
            ax = d;
        }
    }
    const bool slab = g_partitioner == 1;
    std::vector<int> crank(ncells, 0);
    if (nranks > 1 && slab) {
        std::vector<double> cen(ncells, 0.0);
        for (int64_t c = 0; c < ncells; ++c) {
            for (int t = 0; t < nc; ++t) cen[c] += corner(c, t, ax);
            cen[c] /= nc;
        }
        std::vector<int64_t> ord(ncells);
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return cen[a] < cen[b]; });
        for (int r = 0; r < nranks; ++r)
            for (int64_t k = ncells * r / nranks; k < ncells * (r + 1) / nranks; ++k) crank[ord[k]] = r;
    } else if (nranks > 1) {
        std::vector<double> cen((size_t)ncells * dim, 0.0);
        for (int64_t c = 0; c < ncells; ++c)
            for (int d = 0; d < dim; ++d) {
                for (int t = 0; t < nc; ++t) cen[c * dim + d] += corner(c, t, d);
                cen[c * dim + d] /= nc;
            }
        std::vector<int64_t> idx(ncells);
        std::iota(idx.begin(), idx.end(), 0);
        inertial_bisect(dim, cen, idx, 0, ncells, 0, nranks, crank);
    }
    // node owner = highest cell rank
    std::vector<int> own(NT, -1), omin(NT, nranks);
    for (int64_t c = 0; c < ncells; ++c)
        for (int l = 0; l < nn; ++l) {
            const int64_t id = B.tmp[c * nn + l];
            own[id] = std::max(own[id], crank[c]);
            omin[id] = std::min(omin[id], crank[c]);
        }
    if (slab)
        for (int64_t v = 0; v < NT; ++v)
            if (used[v] && own[v] - omin[v] > 1)
                return fail(KLE_ERR_ARG,
                            "slab partition too thin: a node touches cells of ranks %d and %d (use fewer ranks)",
                            omin[v], own[v]);
    // owner range of every cell's nodes
    std::vector<int> emin(ncells, nranks), emax(ncells, -1);
    for (int64_t c = 0; c < ncells; ++c)
        for (int l = 0; l < nn; ++l) {
            const int o = own[B.tmp[c * nn + l]];
            emin[c] = std::min(emin[c], o);
            emax[c] = std::max(emax[c], o);
        }
    // segments.  slab: 0 read by the lower neighbour, 1 interior, 2 read by
    // the upper.  inertial: 1 interior, 2 the row reads a ghost (a cell of the
    // node holds a node of another owner)
    std::vector<uint8_t> seglo(NT, 0), seghi(NT, 0);
    for (int64_t c = 0; c < ncells; ++c)
        for (int l = 0; l < nn; ++l) {
            const int64_t id = B.tmp[c * nn + l];
            if (slab) {
                if (emin[c] == own[id] - 1) seglo[id] = 1;
                if (emax[c] == own[id] + 1) seghi[id] = 1;
            } else if (emin[c] != own[id] || emax[c] != own[id]) {
                seghi[id] = 1;
            }
        }
    if (slab)
        for (int64_t v = 0; v < NT; ++v)
            if (used[v] && seglo[v] && seghi[v])
                return fail(KLE_ERR_ARG, "slab partition too thin: rank %d has a node read by both neighbours "
                                         "(use fewer ranks)", own[v]);
    // final numbering: (owner, segment, Hilbert key of x, temp id)
    std::vector<int64_t> ord;
    ord.reserve(NT);
    for (int64_t v = 0; v < NT; ++v)
        if (used[v]) ord.push_back(v);
    const int64_t N = (int64_t)ord.size();
    std::vector<uint64_t> code(NT, 0);
    // Hilbert order (default): 1M-DoF unstructured SpMV 0.817 -> 0.810 ms,
    // config-5 size 6.84 -> 6.67 ms vs Morton (profiles/r02/um_order*.json);
    // KLE_UMESH_ORDER=0 selects Morton
    const char *oe = getenv("KLE_UMESH_ORDER");
    const bool hilbert = !(oe && atoi(oe) == 0);
    for (int64_t v : ord) {
        uint64_t c = 0;
        uint32_t q[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) {
            const double s = hi[d] > lo[d] ? (X[v * dim + d] - lo[d]) / (hi[d] - lo[d]) : 0.0;
            const uint64_t qd = (uint64_t)std::min(2097151.0, std::max(0.0, s * 2097151.0));
            q[d] = (uint32_t)qd;
            c |= spread3(qd) << d;
        }
        code[v] = hilbert ? hilbert_key(q, dim, 21) : c;
    }
    auto seg = [&](int64_t v) { return seglo[v] ? 0 : seghi[v] ? 2 : 1; };
    std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
        if (own[a] != own[b]) return own[a] < own[b];
        if (seg(a) != seg(b)) return seg(a) < seg(b);
        if (code[a] != code[b]) return code[a] < code[b];
        return a < b;
    });
    std::vector<int64_t> gid(NT, -1);
    for (int64_t k = 0; k < N; ++k) gid[ord[k]] = k;
    std::vector<int64_t> rbeg(nranks + 1, 0), nlo(nranks, 0), nhi(nranks, 0);
    for (int64_t v : ord) {
        rbeg[own[v] + 1]++;
        if (seglo[v]) nlo[own[v]]++;
        if (seghi[v]) nhi[own[v]]++;
    }
    for (int r = 0; r < nranks; ++r) rbeg[r + 1] += rbeg[r];
    for (int r = 0; r < nranks; ++r)
        if (rbeg[r + 1] == rbeg[r]) return fail(KLE_ERR_ARG, "rank %d owns no node (use fewer ranks)", r);

    // local cells: every cell with a node owned here, ascending id
    std::vector<int64_t> lcells;
    for (int64_t c = 0; c < ncells; ++c) {
        if (emin[c] > rank || emax[c] < rank) continue;
        bool mine = slab;
        for (int l = 0; l < nn && !mine; ++l) mine = own[B.tmp[c * nn + l]] == rank;
        if (mine) lcells.push_back(c);
    }
    // ext layout and pseudo ids (tmp id -> pseudo id, -1 outside the ext range)
    std::vector<int64_t> loc(NT, -1), ext_gid;
    int64_t ext_begin, ext_end;
    kle::PlanPtr plan;
    if (slab || nranks == 1) {
        ext_begin = rbeg[rank] - (rank > 0 ? nhi[rank - 1] : 0);
        ext_end = rbeg[rank + 1] + (rank < nranks - 1 ? nlo[rank + 1] : 0);
        for (int64_t v : ord)
            if (gid[v] >= ext_begin && gid[v] < ext_end) loc[v] = gid[v];
    } else {
        // ghosts: nodes of local cells owned elsewhere, ascending global id
        // (= grouped by owner rank, since ids are numbered owner-major)
        std::vector<int64_t> ghosts;
        for (int64_t c : lcells)
            for (int l = 0; l < nn; ++l) {
                const int64_t v = B.tmp[c * nn + l];
                if (own[v] != rank) ghosts.push_back(gid[v]);
            }
        std::sort(ghosts.begin(), ghosts.end());
        ghosts.erase(std::unique(ghosts.begin(), ghosts.end()), ghosts.end());
        const int64_t nglo = std::lower_bound(ghosts.begin(), ghosts.end(), rbeg[rank]) - ghosts.begin();
        ext_begin = rbeg[rank] - nglo;
        ext_end = rbeg[rank + 1] + ((int64_t)ghosts.size() - nglo);
        ext_gid.resize(ext_end - ext_begin);
        for (int64_t k = 0; k < nglo; ++k) ext_gid[k] = ghosts[k];
        for (int64_t g = rbeg[rank]; g < rbeg[rank + 1]; ++g) ext_gid[nglo + g - rbeg[rank]] = g;
        for (size_t k = nglo; k < ghosts.size(); ++k) ext_gid[nglo + (rbeg[rank + 1] - rbeg[rank]) + (k - nglo)] = ghosts[k];
        for (int64_t k = 0; k < (int64_t)ext_gid.size(); ++k) loc[ord[ext_gid[k]]] = ext_begin + k;
        // halo plan: receive each peer's ghost group in place; send the owned
        // nodes that sit in the peer's local cells, ascending global id
        plan = std::make_shared<kle::HaloPlan>();
        plan->n_owned = rbeg[rank + 1] - rbeg[rank];
        std::map<int, std::vector<int64_t>> sends;
        std::vector<int> owners;
        for (int64_t c = 0; c < ncells; ++c) {
            if (emin[c] == emax[c] || emin[c] > rank || emax[c] < rank) continue;
            owners.clear();
            bool mine = false;
            for (int l = 0; l < nn; ++l) {
                const int o = own[B.tmp[c * nn + l]];
                mine |= o == rank;
                owners.push_back(o);
            }
            if (!mine) continue;
            std::sort(owners.begin(), owners.end());
            owners.erase(std::unique(owners.begin(), owners.end()), owners.end());
            for (int q : owners) {
                if (q == rank) continue;
                auto &lst = sends[q];
                for (int l = 0; l < nn; ++l) {
                    const int64_t v = B.tmp[c * nn + l];
                    if (own[v] == rank) lst.push_back(gid[v] - rbeg[rank]);
                }
            }
        }
        std::map<int, std::pair<int64_t, int64_t>> recvs;  // peer -> (ext offset, count)
        for (int64_t k = 0; k < (int64_t)ext_gid.size(); ++k) {
            const int64_t g = ext_gid[k];
            if (g >= rbeg[rank] && g < rbeg[rank + 1]) continue;
            const int q = (int)(std::upper_bound(rbeg.begin(), rbeg.end(), g) - rbeg.begin()) - 1;
            auto it = recvs.find(q);
            if (it == recvs.end()) recvs[q] = {k, 1};
            else it->second.second++;
        }
        for (auto &kv : sends) {
            auto &lst = kv.second;
            std::sort(lst.begin(), lst.end());
            lst.erase(std::unique(lst.begin(), lst.end()), lst.end());
            if (!recvs.count(kv.first)) return fail(KLE_ERR_STATE, "halo plan: rank %d sends to %d but receives nothing", rank, kv.first);
        }
        for (auto &kv : recvs) {
            const int q = kv.first;
            auto it = sends.find(q);
            if (it == sends.end()) return fail(KLE_ERR_STATE, "halo plan: rank %d receives from %d but sends nothing", rank, q);
            plan->peers.push_back(q);
            plan->recv_off.push_back(kv.second.first);
            plan->recv_cnt.push_back(kv.second.second);
            plan->send_off.push_back((int64_t)plan->send_idx.size());
            plan->send_cnt.push_back((int64_t)it->second.size());
            for (int64_t o : it->second) plan->send_idx.push_back((int32_t)o);
        }
    }

    kle_mesh *m = new kle_mesh;
    m->kind = 1;
    m->dim = dim;
    m->ngl = ngl;
    m->p = p;
    m->rank = rank;
    m->nranks = nranks;
    m->N = N;
    m->E = ncells;
    m->nel[0] = ncells;
    m->nel[1] = m->nel[2] = 1;
    m->L[0] = m->L[1] = m->L[2] = 0;
    for (int d = 0; d < 3; ++d) {
        m->lower[d] = d < dim ? lo[d] : 0.0;
        m->upper[d] = d < dim ? hi[d] : 0.0;
    }
    m->xi = xi;
    m->axis = slab ? ax : -1;
    m->node_begin = rbeg[rank];
    m->node_end = rbeg[rank + 1];
    m->ext_begin = ext_begin;
    m->ext_end = ext_end;
    m->plan = plan;
    m->ext_gid = std::move(ext_gid);
    if (slab && rank > 0) {
        m->halo_lo_rank = rank - 1;
        m->halo_lo_nodes = nhi[rank - 1];
        m->send_lo_nodes = nlo[rank];
    }
    if (slab && rank < nranks - 1) {
        m->halo_hi_rank = rank + 1;
        m->halo_hi_nodes = nlo[rank + 1];
        m->send_hi_nodes = nhi[rank];
    }
    m->u_elem = std::move(lcells);
    const int64_t nle = (int64_t)m->u_elem.size();
    m->elem_begin = 0;
    m->elem_end = nle;
    m->u_conn.resize((size_t)nle * nn);
    m->u_corners.resize((size_t)nle * nc * dim);
    const int64_t next = m->ext_end - m->ext_begin, nown = m->node_end - m->node_begin;
    m->u_incp.assign(nown + 1, 0);
    for (int64_t e = 0; e < nle; ++e) {
        const int64_t c = m->u_elem[e];
        for (int l = 0; l < nn; ++l) {
            const int64_t g = loc[B.tmp[c * nn + l]];
            if (g < 0) {
                delete m;
                return fail(KLE_ERR_STATE, "cell %lld node outside the ext range", (long long)c);
            }
            m->u_conn[e * nn + l] = g;
            if (g >= m->node_begin && g < m->node_end) m->u_incp[g - m->node_begin + 1]++;
        }
        for (int s = 0; s < nc; ++s)
            for (int d = 0; d < dim; ++d)
                m->u_corners[(e * nc + s) * dim + d] = corner(c, dim == 2 ? C2T2[s] : C2T3[s], d);
    }
    for (int64_t i = 0; i < nown; ++i) m->u_incp[i + 1] += m->u_incp[i];
    m->u_inc.resize(m->u_incp[nown]);
    {
        std::vector<int64_t> fill(m->u_incp.begin(), m->u_incp.end() - 1);
        for (int64_t e = 0; e < nle; ++e)
            for (int l = 0; l < nn; ++l) {
                const int64_t g = m->u_conn[e * nn + l];
                if (g >= m->node_begin && g < m->node_end) m->u_inc[fill[g - m->node_begin]++] = (int32_t)(e * nn + l);
            }
    }
    m->u_coords.resize((size_t)next * dim);
    for (int64_t v : ord) {
        const int64_t g = loc[v];
        if (g < 0) continue;
        for (int d = 0; d < dim; ++d) m->u_coords[(g - m->ext_begin) * dim + d] = X[v * dim + d];
    }
    // Face Sets: a cell face (edge in 2-D) matching a tagged facet marks all its nodes
    m->u_tags.assign(next, 0);
    if (nfacets > 0) {
        std::unordered_map<Key, uint32_t, KeyHash> ftag;
        ftag.reserve(nfacets * 2);
        for (int64_t f = 0; f < nfacets; ++f) {
            const int t = facet_tags[f];
            if (t < 1 || t > 32) continue;  // untagged / out of the label range
            Key k{-1, -1, -1, -1};
            for (int j = 0; j < nfv; ++j) k[j] = facets[f * nfv + j];
            std::sort(k.begin(), k.begin() + nfv);
            ftag[k] |= 1u << (t - 1);
        }
        for (int64_t c = 0; c < ncells; ++c) {
            const int64_t *V = &B.tv[c * nc];
            for (int d = 0; d < dim; ++d)
                for (int side = 0; side < 2; ++side) {
                    Key k{-1, -1, -1, -1};
                    int j = 0;
                    for (int t = 0; t < nc; ++t)
                        if (((t >> d) & 1) == side) k[j++] = V[t];
                    std::sort(k.begin(), k.begin() + nfv);
                    auto it = ftag.find(k);
                    if (it == ftag.end()) continue;
                    for (int l = 0; l < nn; ++l) {
                        const int q = d == 0 ? l % ngl : d == 1 ? (l / ngl) % ngl : l / (ngl * ngl);
                        if (q != (side ? p : 0)) continue;
                        const int64_t g = loc[B.tmp[c * nn + l]];
                        if (g >= 0) m->u_tags[g - m->ext_begin] |= it->second;
                    }
                }
        }
    }
    m->dir.assign(next, 0);
    *out = m;
    return 0;
}

// Gmsh MSH 4.1 ASCII reader (the format of the reference's fixture
// src/tests/test.msh): $Entities physical tags, $Nodes blocks, $Elements
// blocks.  Cells: 4-node quads (type 3) in 2-D, 8-node hexes (type 5) in 3-D,
// in file order (DMPlex cell numbering).  Facets: 2-node lines (type 1) / quads
// of the boundary carry their entity's first physical tag as the Face Sets
// value.  Points (type 15) are ignored; any other element type is refused.
int kle_mesh_create_gmsh(const char *path, int ngl, int rank, int nranks, kle_mesh **out)
{
    KLE_ARG(path && out, "null arg");
    std::ifstream f(path);
    if (!f) return fail(KLE_ERR_ARG, "cannot open gmsh file '%s'", path);
    std::string tok;
    std::map<std::pair<int, int>, int> ent_phys;  // (dim, entity tag) -> first physical tag
    std::unordered_map<int64_t, int64_t> node_index;
    std::vector<double> vx;
    struct Blk {
        int dim, etag, type;
        std::vector<int64_t> nodes;  // flattened
    };
    std::vector<Blk> blocks;
    bool have_format = false;
    while (f >> tok) {
        if (tok == "$MeshFormat") {
            double ver;
            int ftype, dsize;
            f >> ver >> ftype >> dsize;
            if (ver < 4.0 || ver >= 5.0) return fail(KLE_ERR_SUP, "gmsh format %g: only MSH 4.x is read", ver);
            if (ftype != 0) return fail(KLE_ERR_SUP, "binary gmsh files are not read (save as ASCII)");
            have_format = true;
        } else if (tok == "$Entities") {
            int64_t cnt[4];
            f >> cnt[0] >> cnt[1] >> cnt[2] >> cnt[3];
            for (int d = 0; d < 4; ++d)
                for (int64_t k = 0; k < cnt[d]; ++k) {
                    int tag;
                    double dummy;
                    f >> tag;
                    for (int j = 0; j < (d == 0 ? 3 : 6); ++j) f >> dummy;
                    int64_t nphys;
                    f >> nphys;
                    int first = 0;
                    for (int64_t j = 0; j < nphys; ++j) {
                        int t;
                        f >> t;
                        if (j == 0) first = t;
                    }
                    if (nphys > 0) ent_phys[{d, tag}] = std::abs(first);
                    if (d > 0) {
                        int64_t nb;
                        f >> nb;
                        for (int64_t j = 0; j < nb; ++j) f >> tag;
                    }
                }
        } else if (tok == "$Nodes") {
            int64_t nblk, nnodes, mn, mx;
            f >> nblk >> nnodes >> mn >> mx;
            vx.reserve(nnodes * 3);
            for (int64_t b = 0; b < nblk; ++b) {
                int edim, etag, para;
                int64_t n;
                f >> edim >> etag >> para >> n;
                std::vector<int64_t> tags(n);
                for (auto &t : tags) f >> t;
                for (int64_t k = 0; k < n; ++k) {
                    double x, y, z, u;
                    f >> x >> y >> z;
                    if (para)
                        for (int j = 0; j < edim; ++j) f >> u;
                    node_index[tags[k]] = (int64_t)vx.size() / 3;
                    vx.push_back(x);
                    vx.push_back(y);
                    vx.push_back(z);
                }
            }
        } else if (tok == "$Elements") {
            int64_t nblk, nel, mn, mx;
            f >> nblk >> nel >> mn >> mx;
            for (int64_t b = 0; b < nblk; ++b) {
                Blk B;
                int64_t n;
                f >> B.dim >> B.etag >> B.type >> n;
                const int nv = B.type == 1 ? 2 : B.type == 3 ? 4 : B.type == 5 ? 8 : B.type == 15 ? 1 : -1;
                if (nv < 0)
                    return fail(KLE_ERR_SUP, "gmsh element type %d is not supported (quads/hexes only)", B.type);
                B.nodes.resize(n * nv);
                for (int64_t k = 0; k < n; ++k) {
                    int64_t etag;
                    f >> etag;
                    for (int j = 0; j < nv; ++j) f >> B.nodes[k * nv + j];
                }
                blocks.push_back(std::move(B));
            }
        }
        if (!f) return fail(KLE_ERR_ARG, "malformed gmsh file '%s' near '%s'", path, tok.c_str());
    }
    if (!have_format) return fail(KLE_ERR_ARG, "'%s' has no $MeshFormat section", path);
    int dim = 0;
    for (auto &B : blocks)
        if (B.type == 3 || B.type == 5) dim = std::max(dim, B.type == 5 ? 3 : 2);
    if (!dim) return fail(KLE_ERR_ARG, "'%s' holds no quadrilateral or hexahedral cells", path);
    const int nc = 1 << dim, cell_type = dim == 3 ? 5 : 3, facet_type = dim == 3 ? 3 : 1;
    std::vector<int64_t> cells, facets;
    std::vector<int> ftags;
    auto idx = [&](int64_t tag, int64_t &o) {
        auto it = node_index.find(tag);
        if (it == node_index.end()) return false;
        o = it->second;
        return true;
    };
    for (auto &B : blocks) {
        if (B.type == cell_type && B.dim == dim) {
            for (size_t k = 0; k < B.nodes.size(); ++k) {
                int64_t o;
                if (!idx(B.nodes[k], o)) return fail(KLE_ERR_ARG, "element references unknown node %lld", (long long)B.nodes[k]);
                cells.push_back(o);
            }
        } else if (B.type == facet_type && B.dim == dim - 1) {
            auto it = ent_phys.find({B.dim, B.etag});
            const int t = it == ent_phys.end() ? 0 : it->second;
            const int nfv = nc / 2;
            for (size_t k = 0; k < B.nodes.size() / nfv; ++k) {
                for (int j = 0; j < nfv; ++j) {
                    int64_t o;
                    if (!idx(B.nodes[k * nfv + j], o)) return fail(KLE_ERR_ARG, "facet references unknown node");
                    facets.push_back(o);
                }
                ftags.push_back(t);
            }
        }
    }
    // 2-D meshes keep (x, y); the reader passes 3 components per vertex
    return kle_mesh_create_unstructured(dim, ngl, (int64_t)vx.size() / 3, vx.data(), (int64_t)cells.size() / nc,
                                        cells.data(), (int64_t)ftags.size(), facets.empty() ? nullptr : facets.data(),
                                        ftags.empty() ? nullptr : ftags.data(), rank, nranks, out);
}

}  // extern "C"
