// kle_mesh.cpp -- structured box mesh, slab partition and symbolic patterns.
// Host-only (no HIP calls): usable and testable without a GPU.
//
// Replaces, for structured box meshes, the reference's DMPlex path:
//   BoxDom.create / DMPlexDistribute      dmplex.py:18-29,382-388
//   setFemIndexing (PetscSection offsets)  dmplex.py:31-49, indices.py:22-30
//   getGlobalNodesFromCell                 dmplex.py:193-196, indices.py:70-96
//   getConnectivityNodes (adjacency)       dmplex.py:352-372
//   getBorderNodes / Face Sets             dmplex.py:160-166
//   preAlloc_K_Krhs / preAlloc_Rd_Rw       mat_fs.py:21-94
// Canonical numbering: lattice node id = ix + Lx (iy + Ly iz); cells x-fastest;
// element-local nodes in tensor order (a along x fastest).
#include <algorithm>
#include <cstdlib>
#include <thread>
#include <cmath>
#include <cstring>

#include "kle_basis.hpp"
#include "kle_internal.hpp"

using namespace kle;

namespace {

// DMPlex closure order of the cell corners (test_dmplex_wrapper.py:24-27,106-115)
const int CORN2[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
const int CORN3[8][3] = {{0, 0, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0},
                         {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};

// neighbour box of lattice coordinate c along one axis (nodes sharing a cell)
inline void nbr_range(const kle_mesh *m, int d, int64_t c, int64_t &lo, int64_t &hi)
{
    if (d >= m->dim) {
        lo = hi = 0;
        return;
    }
    const int p = m->p;
    if (c % p == 0) {
        lo = std::max<int64_t>(0, c - p);
        hi = std::min<int64_t>(m->L[d] - 1, c + p);
    } else {
        lo = (c / p) * p;
        hi = lo + p;
    }
}

inline bool is_dir(const kle_mesh *m, int64_t node) { return m->dir[node - m->ext_begin] != 0; }

}  // namespace

// which: 0 K (free x free, Dirichlet rows diagonal), 1 Krhs (free x Dirichlet,
// Dirichlet rows diagonal), 2 Rw (free x all, Dirichlet rows empty),
// 3 operators Curl/SrT/DivSrT (all x all, mat_fs.py:215-236); no-slip
// (dir = no-slip nodes): 4 Kfs (free rows x no-slip nodes, no-slip rows x all),
// 5 Krhsfs (all rows x no-slip nodes), 6 Rwfs (no-slip rows x all), mat_ns.py:7-45,86-122.
// Enumerates the columns of owned node row i in ascending order.
template <class F>
static void row_cols(const kle_mesh *m, int which, int64_t i, F &&emit)
{
    const bool di = is_dir(m, i);
    if (which == 6 && !di) return;
    if (which <= 2 && di) {
        if (which != 2) emit(i);
        return;
    }
    auto filter = [&](int64_t j) {
        switch (which) {
        case 0: return !is_dir(m, j);
        case 1: return is_dir(m, j);
        case 4: return di || is_dir(m, j);
        case 5: return is_dir(m, j);
        default: return true;  // 2, 3, 6
        }
    };
    if (m->kind == 1) {
        thread_local std::vector<int64_t> nb;
        umesh_row_nodes(m, i - m->node_begin, nb);
        for (int64_t j : nb)
            if (filter(j)) emit(j);
        return;
    }
    int64_t c[3], lo[3], hi[3];
    m->lattice_of(i, c);
    for (int d = 0; d < 3; ++d) nbr_range(m, d, c[d], lo[d], hi[d]);
    int64_t q[3];
    for (q[2] = lo[2]; q[2] <= hi[2]; ++q[2])
        for (q[1] = lo[1]; q[1] <= hi[1]; ++q[1])
            for (q[0] = lo[0]; q[0] <= hi[0]; ++q[0]) {
                const int64_t j = m->id_of(q);
                if (filter(j)) emit(j);
            }
}

namespace kle {

int host_threads()
{
    int n = (int)std::thread::hardware_concurrency();
    if (const char *e = getenv("OMP_NUM_THREADS")) n = atoi(e);
    return std::max(1, std::min(n, 16));
}

void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)> &f)
{
    const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 4096));
    if (nt <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
    for (auto &th : pool) th.join();
}

int pattern_csr(const kle_mesh *m, int which, std::vector<int64_t> &rp, std::vector<int64_t> &cols)
{
    const int64_t n = m->node_end - m->node_begin;
    rp.assign(n + 1, 0);
    parallel_for(n, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            int64_t c = 0;
            row_cols(m, which, m->node_begin + i, [&](int64_t) { ++c; });
            rp[i + 1] = c;
        }
    });
    for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
    cols.resize(std::max<int64_t>(rp[n], 1));
    parallel_for(n, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            int64_t k = rp[i];
            row_cols(m, which, m->node_begin + i, [&](int64_t j) { cols[k++] = j; });
        }
    });
    return 0;
}

}  // namespace kle

int64_t kle_mesh::to_pseudo(int64_t gid) const
{
    if (ext_gid.empty()) return gid >= ext_begin && gid < ext_end ? gid : -1;
    // ext_gid ascends (ghost groups ordered by owner, owners number their nodes contiguously)
    auto it = std::lower_bound(ext_gid.begin(), ext_gid.end(), gid);
    return it != ext_gid.end() && *it == gid ? ext_begin + (it - ext_gid.begin()) : -1;
}

extern "C" {

int kle_mesh_create_box(int dim, const int64_t nelem[3], const double lower[3], const double upper[3],
                        int ngl, int rank, int nranks, kle_mesh **out)
{
    KLE_ARG(out && nelem && lower && upper, "null arg");
    KLE_ARG(dim == 2 || dim == 3, "dim must be 2 or 3");
    KLE_ARG(ngl >= 2 && ngl <= 8, "ngl must be in [2,8] (got %d)", ngl);
    KLE_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank");
    kle_mesh *m = new kle_mesh;
    m->dim = dim;
    m->ngl = ngl;
    m->p = ngl - 1;
    m->rank = rank;
    m->nranks = nranks;
    m->N = 1;
    m->E = 1;
    for (int d = 0; d < dim; ++d) {
        if (nelem[d] < 1 || !(upper[d] > lower[d])) {
            delete m;
            return fail(KLE_ERR_ARG, "bad box along axis %d", d);
        }
        m->nel[d] = nelem[d];
        m->L[d] = nelem[d] * m->p + 1;
        m->lower[d] = lower[d];
        m->upper[d] = upper[d];
        m->h[d] = (upper[d] - lower[d]) / nelem[d];
        m->N *= m->L[d];
        m->E *= nelem[d];
    }
    std::vector<double> x, w;
    gauss_lobatto(ngl, x, w);
    m->xi.resize(ngl);
    for (int i = 0; i < ngl; ++i) m->xi[i] = (1.0 + x[i]) / 2.0;
    // slab partition along the slowest axis by whole element layers
    const int A = dim - 1;
    m->axis = A;
    m->plane = 1;
    m->elem_layer = 1;
    for (int d = 0; d < A; ++d) {
        m->plane *= m->L[d];
        m->elem_layer *= m->nel[d];
    }
    const int64_t layers = m->nel[A];
    if (nranks > layers) {
        delete m;
        return fail(KLE_ERR_ARG, "%d ranks > %lld element layers along the partition axis", nranks,
                    (long long)layers);
    }
    auto layer0 = [&](int r) { return layers * r / nranks; };
    const int64_t e0 = layer0(rank), e1 = layer0(rank + 1);
    const int p = m->p;
    m->pl0 = e0 * p;
    m->pl1 = (rank == nranks - 1) ? m->L[A] : e1 * p;
    m->xl0 = std::max<int64_t>(0, m->pl0 - p);
    m->xl1 = std::min<int64_t>(m->L[A], m->pl1 + 1);
    m->el0 = std::max<int64_t>(0, e0 - 1);
    m->el1 = e1;
    m->node_begin = m->pl0 * m->plane;
    m->node_end = m->pl1 * m->plane;
    m->ext_begin = m->xl0 * m->plane;
    m->ext_end = m->xl1 * m->plane;
    m->elem_begin = m->el0 * m->elem_layer;
    m->elem_end = m->el1 * m->elem_layer;
    if (rank > 0) {
        m->halo_lo_rank = rank - 1;
        m->halo_lo_nodes = m->node_begin - m->ext_begin;
        m->send_lo_nodes = m->plane;  // the lower neighbour's single upper ghost plane
    }
    if (rank < nranks - 1) {
        m->halo_hi_rank = rank + 1;
        m->halo_hi_nodes = m->ext_end - m->node_end;
        // the upper neighbour's lower ghosts: min(p, its first plane) planes
        m->send_hi_nodes = std::min<int64_t>(p, m->pl1 - m->pl0) * m->plane;
    }
    m->dir.assign(m->ext_end - m->ext_begin, 0);
    *out = m;
    return 0;
}

int kle_mesh_destroy(kle_mesh *m)
{
    delete m;
    return 0;
}

int kle_set_partitioner(int method)
{
    KLE_ARG(method == 0 || method == 1, "partitioner must be 0 (inertial) or 1 (slab), got %d", method);
    g_partitioner = method;
    return 0;
}

int kle_get_partitioner(void) { return g_partitioner; }

int kle_mesh_get_peers(const kle_mesh *m, int *npeers, int *ranks, int64_t *recv_nodes, int64_t *send_nodes,
                       int64_t *send_list)
{
    KLE_ARG(m && npeers, "null arg");
    if (!m->plan) {
        int k = 0;
        for (int q : {m->halo_lo_rank, m->halo_hi_rank}) {
            if (q < 0) continue;
            if (ranks) ranks[k] = q;
            const bool lo = q == m->halo_lo_rank;
            if (recv_nodes) recv_nodes[k] = lo ? m->halo_lo_nodes : m->halo_hi_nodes;
            if (send_nodes) send_nodes[k] = lo ? m->send_lo_nodes : m->send_hi_nodes;
            ++k;
        }
        if (send_list) {  // contiguous ranges: lowest / highest owned nodes
            int64_t z = 0;
            const int64_t own = m->node_end - m->node_begin;
            if (m->halo_lo_rank >= 0)
                for (int64_t i = 0; i < m->send_lo_nodes; ++i) send_list[z++] = i;
            if (m->halo_hi_rank >= 0)
                for (int64_t i = own - m->send_hi_nodes; i < own; ++i) send_list[z++] = i;
        }
        *npeers = k;
        return 0;
    }
    const HaloPlan &P = *m->plan;
    *npeers = (int)P.peers.size();
    for (size_t k = 0; k < P.peers.size(); ++k) {
        if (ranks) ranks[k] = P.peers[k];
        if (recv_nodes) recv_nodes[k] = P.recv_cnt[k];
        if (send_nodes) send_nodes[k] = P.send_cnt[k];
    }
    if (send_list) std::copy(P.send_idx.begin(), P.send_idx.end(), send_list);
    return 0;
}

int kle_mesh_get_ext_gids(const kle_mesh *m, int64_t *gids)
{
    KLE_ARG(m && gids, "null arg");
    for (int64_t k = m->ext_begin; k < m->ext_end; ++k) gids[k - m->ext_begin] = m->to_global(k);
    return 0;
}

int kle_mesh_get_info(const kle_mesh *m, kle_mesh_info *info)
{
    KLE_ARG(m && info, "null arg");
    memset(info, 0, sizeof(*info));
    info->dim = m->dim;
    info->ngl = m->ngl;
    info->rank = m->rank;
    info->nranks = m->nranks;
    for (int d = 0; d < 3; ++d) {
        info->nelem[d] = d < m->dim ? m->nel[d] : 1;
        info->lattice[d] = d < m->dim ? m->L[d] : 1;
    }
    info->n_nodes = m->N;
    info->n_elems = m->E;
    info->node_begin = m->node_begin;
    info->node_end = m->node_end;
    info->ext_begin = m->ext_begin;
    info->ext_end = m->ext_end;
    info->elem_begin = m->elem_begin;
    info->elem_end = m->elem_end;
    info->kind = m->kind;
    info->axis = m->axis;
    if (m->kind == 1) info->lattice[0] = info->lattice[1] = info->lattice[2] = 0;
    return 0;
}

int kle_mesh_get_elements(const kle_mesh *m, int64_t *ids)
{
    KLE_ARG(m && ids, "null arg");
    if (m->kind == 1) std::copy(m->u_elem.begin(), m->u_elem.end(), ids);
    else
        for (int64_t e = m->elem_begin; e < m->elem_end; ++e) ids[e - m->elem_begin] = e;
    return 0;
}

int kle_mesh_get_conn(const kle_mesh *m, int64_t *conn)
{
    KLE_ARG(m && conn, "null arg");
    if (m->kind == 1) {
        for (size_t k = 0; k < m->u_conn.size(); ++k) conn[k] = m->to_global(m->u_conn[k]);
        return 0;
    }
    const int ngl = m->ngl, nn = m->nn(), p = m->p;
    for (int64_t e = m->elem_begin; e < m->elem_end; ++e) {
        int64_t ex = e % m->nel[0], ey = (e / m->nel[0]) % m->nel[1], ez = e / (m->nel[0] * m->nel[1]);
        int64_t *out = conn + (e - m->elem_begin) * nn;
        for (int l = 0; l < nn; ++l) {
            int a = l % ngl, b = (l / ngl) % ngl, c = m->dim == 3 ? l / (ngl * ngl) : 0;
            int64_t lat[3] = {ex * p + a, ey * p + b, m->dim == 3 ? ez * p + c : 0};
            out[l] = m->id_of(lat);
        }
    }
    return 0;
}

int kle_mesh_get_corners(const kle_mesh *m, double *xyz)
{
    KLE_ARG(m && xyz, "null arg");
    if (m->kind == 1) {
        std::copy(m->u_corners.begin(), m->u_corners.end(), xyz);
        return 0;
    }
    const int nc = 1 << m->dim;
    for (int64_t e = m->elem_begin; e < m->elem_end; ++e) {
        int64_t ei[3] = {e % m->nel[0], (e / m->nel[0]) % m->nel[1], e / (m->nel[0] * m->nel[1])};
        double *o = xyz + (e - m->elem_begin) * nc * m->dim;
        for (int c = 0; c < nc; ++c)
            for (int d = 0; d < m->dim; ++d) {
                int off = m->dim == 2 ? CORN2[c][d] : CORN3[c][d];
                o[c * m->dim + d] = m->lower[d] + (ei[d] + off) * m->h[d];
            }
    }
    return 0;
}

int kle_mesh_get_coords(const kle_mesh *m, double *xyz)
{
    KLE_ARG(m && xyz, "null arg");
    if (m->kind == 1) {
        std::copy(m->u_coords.begin() + (m->node_begin - m->ext_begin) * m->dim,
                  m->u_coords.begin() + (m->node_end - m->ext_begin) * m->dim, xyz);
        return 0;
    }
    for (int64_t n = m->node_begin; n < m->node_end; ++n) {
        int64_t c[3];
        m->lattice_of(n, c);
        for (int d = 0; d < m->dim; ++d) {
            double v;
            if (c[d] == m->L[d] - 1) v = m->upper[d];
            else v = m->lower[d] + (double)(c[d] / m->p + m->xi[c[d] % m->p]) * m->h[d];
            xyz[(n - m->node_begin) * m->dim + d] = v;
        }
    }
    return 0;
}

// face bit -> (axis, side): reference names (dmplex.py:27-30, boundary.py:130)
static bool face_axis(int dim, int f, int &axis, int &side)
{
    static const int F3[6][2] = {{2, 0}, {2, 1}, {1, 0}, {1, 1}, {0, 1}, {0, 0}};
    static const int F2[4][2] = {{1, 0}, {0, 1}, {1, 1}, {0, 0}};
    if (dim == 3 && f < 6) {
        axis = F3[f][0];
        side = F3[f][1];
        return true;
    }
    if (dim == 2 && f < 4) {
        axis = F2[f][0];
        side = F2[f][1];
        return true;
    }
    return false;
}

static bool on_faces(const kle_mesh *m, int64_t node, unsigned mask)
{
    if (m->kind == 1) return (m->u_tags[node - m->ext_begin] & mask) != 0;
    int64_t c[3];
    m->lattice_of(node, c);
    for (int f = 0; f < 6; ++f) {
        if (!(mask & (1u << f))) continue;
        int axis, side;
        if (!face_axis(m->dim, f, axis, side)) continue;
        if (c[axis] == (side ? m->L[axis] - 1 : 0)) return true;
    }
    return false;
}

int kle_mesh_face_nodes(const kle_mesh *m, unsigned mask, int64_t *nodes, int64_t *n)
{
    KLE_ARG(m && n, "null arg");
    int64_t k = 0;
    for (int64_t i = m->node_begin; i < m->node_end; ++i)
        if (on_faces(m, i, mask)) {
            if (nodes) nodes[k] = i;
            ++k;
        }
    *n = k;
    return 0;
}

int kle_mesh_set_dirichlet_faces(kle_mesh *m, unsigned mask)
{
    KLE_ARG(m, "null mesh");
    for (int64_t i = m->ext_begin; i < m->ext_end; ++i) m->dir[i - m->ext_begin] = on_faces(m, i, mask);
    m->dir_set = true;
    return 0;
}

int kle_mesh_set_dirichlet_nodes(kle_mesh *m, const int64_t *nodes, int64_t n)
{
    KLE_ARG(m && (n == 0 || nodes), "null arg");
    std::fill(m->dir.begin(), m->dir.end(), 0);
    for (int64_t k = 0; k < n; ++k) {
        if (nodes[k] < 0 || nodes[k] >= m->N) return fail(KLE_ERR_OUTOFRANGE, "node %lld", (long long)nodes[k]);
        const int64_t q = m->to_pseudo(nodes[k]);
        if (q >= 0) m->dir[q - m->ext_begin] = 1;
    }
    m->dir_set = true;
    return 0;
}

int kle_mesh_set_noslip_dofs(kle_mesh *m, const int64_t *tang, int64_t nt, const int64_t *normal, int64_t nnorm)
{
    KLE_ARG(m && (nt == 0 || tang) && (nnorm == 0 || normal), "null arg");
    const int64_t next = m->ext_end - m->ext_begin;
    m->dof_cls.assign(next * m->dim, DOF_FREE);
    std::fill(m->dir.begin(), m->dir.end(), 0);
    auto mark = [&](const int64_t *dofs, int64_t n, uint8_t c) -> int {
        for (int64_t k = 0; k < n; ++k) {
            if (dofs[k] < 0 || dofs[k] >= m->N * m->dim) return fail(KLE_ERR_OUTOFRANGE, "dof %lld", (long long)dofs[k]);
            const int64_t q = m->to_pseudo(dofs[k] / m->dim);
            if (q < 0) continue;
            // a DoF both normal and tangential is normal (mat_ns.py:60-62)
            uint8_t &slot = m->dof_cls[(q - m->ext_begin) * m->dim + dofs[k] % m->dim];
            slot = std::max(slot, c);
            m->dir[q - m->ext_begin] = 1;
        }
        return 0;
    };
    KLE_TRY(mark(tang, nt, DOF_TANG));
    KLE_TRY(mark(normal, nnorm, DOF_NORMAL));
    m->dir_set = true;
    return 0;
}

int kle_mesh_set_noslip_faces(kle_mesh *m, const int *faces, int nfaces)
{
    KLE_ARG(m && (nfaces == 0 || faces), "null arg");
    // the wall's normal axis comes from its name (NsWalls, nswalls.py), also on
    // unstructured meshes, whose Face Sets values map to the same names
    int axes[6];
    for (int k = 0; k < nfaces; ++k) {
        int side;
        if (!face_axis(m->dim, faces[k], axes[k], side)) return fail(KLE_ERR_ARG, "bad face %d", faces[k]);
    }
    const int64_t next = m->ext_end - m->ext_begin;
    m->dof_cls.assign(next * m->dim, DOF_FREE);
    for (int64_t i = 0; i < next; ++i) {
        const int64_t node = m->ext_begin + i;
        bool normal[3] = {false, false, false}, tang[3] = {false, false, false}, drop_x = false, y_normal = false;
        bool on_any = false;
        for (int k = 0; k < nfaces; ++k) {
            if (!on_faces(m, node, 1u << faces[k])) continue;
            on_any = true;
            // getNoSlipNormalDofs(allGather=True) (boundary_conditions.py:222-238): a
            // left/right x-normal DoF is dropped when the node's y DoF is already
            // normal from an earlier (up/down) wall
            if (axes[k] == 0 && y_normal) drop_x = true;
            normal[axes[k]] = true;
            if (axes[k] == 1) y_normal = true;
            for (int d = 0; d < m->dim; ++d)
                if (d != axes[k]) tang[d] = true;
        }
        if (drop_x) normal[0] = false;
        for (int d = 0; d < m->dim; ++d)
            m->dof_cls[i * m->dim + d] = normal[d] ? DOF_NORMAL : tang[d] ? DOF_TANG : DOF_FREE;
        m->dir[i] = on_any;
    }
    m->dir_set = true;
    return 0;
}


int kle_mesh_pattern_size(const kle_mesh *m, int which, int64_t *nblocks)
{
    KLE_ARG(m && nblocks && which >= 0 && which <= 6, "bad arg");
    int64_t tot = 0;
    for (int64_t i = m->node_begin; i < m->node_end; ++i) row_cols(m, which, i, [&](int64_t) { ++tot; });
    *nblocks = tot;
    return 0;
}

int kle_mesh_pattern(const kle_mesh *m, int which, int64_t *row_ptr, int64_t *cols)
{
    KLE_ARG(m && row_ptr && which >= 0 && which <= 6, "bad arg");
    int64_t k = 0;
    row_ptr[0] = 0;
    for (int64_t i = m->node_begin; i < m->node_end; ++i) {
        row_cols(m, which, i, [&](int64_t j) {
            if (cols) cols[k] = m->to_global(j);  // pseudo order == global order (kle_umesh.cpp)
            ++k;
        });
        row_ptr[i - m->node_begin + 1] = k;
    }
    return 0;
}

int kle_mesh_halo(const kle_mesh *m, int64_t *lo_count, int64_t *hi_count, int64_t *send_lo,
                  int64_t *send_hi, int *lo_rank, int *hi_rank)
{
    KLE_ARG(m, "null mesh");
    if (lo_count) *lo_count = m->halo_lo_nodes;
    if (hi_count) *hi_count = m->halo_hi_nodes;
    if (send_lo) *send_lo = m->send_lo_nodes;
    if (send_hi) *send_hi = m->send_hi_nodes;
    if (lo_rank) *lo_rank = m->halo_lo_rank;
    if (hi_rank) *hi_rank = m->halo_hi_rank;
    return 0;
}

}  // extern "C"
