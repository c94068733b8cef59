// kle_internal.hpp -- shared internals of libkle.so (MI355X / gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kle.h"

namespace kle {

int fail(int code, const char *fmt, ...);
void clear_error();

constexpr int WAVE = 64;

#define KLE_HIP(call)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess)                                                            \
            return kle::fail(KLE_ERR_DEVICE, "%s failed: %s (%s:%d)", #call,             \
                             hipGetErrorString(e_), __FILE__, __LINE__);                 \
    } while (0)

#define KLE_NCCL(call)                                                                   \
    do {                                                                                 \
        ncclResult_t r_ = (call);                                                        \
        if (r_ != ncclSuccess)                                                           \
            return kle::fail(KLE_ERR_COMM, "%s failed: %s", #call, ncclGetErrorString(r_)); \
    } while (0)

#define KLE_TRY(call)                                                                    \
    do {                                                                                 \
        int rc_ = (call);                                                                \
        if (rc_) return rc_;                                                             \
    } while (0)

#define KLE_ARG(cond, ...)                                                               \
    do {                                                                                 \
        if (!(cond)) return kle::fail(KLE_ERR_ARG, __VA_ARGS__);                         \
    } while (0)

// Deterministic two-stage reductions: kernels write one partial per
// workgroup; a single-workgroup kernel sums them in a fixed order.
constexpr int RED_BLOCKS = 2048;   // max workgroups of the grid-stride vector kernels
constexpr int PART_STRIDE = 1 << 18;  // partial slots per reduced quantity
constexpr int NSCAL = 32;          // device scalar slots

// General halo of a graph-partitioned mesh (kle_umesh.cpp, inertial
// bisection).  The ext layout stays [ghosts of lower ranks | owned | ghosts
// of higher ranks], each peer's ghosts one contiguous group in ascending
// global id, so receives land in place; sends gather owned entries through
// an index list (the peer's order).  Counts and offsets are in nodes; a
// vector of block size bs moves bs entries per node.
struct HaloPlan {
    int64_t n_owned = 0;
    std::vector<int> peers;                   // ascending rank
    std::vector<int64_t> recv_off, recv_cnt;  // ghost group of peer k: ext nodes [recv_off, +recv_cnt)
    std::vector<int64_t> send_off, send_cnt;  // peer k's slice of send_idx
    std::vector<int32_t> send_idx;            // owned-local node index
    int32_t *d_send_idx = nullptr;            // device copies (made on first use)
    double *d_sbuf = nullptr;
    int64_t sbuf_cap = 0;
    std::vector<double> h_buf;                // host transport staging
    ~HaloPlan();
};
using PlanPtr = std::shared_ptr<HaloPlan>;
struct IpcState;  // kle_ipc.hip: IPC-mapped mailboxes (KLE_TRANSPORT=ipc)

// Device scalar slots used by the Krylov kernels.
enum Scal {
    S_RHO = 0, S_RHO_OLD, S_PQ, S_ALPHA, S_BETA, S_RR, S_TOL, S_BNORM,
    S_SUM0, S_SUM1, S_SUM2, S_SUM3,  // raw reduction outputs
    S_TMP0, S_TMP1,
    S_PRHO0, S_PRHO1, S_PALPHA0, S_PALPHA1  // pipelined CG: stage inputs, double-buffered by launch parity
};
// Device integer state: [0] reason (0 iterating), [1] iterations done,
// [2] fixed-iteration mode, [3] maxit, [4] arrival ticket of the fused
// dot + reduction kernel (zeroed with the rest at every solve start, reset
// by its last-arriving workgroup).
// I_TICKET: the last-arriver ticket word (kle_ksp.hip grid_last_arriver),
// zeroed at every solve start
// I_PITS0/1: pipelined CG iteration count, double-buffered by launch parity
enum IState { I_REASON = 0, I_ITS, I_FIXED, I_MAXIT, I_TICKET, I_PITS0, I_PITS1, I_COUNT = 8 };

}  // namespace kle

struct kle_ctx {
    int device = 0, rank = 0, nranks = 1;
    hipStream_t stream = nullptr;
    hipStream_t comm_stream = nullptr;        // halo exchange overlapped with interior SpMV rows
    hipEvent_t ev_x_ready = nullptr, ev_halo_done = nullptr;
    ncclComm_t comm = nullptr;
    bool side_busy = false;  // comm-stream kernels run beside the SpMV being launched (kle_mat.hip)
    kle_host_comm hcomm = {};         // host-staged transport (testing), used when comm == nullptr
    kle::IpcState *ipc = nullptr;     // device-to-device transport over IPC mailboxes (kle_ctx_enable_ipc)
    double *h_stage = nullptr;        // pinned staging for the host transport
    int64_t h_stage_n = 0;
    bool profiling = false;
    std::string prof_only;  // time only this kernel tag (empty: all)
    int prof_every = 1;     // time one launch in prof_every (of the filtered tags)
    int64_t prof_seq = 0;
    struct Stat {
        int64_t count = 0;
        double ms = 0;
        std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    };
    std::map<std::string, Stat> stats;
    std::vector<hipEvent_t> event_pool;
    // reduction scratch
    double *d_partials = nullptr;  // [4][PART_STRIDE]
    double *d_scal = nullptr;      // [NSCAL]
    int *d_istate = nullptr;       // [I_COUNT]
    double *h_scal = nullptr;      // pinned mirror
    int *h_istate = nullptr;
    int num_cus = 256;

    // timing helpers (no-ops unless profiling)
    int tic(const char *name, std::pair<hipEvent_t, hipEvent_t> *ev, hipStream_t s = nullptr);
    int toc(const char *name, std::pair<hipEvent_t, hipEvent_t> *ev, hipStream_t s = nullptr);
    int resolve_stats();
    hipEvent_t get_event();
};

struct kle_mesh {
    int dim = 3, ngl = 2, p = 1, rank = 0, nranks = 1;
    int64_t nel[3] = {1, 1, 1}, L[3] = {1, 1, 1};
    int64_t N = 1, E = 1;
    double lower[3] = {0, 0, 0}, upper[3] = {1, 1, 1}, h[3] = {1, 1, 1};
    std::vector<double> xi;  // GLL nodes on [0,1], ascending
    int axis = 2;            // partition axis (slowest lattice axis)
    int64_t plane = 1;       // nodes per lattice plane of the partition axis
    int64_t pl0 = 0, pl1 = 0, xl0 = 0, xl1 = 0, el0 = 0, el1 = 0;  // planes / element layers
    int64_t node_begin = 0, node_end = 0, ext_begin = 0, ext_end = 0;
    int64_t elem_begin = 0, elem_end = 0;
    int64_t elem_layer = 1;  // elements per layer of the partition axis
    std::vector<uint8_t> dir;  // Dirichlet flag per ext node (index - ext_begin)
    bool dir_set = false;
    // no-slip: class of every velocity DoF of the ext range (DOF_FREE /
    // DOF_TANG / DOF_NORMAL, mat_ns.py:58-70); empty for free-slip meshes
    std::vector<uint8_t> dof_cls;
    int halo_lo_rank = -1, halo_hi_rank = -1;
    int64_t halo_lo_nodes = 0, halo_hi_nodes = 0;   // ghost nodes received
    int64_t send_lo_nodes = 0, send_hi_nodes = 0;   // owned nodes sent to neighbours
    // kind 1 (unstructured, kle_umesh.cpp): explicit topology.  Local elements
    // are every cell touching an owned node (owned + ghost cells), ascending
    // global cell id = the reference's ADD order; node ids are global.
    int kind = 0;
    std::vector<int64_t> u_elem;    // global cell id of local element e
    std::vector<int64_t> u_conn;    // [e][nn] global node id, tensor order
    std::vector<double> u_corners;  // [e][2^dim][dim] DMPlex closure order
    std::vector<double> u_coords;   // [ext node][dim]
    std::vector<uint32_t> u_tags;   // [ext node] Face Sets bits (tag t -> bit t-1)
    std::vector<int64_t> u_incp;    // owned row i -> u_inc[u_incp[i] .. u_incp[i+1])
    std::vector<int32_t> u_inc;     // e * nn + l, ascending e
    // graph partitions: u_conn and every ext-indexed array use pseudo ids
    // ext_begin + (ext position); ext_gid maps a position to the global id
    // (empty: pseudo id == global id, the slab layouts)
    kle::PlanPtr plan;
    std::vector<int64_t> ext_gid;
    int64_t to_global(int64_t pseudo) const { return ext_gid.empty() ? pseudo : ext_gid[pseudo - ext_begin]; }
    // global id -> pseudo id, -1 when the node is not in the ext range
    int64_t to_pseudo(int64_t gid) const;
    int64_t n_local_elems() const { return kind ? (int64_t)u_elem.size() : elem_end - elem_begin; }
    int nn() const { return dim == 2 ? ngl * ngl : ngl * ngl * ngl; }
    void lattice_of(int64_t id, int64_t *c) const {
        c[0] = id % L[0];
        id /= L[0];
        c[1] = id % L[1];
        c[2] = id / L[1];
        if (dim == 2) c[2] = 0;
    }
    int64_t id_of(const int64_t *c) const { return c[0] + L[0] * (c[1] + L[1] * c[2]); }
};

struct kle_vec {
    kle_ctx *ctx = nullptr;
    int64_t n_local = 0, n_global = 0, lo = 0;  // owned [lo, lo + n_local)
    int64_t ghost_lo = 0, ghost_hi = 0;         // ghost entries before / after owned
    int bs = 1;
    double *base = nullptr;                     // allocation (ghost_lo + n_local + ghost_hi)
    double *d = nullptr;                        // = base + ghost_lo
    // halo plan (entries, not nodes)
    int lo_rank = -1, hi_rank = -1;
    int64_t send_lo = 0, send_hi = 0;
    kle::PlanPtr plan;  // general halo (graph partitions); overrides lo/hi ranks
    bool owns = true;
};

struct kle_mat {
    kle_ctx *ctx = nullptr;
    int kind = 0;  // 0 node-block, 1 scalar AIJ
    int halo_overlap = 1;          // N>1: interior rows run while the halo is in flight
    int64_t int_lo = 0, int_hi = 0;  // rows [int_lo, int_hi) read no ghost entries
    int64_t row_lat[3] = {1, 1, 1};  // lattice of the owned rows (x, y, z extents)
    int64_t m_global = 0, n_global = 0, m_local = 0, n_local = 0, row_lo = 0, col_lo = 0;
    bool empty_only = false;  // distributed generic AIJ: preallocated without entries (MatFS.Rd)
    // ---- node-block (kind 0)
    int R = 1, C = 1;
    int64_t nrows = 0;         // owned node rows
    int64_t nblocks = 0;
    int64_t node_begin = 0, ext_begin = 0, ext_nodes = 0;
    int *d_rowptr = nullptr;   // [nrows+1] block offsets (rows padded to `pad` blocks)
    int *d_rowcnt = nullptr;   // [nrows] real block count per row (null when pad == 1)
    // value layout: 0 = per-row SoA streams padded to `pad` blocks
    // (v[t * mp + k]); 1 = 16-block chunks + packed tail, rows 128-B aligned
    // (see vofs); d_vptr[i] = first double of row i in d_val
    int vlayout = 0;
    int64_t *d_vptr = nullptr;
    int64_t nvals = 0;
    // structured columns: every row's columns are the ext-lattice box
    // base + [0,nx) + Lx [0,ny) + Lx Ly [0,nz) -> the SpMV computes them
    // instead of streaming bcol (d_rowbox[2*i] = base, [2*i+1] = nx | ny<<8 | nz<<16)
    int *d_rowbox = nullptr;
    int64_t box_lx = 0, box_lxy = 0;
    int box_max = 0;  // largest row-box extent along any axis (structured columns)
    int spmv_struct = 1;  // use d_rowbox when present
    int64_t nblocks_real = 0;
    int pad = 1;
    int *d_bcol = nullptr;     // [nblocks] local ext node index
    // column dictionaries (nb_build_dict; unstructured 3x3 chunked rows): per
    // group of DICT_GROUP consecutive rows the sorted distinct columns
    // d_dict[d_dptr[g] .. d_dptr[g+1]), and per block (bcol's indexing) its
    // position in its group's dictionary
    int *d_dptr = nullptr;
    int *d_dict = nullptr;
    uint16_t *d_lid = nullptr;
    int64_t dict_len = 0;
    double *d_val = nullptr;   // [nblocks*R*C], per row SoA [a][b][k]
    // symmetric storage (kle_mat_set_symmetric = MatSetOption(MAT_SPD), PETSc
    // SBAIJ; structured 3x3 rows, one rank or z slabs): each row's blocks from
    // its diagonal block on, in the chunked layout; per-tile partial sums d_sws
    double *d_sval = nullptr;
    void *sval_raw = nullptr;  // kle_mat_move_values: the allocation d_sval lies in (freed instead of it)
    size_t sval_cap = 0;  // bytes at sval_raw
    int64_t *d_svptr = nullptr;
    double *d_sws = nullptr;
    int *d_stile_e = nullptr;  // per tile: 2^e bounds its transposed row sums (fixed-point scale, k_sym_bound)
    int *d_srow = nullptr;     // per row: offset in its box and box extents, 4 bits each (the SpMV's row set-up)
    double *d_sgsend = nullptr, *d_sgrecv = nullptr;  // N > 1 reverse halo: upper ghost rows' sums out, lowest rows' in
    int64_t sblocks = 0, snvals = 0, sws_entries = 0;  // sws_entries: lattice entries of the tile partials per SpMV
    int sym_P = 0, sym_TZ = 2, sym_TY = 8;
    int sym_wn = 0;
    size_t sws_bytes = 0;     // the partials' workspace (d_sws)  // box: per-component stride of a tile's partials in d_sws (RN, or RN rounded up to 16 doubles)
    int *d_swptr = nullptr;  // graph: per group, its partials' first double in d_sws (128-B aligned with spmv_sym_align)
    int sym_reg[5] = {};  // tile region: PX, RX, PY, RY, RZ (kle_sym.hip SymGeo); graph: slots of launch 1 / 2, groups in launch 1, G
    // graph (unstructured) symmetric storage, one rank (kle_sym.hip gsym_build):
    // d_srow = stored blocks per row, d_stile_e = per-group scale exponents,
    // d_sws = one partial per dictionary entry
    int sym_graph = 0;
    // brick decomposition of the box symmetric storage (kle_brick.hip; one
    // rank): per brick a BrickDesc, per row (brick order) 2 packed ints, per
    // brick the bricks whose regions meet its rows; d_sws holds the bricks'
    // region sums, d_stile_e their bound exponents
    int sym_brick = 0;
    int sym_gbrick = 0;  // unstructured: graph bricks (d_bdesc = GBrickDesc, d_browd = 4 ints per row)
    int brick_lds_u = 0;  // graph bricks: the largest dictionary
    int gather_rps = 0;  // run-mask gather: runs per 64-row slice (rounded up; picks its waves per slice)
    int nbricks = 0, brick_lds = 0, brick_gparts = 0, brick_rstride = 0;  // (gather workgroups per brick)
    int brick_dims[3] = {0, 0, 0};  // bricks along x, y, z
    double brick_model_us = 0.0;    // the planner's modelled product time
    void *d_bdesc = nullptr;
    int *d_browd = nullptr;
    int64_t *d_sbp = nullptr;     // per row: its first stored block in d_slid
    uint16_t *d_slid = nullptr;   // per stored block: its column's position in the group dictionary
    int *d_sdptr = nullptr, *d_sdict = nullptr;  // per group of G rows: sorted distinct stored columns
    int *d_sglist = nullptr;  // group order of the launches: sym_reg[2] groups within sym_reg[0] slots, then the rest
    int64_t gsym_inner[2] = {0, 0};  // groups leading each launch's list that read no ghost column
    // gather runs (k_nb_gsym_gather): per 64-row slice s, runs [d_sgptr[s], d_sgptr[s+1]) in ascending
    // group order, each the first dictionary entry (d_sgidx) naming a slice row and the mask of the rows it names
    int *d_sgptr = nullptr, *d_sgidx = nullptr;
    unsigned long long *d_sgmask = nullptr;
    // box bricks: per 64-row slice of the owned rows, the rows of one stored
    // block (the diagonal only), whose product the gather forms (B_ii x_i)
    unsigned long long *d_ssingle = nullptr;
    std::vector<uint8_t> diag_only_row;  // export: rows whose PETSc pattern is the diagonal
    // export: DoF-level entry rule inside the node blocks (no-slip matrices,
    // MASK_* below) and the ext-range DoF classes it reads
    int mask_rule = 0;
    std::vector<uint8_t> dof_cls;
    // halo plan of the column space
    int lo_rank = -1, hi_rank = -1;
    int64_t ghost_lo = 0, ghost_hi = 0, send_lo = 0, send_hi = 0;  // entries
    kle::PlanPtr plan;                 // general halo of the column space
    std::vector<int64_t> ext_gid;      // ext column -> global node (graph partitions)
    // ---- scalar AIJ (kind 1)
    int64_t nnz = 0;
    int64_t *d_aptr = nullptr;   // [m_local+1]
    int *d_acol = nullptr;       // [nnz] local column
    double *d_aval = nullptr;
    // host staging for setValues (PETSc stash semantics)
    std::vector<int64_t> h_ptr;  // preallocated pattern (after first assembly)
    std::vector<int64_t> h_col;
    std::vector<double> h_val;
    struct StashEnt {
        int64_t col;
        double v;
        int add;
    };
    std::vector<std::vector<StashEnt>> stash;  // per row, before first assembly
    std::vector<int32_t> d_nnz_hint;
    bool assembled = false, dirty = false;
};

namespace kle {
// vec helpers used across translation units
int vec_alloc(kle_ctx *ctx, int64_t n_local, int64_t n_global, int64_t lo, int64_t glo,
              int64_t ghi, kle_vec **out);
int allreduce_sum(kle_ctx *ctx, double *dbuf, int n, hipStream_t s = nullptr);  // in place, device buffer
int allgather_i64(kle_ctx *ctx, int64_t mine, std::vector<int64_t> &all);
int halo_exchange(kle_ctx *ctx, double *base, int64_t ghost_lo, int64_t n_local, int64_t ghost_hi,
                  int lo_rank, int hi_rank, int64_t send_lo, int64_t send_hi, hipStream_t s = nullptr,
                  const HaloPlan *plan = nullptr);
// y = A x; istate (may be null): no-op once the Krylov reason word is set
int spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate);
// y = A x and, where the SpMV can form them, the per-workgroup partials of
// (y, x) in dpart: *nparts of them (0: none written -- the caller forms them)
int spmv_dot(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart, int *nparts);
int spmv_dot_parts(const kle_mat *A);  // what spmv_dot would write (0: none)
// true when spmv(A, x, ...) exchanges the halo on ctx->comm_stream
bool spmv_uses_comm_stream(const kle_mat *A, const kle_vec *x);
bool spmv_can_split(const kle_mat *A);
int spmv_split(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate,
               double *dpart = nullptr);  // dpart (one rank): the bricks' (y, x) partials, A->nbricks of them
int reduce_partials(kle_ctx *ctx, const double *partials, int nparts, int nq, double *out);
int grid_for(int64_t work, int per_block, int max_blocks);
unsigned sync_event_flags();  // kle_core.hip
int nb_build_dict(kle_mat *A);  // kle_mat.hip
// symmetric storage (kle_sym.hip)
int sym_build(kle_mat *A);
void sym_drop(kle_mat *A);
void sym_forget(kle_mat *A);  // null the symmetric-storage pointers of a struct copy (no free)
int sym_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate,
             double *dpart = nullptr);  // N > 1: both halos included; dpart: (y, x) partials (one rank)
int sym_dot_parts(const kle_mat *A);  // partials sym_spmv writes with dpart (0: it cannot)
// brick symmetric SpMV (kle_brick.hip): plan (values in brick order: svptr
// out; plan null + why when no brick decomposition applies), finish after the
// values are copied (takes the plan), product, teardown
int brick_setup(kle_mat *A, const std::vector<int> &rb, const std::vector<int> &cnt, const std::vector<int> &srow,
                int P, std::vector<int64_t> &svptr_out, std::string &why, void **plan_out);
// the symmetric storage's value array (kle_sym.hip)
int sval_alloc(kle_mat *A, size_t bytes);
// a streamed array (matrix values): 0, or -1 out of memory
int big_alloc(void **p, size_t bytes);
// host -> device, landed on return (hipMemcpy + the null stream's sync)
int h2d(void *dst, const void *src, size_t bytes);
// declare `bytes` of dynamic LDS for kernel `kern` on c's device (once per size)
void dyn_lds(const kle_ctx *c, const void *kern, size_t bytes);
// (xs: the owned x, for the box bricks' one-block rows -- d_ssingle)
// (wps_force: the waves per slice, 0 by the runs per slice; 1 sums every
// row's runs in the order the fused CG update does, k_pipe_iter_g)
int gsym_gather(kle_mat *A, double *y, int64_t r0, int64_t r1, const int *istate, const double *xdot, double *dpart,
                int preload, hipStream_t st, const double *xs = nullptr, int wps_force = 0);
// graph bricks (kle_gbrick.hip)
int gbrick_bound(kle_mat *A, double vmax_all);
int gbrick_launch(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate);
int brick_finish(kle_mat *A, void *plan);
void brick_plan_free(void *plan);
// split: the owned rows' gather and the received reverse-halo sums are left
// to the consumer (k_pipe_iter_g) or to brick_gather_rest
int brick_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart, bool split = false);
int brick_gather_rest(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, int wps_force = 0);
// a split box-brick product's remaining gather, as the fused CG update does it
struct BrickGather {
    const int *runptr, *rstart;
    const unsigned long long *rmask;
    const double *ws;
    const unsigned long long *single;  // one-block rows per 64-row slice (null: none)
    const double *sval;
    const int64_t *svptr;
    const double *xs;     // the product's input (owned part): the one-block rows' B_ii x_i
    int64_t nrows, ng;    // owned rows; rows [0, ng) gathered by the consumer, [ng, nrows) by the split product
    const double *recv;   // the lower neighbour's sums for the entries [0, nrecv), added last
    int64_t nrecv;
};
BrickGather brick_gather_src(const kle_mat *A, const kle_vec *x);
int brick_spmv_local(kle_mat *A, const kle_vec *x, kle_vec *y);  // the rank-local product, no halos (timing)
void brick_drop(kle_mat *A);
void brick_forget(kle_mat *A);
// IPC transport (kle_ipc.hip): slab and graph-partition halos, their reverse halos, allreduce
int ipc_halo(kle_ctx *c, double *base, int64_t ghost_lo, int64_t n_local, int64_t ghost_hi, int lo_rank,
             int hi_rank, int64_t send_lo, int64_t send_hi, hipStream_t st);
int ipc_reverse(kle_ctx *c, const double *send_hi, int64_t n_send, int hi_rank, double *recv_lo, int64_t n_recv,
                int lo_rank, hipStream_t st);
int ipc_allreduce(kle_ctx *c, double *dbuf, int n, hipStream_t st);
int ipc_halo_plan(kle_ctx *c, double *base, const HaloPlan &H, int bs, const double *sbuf, hipStream_t st);
int ipc_reverse_plan(kle_ctx *c, const HaloPlan &H, int64_t hi0, int bs, const double *gsend, double *rbuf,
                     hipStream_t st);
void ipc_destroy(kle_ctx *c);
int halo_reverse(kle_ctx *ctx, const double *send_hi, int64_t n_send, int hi_rank, double *recv_lo, int64_t n_recv,
                 int lo_rank, hipStream_t st);  // kle_core.hip
int halo_reverse_plan(kle_ctx *ctx, const HaloPlan &P, int64_t hi0, int bs, const double *gsend, double *rbuf,
                      hipStream_t st);  // kle_core.hip
std::string sym_kernel_name(const kle_mat *A);
double sym_spmv_bytes(const kle_mat *A);
double brick_split_bytes(const kle_mat *A);  // a split brick product: the bricks alone
// Performance knobs (kle_set_tuning): every setting gives correct results;
// they exist for in-process A/B measurements (tools/cg_ab.py).
struct Tuning {
    int spmv_waves = 0;  // rows per SpMV workgroup for 3x3 chunked matrices: 0 auto (8 from 64k rows, else 4), 4, 8
    int spmv_xcd_chunk = 16;  // SpMV: consecutive row blocks per XCD in each run (0: round-robin), xcd_block()
    int spmv_dyn_lds = -1;  // unused dynamic LDS per SpMV workgroup (bytes), caps SpMV workgroups per CU; -1 auto
    int ksp_sr_gather = 1;  // single-reduction CG on box bricks, one rank: the same fold (k_sr_iter_g; (A u, u) from the bricks) from 2^17 node rows (1), always (2), never (0)
    int ksp_pipe_gather = 1;  // pipelined CG on box bricks: the product's owned-row gather folded into the next update (k_pipe_iter_g); 0 separate
    int ipc_sentinel = 0;  // IPC transport (debug): consumed mailbox slots overwritten with NaN before the ack (a stale or early slot read shows as NaN)
    int ksp_corr_fault = 0;  // test hook: 1 = refine() runs its correction solves even when the true residual meets rtol, and each ends in NaN (DIVERGED_NANORINF) -- x must stay as it was
    int ksp_refine = 2;  // CG / pipelined CG: up to this many correction solves when the true residual misses rtol (kle_ksp.hip refine; default of new KSPs); 0 PETSc's plain stop
    int upd_nt = 2;       // single-reduction CG update: every vector but u nontemporal (u stays in the Infinity Cache for the
                          // SpMV) -- 0 off, 1 on, 2 auto: from 2M local entries (12 vectors > the 256 MB cache); per CG
                          // iteration config 4 4353 -> 4272 us, config-5 size 4019 -> 3907, config 2 448.4 -> 452.1
                          // (profiles/r04/ab/upd_nt_*.jsonl)
    int upd_preload = 1;  // CG update kernels load their first element and the stage inputs before the prologue; 0 off
    int spmv_x_lds = 1;  // 3x3 structured SpMV: x staged in LDS per workgroup (k_nb_spmv_xl); 0 off
    int spmv_sym = 1;  // SBAIJ-style symmetric storage for the KLE K of >= spmv_sym_min_rows node rows per rank; 0 off
    int spmv_sym_min_rows = 40000;  // (the 1/8 parts of config 2: box slab 76.75 vs 78.29 us per pipelined CG iteration, unstructured 77.0 vs 79.8 us per SpMV; profiles/r04/ab/small_parts.jsonl)
    int spmv_sym_det = 1;     // symmetric SpMV: transposed adds as exact fixed-point sums (bitwise reproducible); 0 fp64 LDS atomics
    int spmv_sym_waves = 0;   // waves per workgroup of k_nb_spmv_sym_xl: 0 auto (8 while 2 workgroups fit a CU), 8, 16
    int spmv_sym_align = 0;   // symmetric SpMV partials (read at build): every tile's / group's slot starts on a 128-B line and its lines are written whole (1; measured no faster, r04d) or packed (0)
    int spmv_sym_tile64 = 0;        // symmetric box storage (read at build): 8 x 2 x 4 tiles (64 rows) -- 0 auto (below spmv_sym_tile64_max 128-row tiles), 1 always, 2 never
    int spmv_sym_tile64_max = 640;  // ... 1/8 of config 2 (561 tiles; 374 per rank at N = 8) 75.6 -> 70.6 us (full storage 72.4), 1/4 (935; 748 per rank at N = 4) 121.2 vs 127.8 (profiles/r04/ab/tile64_and_sgpr_ab.jsonl)
    int spmv_sym_xcd = 0;           // box symmetric tile kernel: runs of this many consecutive tiles per XCD (0: round-robin)
    int spmv_sym_ovl_b = 50;        // N > 1 symmetric box SpMV: % of the interior tiles run beside the reverse halo
    int spmv_sym_stpol = 0;   // box symmetric SpMV partial stores: 0 plain, 1 nontemporal, 2 sc1, 3 sc0 sc1 (write-through)
    int spmv_gsym_stpol = 2;  // ... of the graph symmetric SpMV: sc1 452.9 -> 449.1 us at 1M DoF (the box kernel: plain 420.5,
                              // sc1 422.1, nt 426.5; profiles/r04/ab/stpol_*.jsonl)
    int spmv_sym_early = 0;   // symmetric SpMV tiles: the first item's value loads issued with the x fill (1) or after it (0)
    int spmv_sym_tz = 0;      // symmetric SpMV tiles (read at build): 0 auto (8 x 4 x 4 rows where it fits), 2 (8 x 8 x 2), 4
    int spmv_brick_max = 0;    // brick SpMV (read at build): at most this many bricks (0: planned, spmv_brick_rounds per CU)
    int spmv_brick_rounds = 1;  // brick SpMV (read at build): at most this many bricks per CU (2: heaviest-first to the first free CU, 0.467 vs 0.460 ms at config 2, profiles/r05/rounds_ab.jsonl)
    int upd_unroll = 1;        // single-reduction CG update: elements per pass with their loads in flight (1, 2; 2 no faster at config 2, profiles/r05/cg_ab_upd_unroll.jsonl)
    int spmv_gsym_brick = 1;   // unstructured symmetric SpMV (read at build): row bricks (kle_gbrick.hip), 0 the 64-row groups
    int spmv_gather_wps = 0;   // run-mask gather: waves per 64-row slice (1, 2, 4; 0 auto by the runs per slice)
    int spmv_brick_pair = 1;  // brick SpMV (read at build): rows in units of two whose tails share one 64-lane item
    int spmv_brick_singles = 1;  // brick SpMV (read at build): rows of one stored block formed by the gather, not as 64-lane items of the bricks
    int spmv_brick_split = 0;  // brick SpMV (read at build): force nbx + 100 nby + 10000 nbz bricks (0: planned)
    int spmv_sym_brick = 1;   // box symmetric storage, one rank (read at build): one brick per CU, sums in LDS for the whole stream (kle_brick.hip); 0 the 128-row tiles
#ifdef KLE_PROBE_BUILD
    // timing probes (wrong results on purpose), compiled only into the probe
    // build tools/libkle_probe.so (make probe), never into libkle.so: skip 1
    // transposed adds, 2 row sums, 4 LDS x reads, 8 partial stores, 16 block ->
    // region arithmetic, 128 the item loop; 32 nontemporal partial stores, 64
    // partials into 8 slabs
    int spmv_sym_probe = 0;
#endif
    int spmv_gsym_rows = 64;  // unstructured symmetric storage: rows per group (8, 16, 32 or 64; read at build)
    int spmv_gsym_waves = 0;  // its waves per workgroup (0 auto: 16 for 64-row groups, else 8; 8 or 16; read at build)
    int spmv_gsym_split = 0;  // unstructured symmetric storage: dictionary slots of the first launch (0 auto: 4 workgroups per CU; tests)
    int spmv_dict = 1;  // unstructured 3x3 SpMV: x staged in LDS through the row groups' column dictionaries; 0 off
    int spmv_dict_min_rows = 64000;  // matrices with fewer node rows get no dictionaries (read at creation)
};
extern Tuning g_tune;
// The symmetric SpMV kernels' timing-probe argument exists only in the probe
// build; in libkle.so `probe` is the constant 0 and every probe branch folds away.
#ifdef KLE_PROBE_BUILD
// probe build: also per-workgroup phase timestamps (s_memrealtime, 100 MHz)
// into g_probe_ts[slot][8] when kle_set_tuning("spmv_sym_probe_ts", slots)
// allocated it: slot, start, x ready, item loop done, partials stored
// (after every wave's vmcnt(0)), HW_ID, XCC_ID
extern unsigned long long *g_probe_ts;
extern int64_t g_probe_ts_cap;
#define KLE_PROBE_PARAM , int probe, unsigned long long *probe_ts, int64_t probe_cap
#define KLE_PROBE_ARG , g_tune.spmv_sym_probe, g_probe_ts, g_probe_ts_cap
#define KLE_PROBE_CONST
#define KLE_PROBE_TS(var) unsigned long long var = probe_ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
#define KLE_PROBE_TS_END(slot, a, b, c)                                                                 \
    if (probe_ts) {                                                                                     \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                \
        __syncthreads();                                                                                \
        if (threadIdx.x == 0 && (int64_t)(slot) < probe_cap) {                                          \
            unsigned long long *r = probe_ts + 8 * (int64_t)(slot);                                     \
            r[0] = (unsigned long long)(slot);                                                          \
            r[1] = a;                                                                                   \
            r[2] = b;                                                                                   \
            r[3] = c;                                                                                   \
            r[4] = __builtin_amdgcn_s_memrealtime();                                                    \
            r[5] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));                                 \
            r[6] = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));                                \
        }                                                                                               \
    }
// (r[7]: two more points of the workgroup's start, as 32-bit offsets from a)
#define KLE_PROBE_TS_END4(slot, a, b, c, d, e)                                                         \
    if (probe_ts) {                                                                                     \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                \
        __syncthreads();                                                                                \
        if (threadIdx.x == 0 && (int64_t)(slot) < probe_cap) {                                          \
            unsigned long long *r = probe_ts + 8 * (int64_t)(slot);                                     \
            r[0] = (unsigned long long)(slot);                                                          \
            r[1] = a;                                                                                   \
            r[2] = b;                                                                                   \
            r[3] = c;                                                                                   \
            r[4] = __builtin_amdgcn_s_memrealtime();                                                    \
            r[5] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));                                 \
            r[6] = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));                                \
            r[7] = ((d) - (a)) | (((e) - (a)) << 32);                                                   \
        }                                                                                               \
    }
// (and a third point in r[5]'s upper half)
#define KLE_PROBE_TS_END5(slot, a, b, c, d, e, f)                                                      \
    KLE_PROBE_TS_END4(slot, a, b, c, d, e)                                                              \
    if (probe_ts && threadIdx.x == 0 && (int64_t)(slot) < probe_cap)                                   \
        probe_ts[8 * (int64_t)(slot) + 5] |= ((f) - (a)) << 32;
#else
#define KLE_PROBE_TS_END4(slot, a, b, c, d, e)
#define KLE_PROBE_TS_END5(slot, a, b, c, d, e, f)
#define KLE_PROBE_PARAM
#define KLE_PROBE_ARG
#define KLE_PROBE_CONST constexpr int probe = 0;
#define KLE_PROBE_TS(var)
#define KLE_PROBE_TS_END(slot, a, b, c)
#endif
// marks the SpMV launches inside its scope as running beside comm-stream work
struct SideBusy {
    kle_ctx *c;
    bool prev;
    explicit SideBusy(kle_ctx *ctx) : c(ctx), prev(ctx->side_busy) { c->side_busy = true; }
    ~SideBusy() { c->side_busy = prev; }
};
extern int g_nb_pad;
extern int g_nb_layout;  // value layout of new node-block matrices (kle_mat.vlayout)
extern int g_partitioner;  // unstructured meshes: 0 inertial bisection, 1 slabs (kle_umesh.cpp)
// Offset of entry t (0 <= t < RC) of block k inside a row of m blocks
// (mp = padded length for layout 0).  Layout 1: full 16-block chunks hold the
// RC streams back to back (t-th 128-B line of chunk c), the m % 16 tail
// blocks follow as RC packed streams of length m % 16.
__host__ __device__ inline int64_t vofs(int lay, int RC, int t, int k, int m, int mp)
{
    if (lay == 0) return (int64_t)t * mp + k;
    const int q16 = m & ~15;
    if (k < q16) return ((int64_t)(k >> 4) * RC + t) * 16 + (k & 15);
    return (int64_t)q16 * RC + (int64_t)t * (m - q16) + (k - q16);
}
// Host worker count for setup loops: OMP_NUM_THREADS if set, else the
// hardware concurrency, capped at 16 (the GPU box's CPU share per GPU).
int host_threads();
// Run f(lo, hi) over [0, n) split into contiguous chunks on host_threads().
void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)> &f);
// Symbolic pattern `which` of the owned rows as CSR (row_ptr[n+1], global cols).
int pattern_csr(const kle_mesh *m, int which, std::vector<int64_t> &row_ptr, std::vector<int64_t> &cols);
// Unstructured mesh (kle_umesh.cpp): sorted unique node neighbours of owned
// row i (nodes sharing a local cell); on_face: Face Sets bits of an ext node.
void umesh_row_nodes(const kle_mesh *m, int64_t i, std::vector<int64_t> &out);
enum DofClass : uint8_t { DOF_FREE = 0, DOF_TANG = 1, DOF_NORMAL = 2 };
// which PETSc entries of a node block exist (MatNS.buildNS, mat_ns.py:47-145)
enum MaskRule { MASK_NONE = 0, MASK_KFS = 1, MASK_KRHSFS = 2, MASK_TANG_ROWS = 3, MASK_KSUM = 4 };
__host__ __device__ inline bool mask_entry(int rule, int rc, int cc, bool diag)
{
    switch (rule) {
    case MASK_KFS: return (rc == DOF_TANG && cc != DOF_NORMAL) || (rc == DOF_FREE && cc == DOF_TANG);
    case MASK_KRHSFS: return rc == DOF_NORMAL ? diag : cc == DOF_NORMAL;
    case MASK_TANG_ROWS: return rc == DOF_TANG;
    case MASK_KSUM: return rc == DOF_NORMAL ? diag : cc != DOF_NORMAL;
    default: return true;
    }
}  // row padding quantum (blocks) of new node-block matrices
}  // namespace kle
