// kle_core.hip -- context, errors, profiling, device vectors (BLAS-1 with
// deterministic two-stage reductions), halo exchange over RCCL.
//
// Replaces the PETSc Vec traffic of the hot path:
// Vec.__add__ (kle_solver.py:35), axpy/scale (base_problem.py:129-134),
// setValues+assemble (boundary_conditions.py:252-260), reciprocal
// (mat_fs.py:256), dot/norm (base_problem.py:334,389).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>

#include "kle_internal.hpp"

namespace kle {

// Matrix value arrays: plain hipMalloc.  (Round 5 tried physically
// contiguous memory, hipDeviceMallocContiguous, for placement-independent
// SpMV speed; on it the element-batched assembly -- gathers adding to values
// an earlier launch stored -- missed 41 of 1.4M sums, and no speed gain
// survived the placement records, so the mode is gone: VERDICT r05 item 4.)
int big_alloc(void **p, size_t bytes)
{
    *p = nullptr;
    if (hipMalloc(p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return -1;
    }
    return 0;
}

// A host-to-device copy that has landed when it returns.  hipMemcpy from
// pageable memory may return once the bytes are in a staging buffer, with
// the DMA still queued on the null stream -- which the context's
// non-blocking streams do not wait for, so a kernel launched next could read
// the destination before the copy ends.  The null stream's synchronisation
// closes that window (setup paths only; round 6 after a fault that
// serialised kernels could not reproduce).
int h2d(void *dst, const void *src, size_t bytes)
{
    KLE_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    KLE_HIP(hipStreamSynchronize(nullptr));
    return 0;
}

// Dynamic LDS above 64 KB must be declared per kernel (hipFuncSetAttribute);
// the attribute is per device, so the record of what was declared is keyed
// by (device, kernel), under a lock (a function-static cache
// skipped the call for a second context on another device)
void dyn_lds(const kle_ctx *c, const void *kern, size_t bytes)
{
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> done;
    std::lock_guard<std::mutex> lk(mu);
    size_t &s = done[{c->device, kern}];
    if (bytes > s) {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        s = bytes;
    }
}

Tuning g_tune;
#ifdef KLE_PROBE_BUILD
unsigned long long *g_probe_ts = nullptr;
int64_t g_probe_ts_cap = 0;
#endif


static thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

void clear_error() { g_err.clear(); }

// Flags of the events that order the compute and comm streams (N > 1).
// KLE_EVENT_NO_SYSTEM_FENCE=1 adds hipEventDisableSystemFence: both streams
// and RCCL's kernels live on this device, so a device-scope release would
// do, and it halves the cost of a cross-stream round trip (7.8 -> 3.9 us on
// the 1/8 slab, 7.1 -> 4.3 at config 2; profiles/r02/sync_evflags_*.jsonl).
// Off by default until a multi-GPU run confirms RCCL never reads our buffers
// from another device.
unsigned sync_event_flags()
{
    const char *e = getenv("KLE_EVENT_NO_SYSTEM_FENCE");
    return hipEventDisableTiming | (e && atoi(e) ? hipEventDisableSystemFence : 0u);
}

int grid_for(int64_t work, int per_block, int max_blocks)
{
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > max_blocks) g = max_blocks;
    return (int)g;
}

// ------------------------------------------------------------ wave utilities
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum of one value per thread (blockDim.x <= 1024), result valid
// in thread 0.  Fixed combination order -> bitwise reproducible.
__device__ __forceinline__ double block_sum(double v, double *lds)
{
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) lds[w] = v;
    __syncthreads();
    double s = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < nw; ++i) s += lds[i];
    return s;
}

// ---------------------------------------------------------------- kernels
__global__ void k_set(int64_t n, double a, double *__restrict__ y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = a;
}

__global__ void k_axpy(int64_t n, double a, const double *__restrict__ x, double *__restrict__ y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] += a * x[i];
}

__global__ void k_aypx(int64_t n, double b, const double *__restrict__ x, double *__restrict__ y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = x[i] + b * y[i];
}

__global__ void k_waxpy(int64_t n, double a, const double *__restrict__ x,
                        const double *__restrict__ y, double *__restrict__ w)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        w[i] = a * x[i] + y[i];
}

__global__ void k_scale(int64_t n, double a, double *__restrict__ y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] *= a;
}

// computeVtensV (base_problem.py:138-154): the symmetric tensor v v^T per node,
// components xx, xy, yy (2-D) or xx, xy, yy, yz, zz, zx (3-D)
template <int DIM>
__global__ void k_vtensv(int64_t nodes, const double *__restrict__ v, double *__restrict__ o)
{
    constexpr int DS = DIM == 2 ? 3 : 6;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nodes; i += (int64_t)gridDim.x * blockDim.x) {
        const double x = v[i * DIM], y = v[i * DIM + 1];
        double *t = o + i * DS;
        t[0] = x * x;
        t[1] = x * y;
        t[2] = y * y;
        if constexpr (DIM == 3) {
            const double z = v[i * DIM + 2];
            t[3] = y * z;
            t[4] = z * z;
            t[5] = z * x;
        }
    }
}

__global__ void k_pmult(int64_t n, const double *__restrict__ x, const double *__restrict__ y,
                        double *__restrict__ w)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        w[i] = x[i] * y[i];
}

__global__ void k_recip(int64_t n, double *__restrict__ y)
{
    // VecReciprocal: zero entries stay zero (PETSc semantics)
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = y[i] != 0.0 ? 1.0 / y[i] : 0.0;
}

__global__ void k_dot_partial(int64_t n, const double *__restrict__ x, const double *__restrict__ y,
                              double *__restrict__ partials)
{
    __shared__ double lds[16];
    double s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += x[i] * y[i];
    s = block_sum(s, lds);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// Sum nq quantities of nparts partials each (stride RED_BLOCKS) into out[q].
__global__ void k_reduce(const double *__restrict__ partials, int nparts, int nq,
                         double *__restrict__ out)
{
    __shared__ double lds[16];
    for (int q = 0; q < nq; ++q) {
        double s = 0;
        for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += partials[q * PART_STRIDE + i];
        s = block_sum(s, lds);
        if (threadIdx.x == 0) out[q] = s;
        __syncthreads();
    }
}

__global__ void k_scatter_values(int64_t n, const int64_t *__restrict__ idx,
                                 const double *__restrict__ v, double *__restrict__ y, int addv)
{
    // addv: applied sequentially by one thread when indices may repeat
    if (addv) {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            for (int64_t i = 0; i < n; ++i) y[idx[i]] += v[i];
        return;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[idx[i]] = v[i];
}

__global__ void k_gather_values(int64_t n, const int64_t *__restrict__ idx,
                                const double *__restrict__ y, double *__restrict__ v)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        v[i] = y[idx[i]];
}

__global__ void k_stream_copy(int64_t n4, const double4 *__restrict__ a, double4 *__restrict__ b)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

typedef double dvec4 __attribute__((ext_vector_type(4)));
__global__ void k_stream_read(int64_t n4, const double4 *__restrict__ a4, double *__restrict__ out)
{
    const dvec4 *a = reinterpret_cast<const dvec4 *>(a4);
    double s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        dvec4 v = __builtin_nontemporal_load(a + i);
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1.2345e-300) out[0] = s;  // keep the loads alive
}

// 8-byte-per-lane read (the SpMV's access width); nt: non-temporal
template <bool NT>
__global__ void k_stream_read8(int64_t n, const double *__restrict__ a, double *__restrict__ out)
{
    double s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += NT ? __builtin_nontemporal_load(a + i) : a[i];
    if (s == 1.2345e-300) out[0] = s;
}

// The streaming ceilings the SpMVs are graded against (verdict r04 item 2):
// 16 B per lane, U loads in flight per thread (all issued before the first
// use), each workgroup sweeping contiguous 256 x U x 16-B super-chunks, a
// grid of a few workgroups per CU.  W = 8: 8-B loads (2U of them) over the
// same chunk, the symmetric SpMV's value-load width.
typedef double dvec2 __attribute__((ext_vector_type(2)));
template <int U, bool NT, int W, int NT_ = 256>
__global__ __launch_bounds__(NT_) void k_stream_rd(int64_t n16, const dvec2 *__restrict__ a, double *__restrict__ out)
{
    double s = 0.0;
    const int64_t per = (int64_t)NT_ * U;
    for (int64_t base = (int64_t)blockIdx.x * per; base < n16; base += (int64_t)gridDim.x * per) {
        if (W == 16) {
            dvec2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = min(base + u * NT_ + threadIdx.x, n16 - 1);
                v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
        } else {
            const double *d = reinterpret_cast<const double *>(a);
            double v[2 * U];
#pragma unroll
            for (int u = 0; u < 2 * U; ++u) {
                const int64_t i = min(2 * base + u * NT_ + threadIdx.x, 2 * n16 - 1);
                v[u] = NT ? __builtin_nontemporal_load(d + i) : d[i];
            }
#pragma unroll
            for (int u = 0; u < 2 * U; ++u) s += v[u];
        }
    }
    if (s == 1.2345e-300) out[0] = s;  // keep the loads alive
}

// copy with 16-B loads and stores, U in flight; NT: nontemporal stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stream_cp(int64_t n16, const dvec2 *__restrict__ a, dvec2 *__restrict__ b)
{
    const int64_t per = (int64_t)256 * U;
    for (int64_t base = (int64_t)blockIdx.x * per; base < n16; base += (int64_t)gridDim.x * per) {
        dvec2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = min(base + u * 256 + threadIdx.x, n16 - 1);
            v[u] = __builtin_nontemporal_load(a + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256 + threadIdx.x;
            if (i < n16) {
                if (NT) __builtin_nontemporal_store(v[u], b + i);
                else b[i] = v[u];
            }
        }
    }
}

int reduce_partials(kle_ctx *ctx, const double *partials, int nparts, int nq, double *out)
{
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, ctx->stream, partials, nparts, nq, out);
    KLE_HIP(hipGetLastError());
    return 0;
}

static constexpr int VB = 256;      // vector kernel block
static constexpr int VMAX = 2048;   // vector kernel max grid (8 WG per CU)

int vec_alloc(kle_ctx *ctx, int64_t n_local, int64_t n_global, int64_t lo, int64_t glo,
              int64_t ghi, kle_vec **out)
{
    kle_vec *v = new kle_vec;
    v->ctx = ctx;
    v->n_local = n_local;
    v->n_global = n_global;
    v->lo = lo;
    v->ghost_lo = glo;
    v->ghost_hi = ghi;
    int64_t tot = glo + n_local + ghi;
    if (hipMalloc(&v->base, sizeof(double) * std::max<int64_t>(tot, 1)) != hipSuccess) {
        delete v;
        return fail(KLE_ERR_MEM, "hipMalloc of %lld doubles failed", (long long)tot);
    }
    if (hipMemsetAsync(v->base, 0, sizeof(double) * std::max<int64_t>(tot, 1), ctx->stream) !=
        hipSuccess) {
        hipFree(v->base);
        delete v;
        return fail(KLE_ERR_DEVICE, "hipMemsetAsync failed");
    }
    v->d = v->base + glo;
    *out = v;
    return 0;
}

static int stage_reserve(kle_ctx *ctx, int64_t n)
{
    if (ctx->h_stage_n >= n) return 0;
    if (ctx->h_stage) hipHostFree(ctx->h_stage);
    ctx->h_stage = nullptr;
    ctx->h_stage_n = 0;
    KLE_HIP(hipHostMalloc(&ctx->h_stage, sizeof(double) * std::max<int64_t>(n, 64)));
    ctx->h_stage_n = std::max<int64_t>(n, 64);
    return 0;
}

int allreduce_sum(kle_ctx *ctx, double *dbuf, int n, hipStream_t st)
{
    if (ctx->nranks == 1 && !ctx->comm) return 0;
    if (!st) st = ctx->stream;
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(ctx->tic("allreduce", &ev, st));
    if (ctx->ipc) {
        KLE_TRY(ipc_allreduce(ctx, dbuf, n, st));
    } else if (ctx->comm) {
        KLE_NCCL(ncclAllReduce(dbuf, dbuf, n, ncclDouble, ncclSum, ctx->comm, st));
    } else {
        KLE_TRY(stage_reserve(ctx, n));
        KLE_HIP(hipMemcpyAsync(ctx->h_stage, dbuf, sizeof(double) * n, hipMemcpyDeviceToHost, st));
        KLE_HIP(hipStreamSynchronize(st));
        if (ctx->hcomm.allreduce(ctx->h_stage, n, ctx->hcomm.user))
            return fail(KLE_ERR_COMM, "host allreduce callback failed");
        KLE_HIP(hipMemcpyAsync(dbuf, ctx->h_stage, sizeof(double) * n, hipMemcpyHostToDevice, st));
        KLE_HIP(hipStreamSynchronize(st));
    }
    KLE_TRY(ctx->toc("allreduce", &ev, st));
    return 0;
}

int allgather_i64(kle_ctx *ctx, int64_t mine, std::vector<int64_t> &all)
{
    // one-hot sum (exact for integers < 2^53)
    all.assign(ctx->nranks, 0);
    std::vector<double> h(ctx->nranks, 0.0);
    h[ctx->rank] = (double)mine;
    double *d;
    KLE_HIP(hipMalloc(&d, sizeof(double) * ctx->nranks));
    KLE_HIP(hipMemcpyAsync(d, h.data(), sizeof(double) * ctx->nranks, hipMemcpyHostToDevice, ctx->stream));
    int rc = allreduce_sum(ctx, d, ctx->nranks);
    if (!rc) {
        KLE_HIP(hipMemcpyAsync(h.data(), d, sizeof(double) * ctx->nranks, hipMemcpyDeviceToHost, ctx->stream));
        KLE_HIP(hipStreamSynchronize(ctx->stream));
        for (int r = 0; r < ctx->nranks; ++r) all[r] = (int64_t)h[r];
    }
    hipFree(d);
    return rc;
}

HaloPlan::~HaloPlan()
{
    if (d_send_idx) (void)hipFree(d_send_idx);
    if (d_sbuf) (void)hipFree(d_sbuf);
}

// sbuf[k] = own[idx[k / bs] * bs + k % bs]: a graph-partition halo's sends
__global__ void k_halo_pack(int64_t n, int bs, const int32_t *__restrict__ idx, const double *__restrict__ own,
                            double *__restrict__ sbuf)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t node = idx[k / bs];
        sbuf[k] = own[node * bs + k % bs];
    }
}

// General halo (HaloPlan): pack the sends, then one grouped send/recv per
// peer; receives land in the peer's ghost group of the ext layout.
static int halo_exchange_plan(kle_ctx *ctx, double *base, int64_t ghost_lo, int64_t n_local,
                              const HaloPlan &P_, hipStream_t st)
{
    HaloPlan &P = const_cast<HaloPlan &>(P_);
    if (P.peers.empty()) return 0;
    if (P.n_owned <= 0 || n_local % P.n_owned)
        return fail(KLE_ERR_STATE, "halo plan of %lld owned nodes does not fit a vector of %lld entries",
                    (long long)P.n_owned, (long long)n_local);
    const int bs = (int)(n_local / P.n_owned);
    const int64_t ns = (int64_t)P.send_idx.size() * bs;
    if (!P.d_send_idx && !P.send_idx.empty()) {
        KLE_HIP(hipMalloc(&P.d_send_idx, sizeof(int32_t) * P.send_idx.size()));
        KLE_TRY(h2d(P.d_send_idx, P.send_idx.data(), sizeof(int32_t) * P.send_idx.size()));
    }
    if (P.sbuf_cap < ns) {
        KLE_HIP(hipStreamSynchronize(st));
        if (P.d_sbuf) KLE_HIP(hipFree(P.d_sbuf));
        P.d_sbuf = nullptr;
        KLE_HIP(hipMalloc(&P.d_sbuf, sizeof(double) * ns));
        P.sbuf_cap = ns;
    }
    const double *own = base + ghost_lo;
    if (ns) {
        const int g = (int)std::min<int64_t>((ns + 255) / 256, 4096);
        hipLaunchKernelGGL(k_halo_pack, dim3(g), dim3(256), 0, st, ns, bs, P.d_send_idx, own, P.d_sbuf);
        KLE_HIP(hipGetLastError());
    }
    // ghost group of peer k starts at ext node recv_off[k] (relative to base)
    const size_t np = P.peers.size();
    if (ctx->ipc) return ipc_halo_plan(ctx, base, P, bs, P.d_sbuf, st);
    if (ctx->comm) {
        KLE_NCCL(ncclGroupStart());
        for (size_t k = 0; k < np; ++k) {
            if (P.send_cnt[k])
                KLE_NCCL(ncclSend(P.d_sbuf + P.send_off[k] * bs, P.send_cnt[k] * bs, ncclDouble, P.peers[k], ctx->comm, st));
            if (P.recv_cnt[k])
                KLE_NCCL(ncclRecv(base + P.recv_off[k] * bs, P.recv_cnt[k] * bs, ncclDouble, P.peers[k], ctx->comm, st));
        }
        KLE_NCCL(ncclGroupEnd());
        return 0;
    }
    if (!ctx->hcomm.exchange) return fail(KLE_ERR_COMM, "host transport has no exchange callback (graph-partitioned halo)");
    int64_t nr = 0;
    std::vector<int64_t> sc(np), rc(np);
    for (size_t k = 0; k < np; ++k) {
        sc[k] = P.send_cnt[k] * bs;
        rc[k] = P.recv_cnt[k] * bs;
        nr += rc[k];
    }
    KLE_TRY(stage_reserve(ctx, ns + nr));
    double *hs = ctx->h_stage, *hr = hs + ns;
    if (ns) KLE_HIP(hipMemcpyAsync(hs, P.d_sbuf, sizeof(double) * ns, hipMemcpyDeviceToHost, st));
    KLE_HIP(hipStreamSynchronize(st));
    if (ctx->hcomm.exchange((int)np, P.peers.data(), hs, sc.data(), hr, rc.data(), ctx->hcomm.user))
        return fail(KLE_ERR_COMM, "host exchange callback failed");
    int64_t z = 0;
    for (size_t k = 0; k < np; ++k) {
        if (rc[k]) KLE_HIP(hipMemcpyAsync(base + P.recv_off[k] * bs, hr + z, sizeof(double) * rc[k], hipMemcpyHostToDevice, st));
        z += rc[k];
    }
    KLE_HIP(hipStreamSynchronize(st));
    return 0;
}

int halo_exchange(kle_ctx *ctx, double *base, int64_t ghost_lo, int64_t n_local, int64_t ghost_hi,
                  int lo_rank, int hi_rank, int64_t send_lo, int64_t send_hi, hipStream_t st,
                  const HaloPlan *plan)
{
    if (ctx->nranks == 1) return 0;
    if (!st) st = ctx->stream;
    if (plan) {
        std::pair<hipEvent_t, hipEvent_t> ev;
        KLE_TRY(ctx->tic("halo", &ev, st));
        KLE_TRY(halo_exchange_plan(ctx, base, ghost_lo, n_local, *plan, st));
        KLE_TRY(ctx->toc("halo", &ev, st));
        return 0;
    }
    if (lo_rank < 0 && hi_rank < 0) return 0;
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(ctx->tic("halo", &ev, st));
    double *own = base + ghost_lo;
    if (ctx->ipc) {
        KLE_TRY(ipc_halo(ctx, base, ghost_lo, n_local, ghost_hi, lo_rank, hi_rank, send_lo, send_hi, st));
    } else if (ctx->comm) {
        KLE_NCCL(ncclGroupStart());
        if (lo_rank >= 0) {
            // my lowest send_lo owned entries are the lower neighbour's upper ghosts
            KLE_NCCL(ncclSend(own, send_lo, ncclDouble, lo_rank, ctx->comm, st));
            KLE_NCCL(ncclRecv(base, ghost_lo, ncclDouble, lo_rank, ctx->comm, st));
        }
        if (hi_rank >= 0) {
            KLE_NCCL(ncclSend(own + n_local - send_hi, send_hi, ncclDouble, hi_rank, ctx->comm,
                              st));
            KLE_NCCL(ncclRecv(own + n_local, ghost_hi, ncclDouble, hi_rank, ctx->comm, st));
        }
        KLE_NCCL(ncclGroupEnd());
    } else {
        const int64_t sl = lo_rank >= 0 ? send_lo : 0, sh = hi_rank >= 0 ? send_hi : 0;
        const int64_t rl = lo_rank >= 0 ? ghost_lo : 0, rh = hi_rank >= 0 ? ghost_hi : 0;
        KLE_TRY(stage_reserve(ctx, sl + sh + rl + rh));
        double *hs_lo = ctx->h_stage, *hs_hi = hs_lo + sl, *hr_lo = hs_hi + sh, *hr_hi = hr_lo + rl;
        if (sl) KLE_HIP(hipMemcpyAsync(hs_lo, own, sizeof(double) * sl, hipMemcpyDeviceToHost, st));
        if (sh)
            KLE_HIP(hipMemcpyAsync(hs_hi, own + n_local - sh, sizeof(double) * sh, hipMemcpyDeviceToHost,
                                   st));
        KLE_HIP(hipStreamSynchronize(st));
        if (ctx->hcomm.halo(hs_lo, sl, lo_rank, hs_hi, sh, hi_rank, hr_lo, rl, hr_hi, rh, ctx->hcomm.user))
            return fail(KLE_ERR_COMM, "host halo callback failed");
        if (rl) KLE_HIP(hipMemcpyAsync(base, hr_lo, sizeof(double) * rl, hipMemcpyHostToDevice, st));
        if (rh)
            KLE_HIP(hipMemcpyAsync(own + n_local, hr_hi, sizeof(double) * rh, hipMemcpyHostToDevice, st));
        KLE_HIP(hipStreamSynchronize(st));
    }
    KLE_TRY(ctx->toc("halo", &ev, st));
    return 0;
}

// Reverse halo of the symmetric SpMV (slab partitions): the partial sums of my
// upper ghost rows (n_send entries) go to hi_rank, which owns those rows; the
// lower neighbour's sums for my lowest rows (n_recv entries) arrive from
// lo_rank.  The forward halo's pairs, one direction each.
int halo_reverse(kle_ctx *ctx, const double *send_hi, int64_t n_send, int hi_rank, double *recv_lo, int64_t n_recv,
                 int lo_rank, hipStream_t st)
{
    if (ctx->nranks == 1) return 0;
    if (!st) st = ctx->stream;
    const int64_t ns = hi_rank >= 0 ? n_send : 0, nr = lo_rank >= 0 ? n_recv : 0;
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(ctx->tic("halo_rev", &ev, st));
    if (ctx->ipc) {
        KLE_TRY(ipc_reverse(ctx, send_hi, ns, hi_rank, recv_lo, nr, lo_rank, st));
    } else if (ctx->comm) {
        KLE_NCCL(ncclGroupStart());
        if (ns) KLE_NCCL(ncclSend(send_hi, ns, ncclDouble, hi_rank, ctx->comm, st));
        if (nr) KLE_NCCL(ncclRecv(recv_lo, nr, ncclDouble, lo_rank, ctx->comm, st));
        KLE_NCCL(ncclGroupEnd());
    } else {
        KLE_TRY(stage_reserve(ctx, ns + nr));
        double *hs = ctx->h_stage, *hr = hs + ns;
        if (ns) KLE_HIP(hipMemcpyAsync(hs, send_hi, sizeof(double) * ns, hipMemcpyDeviceToHost, st));
        KLE_HIP(hipStreamSynchronize(st));
        if (ctx->hcomm.halo(nullptr, 0, lo_rank, hs, ns, hi_rank, hr, nr, nullptr, 0, ctx->hcomm.user))
            return fail(KLE_ERR_COMM, "host halo callback failed (reverse halo)");
        if (nr) KLE_HIP(hipMemcpyAsync(recv_lo, hr, sizeof(double) * nr, hipMemcpyHostToDevice, st));
        KLE_HIP(hipStreamSynchronize(st));
    }
    KLE_TRY(ctx->toc("halo_rev", &ev, st));
    return 0;
}

// Reverse of a graph-partition halo (symmetric storage: MPISBAIJ's reverse
// scatter with ADD, the transfer only): each peer of higher rank gets the
// sums of its ghost group (gsend: the upper ghost groups back to back in peer
// order, from ext node hi0 on, bs entries per node), each peer of lower rank
// sends the sums for the owned nodes it ghosts into rbuf (the forward halo's
// send slices of the lower peers, which lead the send list).  The caller adds
// rbuf into y through the send index lists.
int halo_reverse_plan(kle_ctx *ctx, const HaloPlan &P, int64_t hi0, int bs, const double *gsend, double *rbuf,
                      hipStream_t st)
{
    if (ctx->nranks == 1 || P.peers.empty()) return 0;
    if (!st) st = ctx->stream;
    const size_t np = P.peers.size();
    std::vector<int64_t> sc(np, 0), rc(np, 0);
    int64_t ns = 0, nr = 0;
    for (size_t k = 0; k < np; ++k) {
        if (P.peers[k] > ctx->rank) sc[k] = P.recv_cnt[k] * bs;
        if (P.peers[k] < ctx->rank) rc[k] = P.send_cnt[k] * bs;
        ns += sc[k];
        nr += rc[k];
    }
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(ctx->tic("halo_rev", &ev, st));
    if (ctx->ipc) {
        KLE_TRY(ipc_reverse_plan(ctx, P, hi0, bs, gsend, rbuf, st));
    } else if (ctx->comm) {
        KLE_NCCL(ncclGroupStart());
        for (size_t k = 0; k < np; ++k) {
            if (sc[k])
                KLE_NCCL(ncclSend(gsend + (P.recv_off[k] - hi0) * bs, sc[k], ncclDouble, P.peers[k], ctx->comm, st));
            if (rc[k]) KLE_NCCL(ncclRecv(rbuf + P.send_off[k] * bs, rc[k], ncclDouble, P.peers[k], ctx->comm, st));
        }
        KLE_NCCL(ncclGroupEnd());
    } else {
        if (!ctx->hcomm.exchange) return fail(KLE_ERR_COMM, "host transport has no exchange callback (reverse halo)");
        KLE_TRY(stage_reserve(ctx, ns + nr));
        double *hs = ctx->h_stage, *hr = hs + ns;
        // (the upper ghost groups are contiguous in peer order, the lower
        // peers' send slices lead the send list: both buffers are packed)
        if (ns) KLE_HIP(hipMemcpyAsync(hs, gsend, sizeof(double) * ns, hipMemcpyDeviceToHost, st));
        KLE_HIP(hipStreamSynchronize(st));
        if (ctx->hcomm.exchange((int)np, P.peers.data(), hs, sc.data(), hr, rc.data(), ctx->hcomm.user))
            return fail(KLE_ERR_COMM, "host exchange callback failed (reverse halo)");
        if (nr) KLE_HIP(hipMemcpyAsync(rbuf, hr, sizeof(double) * nr, hipMemcpyHostToDevice, st));
        KLE_HIP(hipStreamSynchronize(st));
    }
    KLE_TRY(ctx->toc("halo_rev", &ev, st));
    return 0;
}

}  // namespace kle

using namespace kle;

// ----------------------------------------------------------- ctx profiling
hipEvent_t kle_ctx::get_event()
{
    if (!event_pool.empty()) {
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int kle_ctx::tic(const char *name, std::pair<hipEvent_t, hipEvent_t> *ev, hipStream_t s)
{
    if (!s) s = stream;
    ev->first = ev->second = nullptr;
    if (!profiling || (!prof_only.empty() && prof_only != name)) return 0;
    // sampling: time one launch in prof_every (the events cost a few us per
    // launch on the stream, 6 % of a CG iteration on a 1/8 slab)
    if (prof_every > 1 && (prof_seq++ % prof_every) != 0) return 0;
    ev->first = get_event();
    ev->second = get_event();
    if (!ev->first || !ev->second) return fail(KLE_ERR_DEVICE, "hipEventCreate failed");
    KLE_HIP(hipEventRecord(ev->first, s));
    return 0;
}

int kle_ctx::toc(const char *name, std::pair<hipEvent_t, hipEvent_t> *ev, hipStream_t s)
{
    if (!profiling || !ev->first) return 0;
    KLE_HIP(hipEventRecord(ev->second, s ? s : stream));
    Stat &st = stats[name];
    st.pending.push_back(*ev);
    if (st.pending.size() > 8192) return resolve_stats();
    return 0;
}

int kle_ctx::resolve_stats()
{
    for (auto &kv : stats) {
        for (auto &pr : kv.second.pending) {
            KLE_HIP(hipEventSynchronize(pr.second));
            float ms = 0;
            KLE_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
            kv.second.ms += ms;
            kv.second.count += 1;
            event_pool.push_back(pr.first);
            event_pool.push_back(pr.second);
        }
        kv.second.pending.clear();
    }
    return 0;
}

// ------------------------------------------------------------------ C ABI
extern "C" {

const char *kle_last_error(void) { return g_err.c_str(); }

int kle_set_tuning(const char *key, int value)
{
    KLE_ARG(key, "null key");
    const std::string k(key);
    if (k == "spmv_waves") {
        KLE_ARG(value == 0 || value == 4 || value == 8, "spmv_waves: 0 (auto), 4 or 8");
        g_tune.spmv_waves = value;
    } else if (k == "upd_nt") {
        KLE_ARG(value >= 0 && value <= 2, "upd_nt: 0 off, 1 on, 2 auto");
        g_tune.upd_nt = value;
    } else if (k == "upd_preload") {
        KLE_ARG(value == 0 || value == 1, "upd_preload: 0 or 1");
        g_tune.upd_preload = value;
    } else if (k == "spmv_dict") {
        KLE_ARG(value == 0 || value == 1, "spmv_dict: 0 or 1");
        g_tune.spmv_dict = value;
    } else if (k == "spmv_dict_min_rows") {
        KLE_ARG(value >= 0, "spmv_dict_min_rows: >= 0");
        g_tune.spmv_dict_min_rows = value;
    } else if (k == "spmv_sym") {
        KLE_ARG(value == 0 || value == 1, "spmv_sym: 0 or 1");
        g_tune.spmv_sym = value;
    } else if (k == "spmv_sym_det") {
        KLE_ARG(value == 0 || value == 1, "spmv_sym_det: 0 or 1");
        g_tune.spmv_sym_det = value;
    } else if (k == "spmv_sym_waves") {
        KLE_ARG(value == 0 || value == 8 || value == 16, "spmv_sym_waves: 0 (auto), 8 or 16");
        g_tune.spmv_sym_waves = value;
    } else if (k == "spmv_sym_tile64") {
        KLE_ARG(value >= 0 && value <= 2, "spmv_sym_tile64: 0 auto, 1 always, 2 never");
        g_tune.spmv_sym_tile64 = value;
    } else if (k == "spmv_sym_tile64_max") {
        KLE_ARG(value >= 0, "spmv_sym_tile64_max: >= 0 tiles");
        g_tune.spmv_sym_tile64_max = value;
    } else if (k == "spmv_sym_xcd") {
        KLE_ARG(value >= 0 && value <= 4096, "spmv_sym_xcd: 0 .. 4096 tiles");
        g_tune.spmv_sym_xcd = value;
    } else if (k == "spmv_sym_ovl_b") {
        KLE_ARG(value >= 0 && value <= 100, "spmv_sym_ovl_b: 0 .. 100 %");
        g_tune.spmv_sym_ovl_b = value;
    } else if (k == "spmv_sym_stpol") {
        KLE_ARG(value >= 0 && value <= 3, "spmv_sym_stpol: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1");
        g_tune.spmv_sym_stpol = value;
    } else if (k == "spmv_gsym_stpol") {
        KLE_ARG(value >= 0 && value <= 3, "spmv_gsym_stpol: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1");
        g_tune.spmv_gsym_stpol = value;
    } else if (k == "spmv_sym_align") {
        KLE_ARG(value == 0 || value == 1, "spmv_sym_align: 0 or 1");
        g_tune.spmv_sym_align = value;
    } else if (k == "spmv_sym_early") {
        KLE_ARG(value == 0 || value == 1, "spmv_sym_early: 0 or 1");
        g_tune.spmv_sym_early = value;
        } else if (k == "upd_unroll") {
        KLE_ARG(value == 1 || value == 2, "upd_unroll: 1 or 2");
        g_tune.upd_unroll = value;
    } else if (k == "spmv_gsym_brick") {
        KLE_ARG(value == 0 || value == 1, "spmv_gsym_brick: 0 or 1");
        g_tune.spmv_gsym_brick = value;
        } else if (k == "spmv_brick_pair") {
        KLE_ARG(value == 0 || value == 1, "spmv_brick_pair: 0 or 1");
        g_tune.spmv_brick_pair = value;
    } else if (k == "spmv_brick_singles") {
        KLE_ARG(value == 0 || value == 1, "spmv_brick_singles: 0 or 1");
        g_tune.spmv_brick_singles = value;
                        } else if (k == "spmv_gather_wps") {
        KLE_ARG(value == 0 || value == 1 || value == 2 || value == 4, "spmv_gather_wps: 0 (auto), 1, 2 or 4");
        g_tune.spmv_gather_wps = value;
                } else if (k == "spmv_brick_split") {
        KLE_ARG(value >= 0, "spmv_brick_split: nbx + 100 nby + 10000 nbz (0: planned)");
        g_tune.spmv_brick_split = value;
    } else if (k == "spmv_brick_rounds") {
        KLE_ARG(value >= 1 && value <= 4, "spmv_brick_rounds: 1 .. 4 bricks per CU");
        g_tune.spmv_brick_rounds = value;
    } else if (k == "spmv_brick_max") {
        KLE_ARG(value >= 0, "spmv_brick_max: >= 0 (0: one brick per CU)");
        g_tune.spmv_brick_max = value;
    } else if (k == "spmv_sym_brick") {
        KLE_ARG(value == 0 || value == 1, "spmv_sym_brick: 0 (128-row tiles) or 1 (bricks)");
        g_tune.spmv_sym_brick = value;
    } else if (k == "spmv_sym_tz") {
        KLE_ARG(value == 0 || value == 2 || value == 4, "spmv_sym_tz: 0 (auto), 2 or 4");
        g_tune.spmv_sym_tz = value;
    } else if (k == "ksp_pipe_gather") {
        KLE_ARG(value == 0 || value == 1, "ksp_pipe_gather: 0 or 1");
        g_tune.ksp_pipe_gather = value;
    } else if (k == "ksp_sr_gather") {
        KLE_ARG(value >= 0 && value <= 2, "ksp_sr_gather: 0, 1 or 2");
        g_tune.ksp_sr_gather = value;
    } else if (k == "ipc_sentinel") {
        KLE_ARG(value == 0 || value == 1, "ipc_sentinel: 0 or 1");
        g_tune.ipc_sentinel = value;
    } else if (k == "ksp_corr_fault") {
        KLE_ARG(value == 0 || value == 1, "ksp_corr_fault: 0 or 1 (test hook)");
        g_tune.ksp_corr_fault = value;
    } else if (k == "ksp_refine") {
        KLE_ARG(value >= 0 && value <= 8, "ksp_refine: 0 .. 8");
        g_tune.ksp_refine = value;
    } else if (k == "spmv_gsym_rows") {
        KLE_ARG(value == 8 || value == 16 || value == 32 || value == 64 || value == 128,
                "spmv_gsym_rows: 8, 16, 32, 64 or 128");
        g_tune.spmv_gsym_rows = value;
    } else if (k == "spmv_gsym_waves") {
        KLE_ARG(value == 0 || value == 8 || value == 16, "spmv_gsym_waves: 0, 8 or 16");
        g_tune.spmv_gsym_waves = value;
    } else if (k == "spmv_gsym_split") {
        KLE_ARG(value >= 0, "spmv_gsym_split: >= 0");
        g_tune.spmv_gsym_split = value;
#ifdef KLE_PROBE_BUILD
    } else if (k == "spmv_sym_probe") {
        KLE_ARG(value >= 0, "spmv_sym_probe: bit mask (< 4096) | ring slots << 12");
        g_tune.spmv_sym_probe = value;
    } else if (k == "spmv_sym_probe_ts") {
        KLE_ARG(value >= 0, "spmv_sym_probe_ts: workgroup slots (0: off)");
        if (g_probe_ts) (void)hipFree(g_probe_ts);
        g_probe_ts = nullptr;
        g_probe_ts_cap = 0;
        if (value > 0) {
            KLE_HIP(hipMalloc(&g_probe_ts, sizeof(unsigned long long) * 8 * (size_t)value));
            KLE_HIP(hipMemset(g_probe_ts, 0, sizeof(unsigned long long) * 8 * (size_t)value));
            g_probe_ts_cap = value;
        }
#endif
    } else if (k == "spmv_sym_min_rows") {
        KLE_ARG(value >= 0, "spmv_sym_min_rows: >= 0");
        g_tune.spmv_sym_min_rows = value;
    } else if (k == "spmv_x_lds") {
        KLE_ARG(value == 0 || value == 1, "spmv_x_lds: 0 or 1");
        g_tune.spmv_x_lds = value;
    } else if (k == "spmv_xcd_chunk") {
        KLE_ARG(value >= 0 && value <= 4096, "spmv_xcd_chunk: 0 (round-robin) or row blocks per XCD run");
        g_tune.spmv_xcd_chunk = value;
    } else if (k == "spmv_dyn_lds") {
        KLE_ARG(value >= -1 && value <= 65536, "spmv_dyn_lds: -1 (auto) or 0..65536 bytes");
        g_tune.spmv_dyn_lds = value;
    } else {
        return fail(KLE_ERR_ARG, "unknown tuning key '%s'", key);
    }
    return 0;
}

#ifdef KLE_PROBE_BUILD
// probe build only: the phase timestamps of the last instrumented launches
extern "C" int kle_probe_timestamps(unsigned long long *out, int64_t slots)
{
    KLE_ARG(out && slots >= 0 && slots <= g_probe_ts_cap, "bad arg");
    KLE_HIP(hipDeviceSynchronize());
    KLE_HIP(hipMemcpy(out, g_probe_ts, sizeof(unsigned long long) * 8 * (size_t)slots, hipMemcpyDeviceToHost));
    return 0;
}
#endif

int kle_get_tuning(const char *key, int *value)
{
    KLE_ARG(key && value, "null arg");
    const std::string k(key);
    if (k == "spmv_waves") *value = g_tune.spmv_waves;
    else if (k == "spmv_dyn_lds") *value = g_tune.spmv_dyn_lds;
    else if (k == "spmv_xcd_chunk") *value = g_tune.spmv_xcd_chunk;
    else if (k == "spmv_x_lds") *value = g_tune.spmv_x_lds;
    else if (k == "spmv_dict") *value = g_tune.spmv_dict;
    else if (k == "upd_preload") *value = g_tune.upd_preload;
    else if (k == "upd_nt") *value = g_tune.upd_nt;
    else if (k == "spmv_dict_min_rows") *value = g_tune.spmv_dict_min_rows;
    else if (k == "spmv_sym") *value = g_tune.spmv_sym;
    else if (k == "spmv_sym_det") *value = g_tune.spmv_sym_det;
    else if (k == "spmv_sym_waves") *value = g_tune.spmv_sym_waves;
    else if (k == "spmv_sym_tz") *value = g_tune.spmv_sym_tz;
    else if (k == "spmv_sym_brick") *value = g_tune.spmv_sym_brick;
    else if (k == "spmv_brick_max") *value = g_tune.spmv_brick_max;
    else if (k == "spmv_brick_rounds") *value = g_tune.spmv_brick_rounds;
    else if (k == "spmv_brick_split") *value = g_tune.spmv_brick_split;
    else if (k == "spmv_brick_singles") *value = g_tune.spmv_brick_singles;
    else if (k == "spmv_brick_pair") *value = g_tune.spmv_brick_pair;
    else if (k == "spmv_gather_wps") *value = g_tune.spmv_gather_wps;
    else if (k == "spmv_gsym_brick") *value = g_tune.spmv_gsym_brick;
    else if (k == "upd_unroll") *value = g_tune.upd_unroll;
    else if (k == "spmv_sym_early") *value = g_tune.spmv_sym_early;
    else if (k == "spmv_sym_align") *value = g_tune.spmv_sym_align;
    else if (k == "spmv_sym_stpol") *value = g_tune.spmv_sym_stpol;
    else if (k == "spmv_gsym_stpol") *value = g_tune.spmv_gsym_stpol;
    else if (k == "spmv_sym_ovl_b") *value = g_tune.spmv_sym_ovl_b;
    else if (k == "spmv_sym_xcd") *value = g_tune.spmv_sym_xcd;
    else if (k == "spmv_sym_tile64") *value = g_tune.spmv_sym_tile64;
    else if (k == "spmv_sym_tile64_max") *value = g_tune.spmv_sym_tile64_max;
#ifdef KLE_PROBE_BUILD
    else if (k == "spmv_sym_probe") *value = g_tune.spmv_sym_probe;
#endif
    else if (k == "spmv_gsym_rows") *value = g_tune.spmv_gsym_rows;
    else if (k == "ksp_refine") *value = g_tune.ksp_refine;
    else if (k == "ksp_corr_fault") *value = g_tune.ksp_corr_fault;
    else if (k == "ipc_sentinel") *value = g_tune.ipc_sentinel;
    else if (k == "ksp_pipe_gather") *value = g_tune.ksp_pipe_gather;
    else if (k == "ksp_sr_gather") *value = g_tune.ksp_sr_gather;
    else if (k == "spmv_gsym_split") *value = g_tune.spmv_gsym_split;
    else if (k == "spmv_gsym_waves") *value = g_tune.spmv_gsym_waves;
    else if (k == "spmv_sym_min_rows") *value = g_tune.spmv_sym_min_rows;
    else return fail(KLE_ERR_ARG, "unknown tuning key '%s'", key);
    return 0;
}
int kle_version(void) { return 1; }

int kle_get_unique_id(unsigned char out[128])
{
    ncclUniqueId id;
    KLE_NCCL(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(out, &id, 128);
    return 0;
}

static int ctx_init(int device, int rank, int nranks, kle_ctx **out)
{
    KLE_ARG(out, "null output");
    KLE_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank %d / nranks %d", rank, nranks);
    int ndev = 0;
    KLE_HIP(hipGetDeviceCount(&ndev));
    KLE_ARG(device >= 0 && device < ndev, "device %d not present (%d visible)", device, ndev);
    KLE_HIP(hipSetDevice(device));
    kle_ctx *c = new kle_ctx;
    c->device = device;
    c->rank = rank;
    c->nranks = nranks;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    // the comm stream carries the halo exchange and the Krylov reductions /
    // allreduce that run beside the SpMV; at the highest priority its few
    // workgroups are dispatched as soon as SpMV workgroups retire instead of
    // queueing behind the SpMV's whole grid
    int prio_lo = 0, prio_hi = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = 0;
    const hipError_t se = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (se != hipSuccess ||
        hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_x_ready, sync_event_flags()) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_halo_done, sync_event_flags()) != hipSuccess) {
        kle_ctx_destroy(c);
        return fail(KLE_ERR_DEVICE, "hipStreamCreate / hipEventCreate failed");
    }
    if (hipMalloc(&c->d_partials, sizeof(double) * 4 * PART_STRIDE) != hipSuccess ||
        hipMalloc(&c->d_scal, sizeof(double) * NSCAL) != hipSuccess ||
        hipMalloc(&c->d_istate, sizeof(int) * I_COUNT) != hipSuccess ||
        hipHostMalloc(&c->h_scal, sizeof(double) * NSCAL) != hipSuccess ||
        hipHostMalloc(&c->h_istate, sizeof(int) * I_COUNT) != hipSuccess) {
        kle_ctx_destroy(c);
        return fail(KLE_ERR_MEM, "context scratch allocation failed");
    }
    hipMemset(c->d_scal, 0, sizeof(double) * NSCAL);
    hipMemset(c->d_istate, 0, sizeof(int) * I_COUNT);
    *out = c;
    return 0;
}

// ncclCommInitRank blocks until every rank has joined; a rank that died
// before joining would hang this one (and the 8-GPU bench) for ever.  Run the
// init on a helper thread and give up after KLE_COMM_TIMEOUT_S seconds
// (default 300): the caller gets KLE_ERR_COMM and exits non-zero; the helper
// is left blocked (the process is about to end).
static int comm_init_deadline(kle_ctx *c, int nranks, const ncclUniqueId &id, int rank)
{
    struct Job {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false;
        ncclComm_t comm = nullptr;
        ncclResult_t r = ncclInternalError;
    };
    auto job = std::make_shared<Job>();
    const int device = c->device;
    std::thread th([job, device, nranks, id, rank]() {
        ncclComm_t comm = nullptr;
        ncclResult_t r = ncclInternalError;
        if (hipSetDevice(device) == hipSuccess) r = ncclCommInitRank(&comm, nranks, id, rank);
        std::lock_guard<std::mutex> lk(job->mu);
        job->comm = comm;
        job->r = r;
        job->done = true;
        job->cv.notify_all();
    });
    const char *e = getenv("KLE_COMM_TIMEOUT_S");
    const double tmo = e && atof(e) > 0 ? atof(e) : 300.0;
    bool done;
    {
        std::unique_lock<std::mutex> lk(job->mu);
        done = job->cv.wait_for(lk, std::chrono::duration<double>(tmo), [&] { return job->done; });
    }
    if (!done) {
        th.detach();
        return fail(KLE_ERR_COMM, "ncclCommInitRank (rank %d of %d) did not complete within %.0f s "
                    "(KLE_COMM_TIMEOUT_S): a peer never joined", rank, nranks, tmo);
    }
    th.join();
    if (job->r != ncclSuccess) return fail(KLE_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(job->r));
    c->comm = job->comm;
    return 0;
}

int kle_ctx_create(int device, int rank, int nranks, const unsigned char *unique_id, kle_ctx **out)
{
    KLE_ARG(nranks == 1 || unique_id, "nranks > 1 needs an RCCL unique id");
    kle_ctx *c;
    KLE_TRY(ctx_init(device, rank, nranks, &c));
    // nranks == 1 with an id: a one-rank communicator, so the RCCL calls of
    // the solver (allreduce on the compute / comm streams) run on one GPU too
    if (unique_id) {
        ncclUniqueId id;
        memcpy(&id, unique_id, 128);
        int rc = comm_init_deadline(c, nranks, id, rank);
        if (rc) {
            kle_ctx_destroy(c);
            return rc;
        }
    }
    *out = c;
    return 0;
}

int kle_ctx_create_host_comm(int device, int rank, int nranks, const kle_host_comm *comm, kle_ctx **out)
{
    KLE_ARG(comm && comm->allreduce && comm->halo, "host transport needs allreduce and halo callbacks");
    kle_ctx *c;
    KLE_TRY(ctx_init(device, rank, nranks, &c));
    c->hcomm = *comm;
    *out = c;
    return 0;
}

int kle_ctx_destroy(kle_ctx *c)
{
    if (!c) return 0;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    c->resolve_stats();
    ipc_destroy(c);
    for (auto e : c->event_pool) hipEventDestroy(e);
    if (c->comm) ncclCommDestroy(c->comm);
    hipFree(c->d_partials);
    hipFree(c->d_scal);
    hipFree(c->d_istate);
    hipHostFree(c->h_scal);
    hipHostFree(c->h_istate);
    if (c->h_stage) hipHostFree(c->h_stage);
    if (c->stream) hipStreamDestroy(c->stream);
    if (c->comm_stream) hipStreamDestroy(c->comm_stream);
    if (c->ev_x_ready) hipEventDestroy(c->ev_x_ready);
    if (c->ev_halo_done) hipEventDestroy(c->ev_halo_done);
    delete c;
    return 0;
}

int kle_ctx_synchronize(kle_ctx *c)
{
    KLE_ARG(c, "null ctx");
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int kle_ctx_barrier(kle_ctx *c)
{
    KLE_ARG(c, "null ctx");
    // a one-double allreduce on the stream is the device-side barrier
    KLE_TRY(allreduce_sum(c, c->d_scal + S_TMP1, 1));
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int kle_ctx_get_device(kle_ctx *c, int *device, char *pci_bus_id, int len, int *transport)
{
    KLE_ARG(c && device && transport && (pci_bus_id == nullptr || len > 0), "bad arg");
    *device = c->device;
    *transport = c->comm ? 1 : c->ipc ? 3 : (c->nranks > 1 ? 2 : 0);
    if (pci_bus_id) KLE_HIP(hipDeviceGetPCIBusId(pci_bus_id, len, c->device));
    return 0;
}

int kle_ctx_get_comm_info(kle_ctx *c, int *count, int *rank)
{
    KLE_ARG(c && count && rank, "bad arg");
    *count = 0;
    *rank = -1;
    if (c->comm) {
        KLE_NCCL(ncclCommCount(c->comm, count));
        KLE_NCCL(ncclCommUserRank(c->comm, rank));
    }
    return 0;
}

int kle_ctx_set_profiling(kle_ctx *c, int on)
{
    KLE_ARG(c, "null ctx");
    c->profiling = on != 0;
    return 0;
}

int kle_ctx_set_profiling_filter(kle_ctx *c, const char *name)
{
    KLE_ARG(c, "null ctx");
    c->prof_only = name ? name : "";
    return 0;
}

int kle_ctx_set_profiling_sample(kle_ctx *c, int every)
{
    KLE_ARG(c && every >= 1, "bad arg");
    c->prof_every = every;
    c->prof_seq = 0;
    return 0;
}

int kle_ctx_get_kernel_stats(kle_ctx *c, const char *name, int64_t *count, double *total_ms)
{
    KLE_ARG(c && name, "null arg");
    KLE_TRY(c->resolve_stats());
    auto it = c->stats.find(name);
    *count = it == c->stats.end() ? 0 : it->second.count;
    *total_ms = it == c->stats.end() ? 0 : it->second.ms;
    return 0;
}

int kle_ctx_reset_kernel_stats(kle_ctx *c)
{
    KLE_ARG(c, "null ctx");
    KLE_TRY(c->resolve_stats());
    for (auto &kv : c->stats) {
        kv.second.count = 0;
        kv.second.ms = 0;
    }
    return 0;
}

// --------------------------------------------------------------------- vec
int kle_vec_create(kle_ctx *ctx, int64_t n_local, int64_t n_global, kle_vec **out)
{
    KLE_ARG(ctx && out, "null arg");
    KLE_ARG(n_local >= 0, "negative size");
    int64_t lo = 0;
    if (ctx->nranks > 1) {
        // ownership ranges follow rank order: prefix sum over ranks
        std::vector<int64_t> all;
        KLE_TRY(allgather_i64(ctx, n_local, all));
        int64_t tot = 0;
        for (int r = 0; r < ctx->nranks; ++r) {
            if (r == ctx->rank) lo = tot;
            tot += all[r];
        }
        if (n_global < 0) n_global = tot;
        KLE_ARG(n_global == tot, "global size %lld != sum of local sizes %lld",
                (long long)n_global, (long long)tot);
    } else {
        if (n_global < 0) n_global = n_local;
        KLE_ARG(n_global == n_local, "single rank: global size must equal local size");
    }
    return vec_alloc(ctx, n_local, n_global, lo, 0, 0, out);
}

int kle_vec_create_mesh(kle_ctx *ctx, const kle_mesh *m, int bs, kle_vec **out)
{
    KLE_ARG(ctx && m && out, "null arg");
    KLE_ARG(bs >= 1 && bs <= 16, "bad block size %d", bs);
    KLE_ARG(m->nranks == ctx->nranks && m->rank == ctx->rank, "mesh partition does not match ctx");
    int64_t own = (m->node_end - m->node_begin) * bs;
    KLE_TRY(vec_alloc(ctx, own, m->N * bs, m->node_begin * bs,
                      (m->node_begin - m->ext_begin) * bs, (m->ext_end - m->node_end) * bs, out));
    kle_vec *v = *out;
    v->bs = bs;
    v->lo_rank = m->halo_lo_rank;
    v->hi_rank = m->halo_hi_rank;
    v->send_lo = m->send_lo_nodes * bs;
    v->send_hi = m->send_hi_nodes * bs;
    v->plan = m->plan;
    return 0;
}

int kle_vec_duplicate(const kle_vec *v, kle_vec **out)
{
    KLE_ARG(v && out, "null arg");
    KLE_TRY(vec_alloc(v->ctx, v->n_local, v->n_global, v->lo, v->ghost_lo, v->ghost_hi, out));
    kle_vec *w = *out;
    w->bs = v->bs;
    w->lo_rank = v->lo_rank;
    w->hi_rank = v->hi_rank;
    w->send_lo = v->send_lo;
    w->send_hi = v->send_hi;
    w->plan = v->plan;
    return 0;
}

int kle_vec_destroy(kle_vec *v)
{
    if (!v) return 0;
    if (v->owns) hipFree(v->base);
    delete v;
    return 0;
}

int kle_vec_get_sizes(const kle_vec *v, int64_t *nl, int64_t *ng)
{
    KLE_ARG(v, "null vec");
    if (nl) *nl = v->n_local;
    if (ng) *ng = v->n_global;
    return 0;
}

int kle_vec_get_ownership_range(const kle_vec *v, int64_t *lo, int64_t *hi)
{
    KLE_ARG(v, "null vec");
    *lo = v->lo;
    *hi = v->lo + v->n_local;
    return 0;
}

#define VGRID(n) kle::grid_for((n), VB, VMAX)

int kle_vec_set(kle_vec *v, double a)
{
    KLE_ARG(v, "null vec");
    hipLaunchKernelGGL(k_set, dim3(VGRID(v->n_local)), dim3(VB), 0, v->ctx->stream, v->n_local, a,
                       v->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

static int same_layout(const kle_vec *a, const kle_vec *b)
{
    if (a->n_local != b->n_local || a->n_global != b->n_global)
        return fail(KLE_ERR_SIZ, "vector sizes differ (%lld/%lld vs %lld/%lld)",
                    (long long)a->n_local, (long long)a->n_global, (long long)b->n_local,
                    (long long)b->n_global);
    return 0;
}

int kle_vec_copy(const kle_vec *x, kle_vec *y)
{
    KLE_ARG(x && y, "null vec");
    KLE_TRY(same_layout(x, y));
    KLE_HIP(hipMemcpyAsync(y->d, x->d, sizeof(double) * x->n_local, hipMemcpyDeviceToDevice,
                           x->ctx->stream));
    return 0;
}

int kle_vec_axpy(kle_vec *y, double a, const kle_vec *x)
{
    KLE_ARG(x && y, "null vec");
    KLE_TRY(same_layout(x, y));
    hipLaunchKernelGGL(k_axpy, dim3(VGRID(y->n_local)), dim3(VB), 0, y->ctx->stream, y->n_local, a,
                       x->d, y->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_aypx(kle_vec *y, double b, const kle_vec *x)
{
    KLE_ARG(x && y, "null vec");
    KLE_TRY(same_layout(x, y));
    hipLaunchKernelGGL(k_aypx, dim3(VGRID(y->n_local)), dim3(VB), 0, y->ctx->stream, y->n_local, b,
                       x->d, y->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_waxpy(kle_vec *w, double a, const kle_vec *x, const kle_vec *y)
{
    KLE_ARG(w && x && y, "null vec");
    KLE_TRY(same_layout(x, y));
    KLE_TRY(same_layout(x, w));
    hipLaunchKernelGGL(k_waxpy, dim3(VGRID(w->n_local)), dim3(VB), 0, w->ctx->stream, w->n_local,
                       a, x->d, y->d, w->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_scale(kle_vec *v, double a)
{
    KLE_ARG(v, "null vec");
    hipLaunchKernelGGL(k_scale, dim3(VGRID(v->n_local)), dim3(VB), 0, v->ctx->stream, v->n_local, a,
                       v->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_pointwise_mult(kle_vec *w, const kle_vec *x, const kle_vec *y)
{
    KLE_ARG(w && x && y, "null vec");
    KLE_TRY(same_layout(x, y));
    KLE_TRY(same_layout(x, w));
    hipLaunchKernelGGL(k_pmult, dim3(VGRID(w->n_local)), dim3(VB), 0, w->ctx->stream, w->n_local,
                       x->d, y->d, w->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_tensor_square(const kle_vec *v, int dim, kle_vec *out)
{
    KLE_ARG(v && out, "null vec");
    KLE_ARG(dim == 2 || dim == 3, "dim must be 2 or 3");
    const int ds = dim == 2 ? 3 : 6;
    KLE_ARG(v->n_local % dim == 0 && out->n_local == v->n_local / dim * ds, "sizes do not match dim %d", dim);
    const int64_t nodes = v->n_local / dim;
    if (dim == 2)
        hipLaunchKernelGGL(k_vtensv<2>, dim3(VGRID(nodes)), dim3(VB), 0, v->ctx->stream, nodes, v->d, out->d);
    else
        hipLaunchKernelGGL(k_vtensv<3>, dim3(VGRID(nodes)), dim3(VB), 0, v->ctx->stream, nodes, v->d, out->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_reciprocal(kle_vec *v)
{
    KLE_ARG(v, "null vec");
    hipLaunchKernelGGL(k_recip, dim3(VGRID(v->n_local)), dim3(VB), 0, v->ctx->stream, v->n_local,
                       v->d);
    KLE_HIP(hipGetLastError());
    return 0;
}

int kle_vec_dot(const kle_vec *x, const kle_vec *y, double *out)
{
    KLE_ARG(x && y && out, "null arg");
    KLE_TRY(same_layout(x, y));
    kle_ctx *c = x->ctx;
    int g = VGRID(x->n_local);
    hipLaunchKernelGGL(k_dot_partial, dim3(g), dim3(VB), 0, c->stream, x->n_local, x->d, y->d,
                       c->d_partials);
    KLE_HIP(hipGetLastError());
    KLE_TRY(reduce_partials(c, c->d_partials, g, 1, c->d_scal + S_TMP0));
    KLE_TRY(allreduce_sum(c, c->d_scal + S_TMP0, 1));
    KLE_HIP(hipMemcpyAsync(c->h_scal + S_TMP0, c->d_scal + S_TMP0, sizeof(double),
                           hipMemcpyDeviceToHost, c->stream));
    KLE_HIP(hipStreamSynchronize(c->stream));
    *out = c->h_scal[S_TMP0];
    return 0;
}

int kle_vec_norm2(const kle_vec *x, double *out)
{
    double d;
    KLE_TRY(kle_vec_dot(x, x, &d));
    *out = std::sqrt(d);
    return 0;
}

int kle_vec_set_values(kle_vec *v, int64_t n, const int64_t *idx, const double *vals, int addv)
{
    KLE_ARG(v && (n == 0 || (idx && vals)), "null arg");
    if (n == 0) return 0;
    std::vector<int64_t> loc(n);
    for (int64_t i = 0; i < n; ++i) {
        int64_t l = idx[i] - v->lo;
        if (l < 0 || l >= v->n_local)
            return fail(KLE_ERR_OUTOFRANGE, "index %lld not owned ([%lld,%lld))",
                        (long long)idx[i], (long long)v->lo, (long long)(v->lo + v->n_local));
        loc[i] = l;
    }
    int64_t *di;
    double *dv;
    KLE_HIP(hipMalloc(&di, sizeof(int64_t) * n));
    KLE_HIP(hipMalloc(&dv, sizeof(double) * n));
    KLE_HIP(hipMemcpyAsync(di, loc.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice,
                           v->ctx->stream));
    KLE_HIP(hipMemcpyAsync(dv, vals, sizeof(double) * n, hipMemcpyHostToDevice, v->ctx->stream));
    hipLaunchKernelGGL(k_scatter_values, dim3(VGRID(n)), dim3(VB), 0, v->ctx->stream, n, di, dv,
                       v->d, addv);
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(v->ctx->stream));
    hipFree(di);
    hipFree(dv);
    return 0;
}

int kle_vec_get_values(const kle_vec *v, int64_t n, const int64_t *idx, double *vals)
{
    KLE_ARG(v && (n == 0 || (idx && vals)), "null arg");
    if (n == 0) return 0;
    std::vector<int64_t> loc(n);
    for (int64_t i = 0; i < n; ++i) {
        int64_t l = idx[i] - v->lo;
        if (l < -v->ghost_lo || l >= v->n_local + v->ghost_hi)
            return fail(KLE_ERR_OUTOFRANGE, "index %lld not local", (long long)idx[i]);
        loc[i] = l;
    }
    int64_t *di;
    double *dv;
    KLE_HIP(hipMalloc(&di, sizeof(int64_t) * n));
    KLE_HIP(hipMalloc(&dv, sizeof(double) * n));
    KLE_HIP(hipMemcpyAsync(di, loc.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice,
                           v->ctx->stream));
    hipLaunchKernelGGL(k_gather_values, dim3(VGRID(n)), dim3(VB), 0, v->ctx->stream, n, di, v->d,
                       dv);
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipMemcpyAsync(vals, dv, sizeof(double) * n, hipMemcpyDeviceToHost, v->ctx->stream));
    KLE_HIP(hipStreamSynchronize(v->ctx->stream));
    hipFree(di);
    hipFree(dv);
    return 0;
}

int kle_vec_get_array(const kle_vec *v, double *host)
{
    KLE_ARG(v && host, "null arg");
    KLE_HIP(hipMemcpyAsync(host, v->d, sizeof(double) * v->n_local, hipMemcpyDeviceToHost,
                           v->ctx->stream));
    KLE_HIP(hipStreamSynchronize(v->ctx->stream));
    return 0;
}

int kle_vec_set_array(kle_vec *v, const double *host)
{
    KLE_ARG(v && host, "null arg");
    KLE_HIP(hipMemcpyAsync(v->d, host, sizeof(double) * v->n_local, hipMemcpyHostToDevice,
                           v->ctx->stream));
    KLE_HIP(hipStreamSynchronize(v->ctx->stream));
    return 0;
}

int kle_vec_restore_array(kle_vec *v, const double *host) { return kle_vec_set_array(v, host); }

int kle_vec_assemble(kle_vec *v)
{
    KLE_ARG(v, "null vec");
    KLE_HIP(hipStreamSynchronize(v->ctx->stream));
    return 0;
}

int kle_vec_ghost_update(kle_vec *v)
{
    KLE_ARG(v, "null vec");
    return halo_exchange(v->ctx, v->base, v->ghost_lo, v->n_local, v->ghost_hi, v->lo_rank,
                         v->hi_rank, v->send_lo, v->send_hi, nullptr, v->plan.get());
}

int kle_vec_device_ptr(const kle_vec *v, double **p)
{
    KLE_ARG(v && p, "null arg");
    *p = v->d;
    return 0;
}

int kle_stream_bench(kle_ctx *ctx, int64_t bytes, int reps, int mode, double *gbps)
{
    KLE_ARG(ctx && gbps && bytes >= 64 && reps >= 1, "bad arg");
    int64_t n4 = bytes / 32;
    double4 *a, *b;
    KLE_HIP(hipMalloc(&a, n4 * 32));
    const bool copy = mode == 0 || mode == 11 || mode == 12;
    KLE_HIP(hipMalloc(&b, copy ? n4 * 32 : 64));
    KLE_HIP(hipMemsetAsync(a, 0, n4 * 32, ctx->stream));
    KLE_ARG(mode >= 0 && mode <= 13, "stream mode 0..13");
    const int g = ctx->num_cus * 8;
    // mode 13: 1024-thread workgroups, 16 B x 4 in flight, KLE_STREAM_WGS of
    // them (default one per CU): the streaming rate of a part of the CUs
    const char *wg_env = getenv("KLE_STREAM_WGS");
    const int g13 = wg_env && atoi(wg_env) > 0 ? atoi(wg_env) : ctx->num_cus;
    const int64_t n16 = n4 * 2;
    const dvec2 *a2 = reinterpret_cast<const dvec2 *>(a);
    double *o = reinterpret_cast<double *>(b);
    // 0 copy (16 B, 4 in flight, nt stores), 1 read (16 B, 4 in flight, nt):
    // the ceilings bench.py reports; the rest are variants of them
    auto launch = [&]() {
        switch (mode) {
        case 0: hipLaunchKernelGGL((k_stream_cp<4, true>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, reinterpret_cast<dvec2 *>(b)); break;
        case 1: hipLaunchKernelGGL((k_stream_rd<4, true, 16>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 2: hipLaunchKernelGGL(k_stream_read8<true>, dim3(g), dim3(256), 0, ctx->stream, n4 * 4, (const double *)a, o); break;
        case 3: hipLaunchKernelGGL(k_stream_read8<false>, dim3(g), dim3(256), 0, ctx->stream, n4 * 4, (const double *)a, o); break;
        case 4: hipLaunchKernelGGL(k_stream_read, dim3(g), dim3(256), 0, ctx->stream, n4, a, o); break;  // (round 1-4 "read ceiling")
        case 5: hipLaunchKernelGGL((k_stream_rd<4, false, 16>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 6: hipLaunchKernelGGL((k_stream_rd<8, true, 16>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 7: hipLaunchKernelGGL((k_stream_rd<4, true, 16>), dim3(g / 2), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 8: hipLaunchKernelGGL((k_stream_rd<2, true, 16>), dim3(g * 2), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 9: hipLaunchKernelGGL((k_stream_rd<4, true, 8>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 10: hipLaunchKernelGGL((k_stream_rd<8, true, 8>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, o); break;
        case 11: hipLaunchKernelGGL(k_stream_copy, dim3(g), dim3(256), 0, ctx->stream, n4, a, b); break;  // (round 1-4 copy)
        case 13: hipLaunchKernelGGL((k_stream_rd<4, true, 16, 1024>), dim3(g13), dim3(1024), 0, ctx->stream, n16, a2, o); break;
        default: hipLaunchKernelGGL((k_stream_cp<4, false>), dim3(g), dim3(256), 0, ctx->stream, n16, a2, reinterpret_cast<dvec2 *>(b)); break;
        }
    };
    launch();
    hipEvent_t e0, e1;
    KLE_HIP(hipEventCreate(&e0));
    KLE_HIP(hipEventCreate(&e1));
    KLE_HIP(hipEventRecord(e0, ctx->stream));
    for (int r = 0; r < reps; ++r) launch();
    KLE_HIP(hipEventRecord(e1, ctx->stream));
    KLE_HIP(hipEventSynchronize(e1));
    float ms;
    KLE_HIP(hipEventElapsedTime(&ms, e0, e1));
    *gbps = (copy ? 2.0 : 1.0) * n4 * 32 * reps / (ms * 1e-3) / 1e9;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipFree(a);
    hipFree(b);
    return 0;
}

int kle_stream_copy_bench(kle_ctx *ctx, int64_t bytes, int reps, double *gbps)
{
    return kle_stream_bench(ctx, bytes, reps, 0, gbps);
}

}  // extern "C"
