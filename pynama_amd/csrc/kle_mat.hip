// kle_mat.hip -- device sparse matrices and SpMV kernels for gfx950.
//
// Two formats:
//  * node-block ("nb"): the KLE operators couple whole nodes, so every row of
//    nodes shares one column list.  Per node row i: m_i block columns (int32,
//    local ghosted node index) and R*C value streams laid out [a][b][k]
//    (structure of arrays inside the row), so lane k of a wavefront reads
//    value (a,b) of block k with unit stride: every load instruction is a
//    fully coalesced 512-byte sweep and the column index costs 4/(R*C)
//    bytes per value instead of 4.  Values keep PETSc's pattern (explicit
//    zeros included), only the index storage is shared.
//  * scalar CSR ("aij"): MatSeqAIJ layout (int64 row pointers, int32
//    columns), used by the generic petsc4py-style setValues/assemble path.
//
// SpMV = MatMult (MatMult_SeqAIJ / MatMult_MPIAIJ; kle_solver.py:35-41,
// base_problem.py:123-136): one 64-lane wavefront per node row (per scalar row
// for aij), matrix streams read with non-temporal loads so they do not evict
// the ghosted x vector from L2, shuffle reductions, optional fused dot(y, p)
// partials for the Krylov loop.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <atomic>
#include <map>
#include <string>
#include <thread>

#include "kle_internal.hpp"

namespace kle {

int g_nb_pad = 16;  // 128-B aligned row streams (profiles/r01/spmv_sweep_pad.jsonl)
int g_nb_layout = 1;  // chunked rows (profiles/r01/layout_ab.jsonl)

__device__ __forceinline__ double wsum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <class T>
__device__ __forceinline__ T ntload(const T *p)
{
    return __builtin_nontemporal_load(p);
}

constexpr int SPMV_BLOCK = 256;
constexpr int SPMV_WAVES = SPMV_BLOCK / 64;

// rows [a0, a0 + na) then [b0, b0 + nb): the whole matrix, or the interior /
// ghost-dependent split used to overlap the halo exchange (N > 1)
struct RowMap {
    int64_t a0, na, b0, nb;
};

// Logical row block of this workgroup.  Blocks b, b+8, ... share an XCD
// (round-robin dispatch, MI355X_MICROARCH.md): within each run of 8*ch
// blocks, XCD slot b%8 takes ch consecutive row blocks, so an XCD's L2 sees
// compact x footprints while all XCDs stay in the same region of the matrix
// (balance); the partial last run keeps the round-robin order.  ch = 0: plain
// round-robin.  ch = 16: config 2 802.7 -> 797.4 us per CG iteration, 1M-DoF
// unstructured 863.6 -> 853.5, 1/8 slab 90.1 -> 89.1 (one contiguous eighth
// per XCD: +4 % / +25 % slower from imbalance; profiles/r02/xcd_chunk_*.jsonl).
__device__ __forceinline__ int64_t xcd_block(int ch)
{
    int64_t blk = blockIdx.x;
    if (ch > 0) {
        const int64_t k = blk >> 3, xc = blk & 7, S = (int64_t)gridDim.x / (8 * ch);
        if (k < S * ch) {
            const int64_t sb = k / ch;
            blk = sb * 8 * ch + xc * ch + (k - sb * ch);
        }
    }
    return blk;
}

// Node-block SpMV: one 64-lane wavefront per node row, WV rows per
// workgroup, one block column per lane in flight, non-temporal value/column
// loads (read once; they must not evict the gathered x from L2), shuffle
// reduction of the R row sums.  Specialised on the value layout and on
// structured columns so no run-time branch costs registers (62 VGPRs at
// R = C = 3: occupancy 8).
// LAY 1: while the wave's 64 blocks lie inside the row's full 16-block chunks
// the RC value loads of a lane share one base address (immediate offsets of
// 128 B); the last, partial pass uses the packed-tail rule of vofs().
// STRUCT: the row's columns form a lattice box (K, Rw, operators on box
// meshes): the column of block k is computed from 8 B per row, no bcol stream.
// Variants measured and rejected in round 1 (lanes per row 32/16, two blocks
// per lane in flight, persistent grid, XCD-chunked and (x,y)-tiled row
// orders, rows-per-wave prefetch, buffer-descriptor cache policies, the dot
// fused into the epilogue): DESIGN.md §3; code in git history (a54a1e5^).
template <int R, int C, int LAY, bool STRUCT, int WV>
__global__ __launch_bounds__(64 * WV, (R * C <= 9 ? 8 : 4)) void k_nb_spmv(RowMap rm, const int *__restrict__ rowptr,
                                                        const int *__restrict__ rowcnt,
                                                        const int *__restrict__ rowbox, int lx, int lxy,
                                                        const int64_t *__restrict__ vptr,
                                                        const int *__restrict__ bcol,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x, double *__restrict__ y,
                                                        const int *__restrict__ istate, int xcd_chunk)
{
    // the solve has ended (reason word set): every kernel a no-op.  Loaded
    // with the row's descriptors and tested before its value loads.
    const int stop = istate ? istate[I_REASON] : 0;
    constexpr int RC = R * C;
    const int lane = threadIdx.x & 63;
    const int64_t blk = xcd_block(xcd_chunk);
    const int64_t r = blk * WV + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (r >= rm.na + rm.nb) return;
    const int64_t i = r < rm.na ? rm.a0 + r : rm.b0 + (r - rm.na);
    const int b0 = rowptr[i], mp = rowptr[i + 1] - b0, m = rowcnt ? rowcnt[i] : mp;
    const double *v = val + vptr[i];
    if (stop) return;
    int bbase = 0, bnx = 1, bnxy = 1;
    if constexpr (STRUCT) {
        bbase = rowbox[2 * i];
        const int d = rowbox[2 * i + 1];
        bnx = d & 255;
        bnxy = bnx * ((d >> 8) & 255);
    }
    const int q16 = LAY == 1 ? (m & ~15) : 0;
    // one pass: the values of block kb + lane and the x entries they multiply
    auto load = [&](int kb, double *vv, double *xv) {
        const int k = kb + lane;
        const bool on = k < m;
        int j = 0;
        if (on) {
            if constexpr (STRUCT) {
                const int kz = k / bnxy, rem = k - kz * bnxy, ky = rem / bnx, kx = rem - ky * bnx;
                j = bbase + kx + lx * ky + lxy * kz;
            } else {
                j = __builtin_nontemporal_load(bcol + b0 + k);
            }
        }
        if (LAY == 1 && kb + 64 <= q16) {
            // whole wave inside full chunks: stream t at +16 t doubles
            const double *p = v + (k >> 4) * (RC * 16) + (k & 15);
#pragma unroll
            for (int t = 0; t < RC; ++t) vv[t] = __builtin_nontemporal_load(p + t * 16);
        } else if (on) {
            const int64_t o0 = vofs(LAY, RC, 0, k, m, mp);
            const int64_t st = LAY == 1 ? (k < q16 ? 16 : m - q16) : mp;
#pragma unroll
            for (int t = 0; t < RC; ++t) vv[t] = __builtin_nontemporal_load(v + o0 + t * st);
        } else {
#pragma unroll
            for (int t = 0; t < RC; ++t) vv[t] = 0.0;
        }
#pragma unroll
        for (int b = 0; b < C; ++b) xv[b] = on ? x[(int64_t)j * C + b] : 0.0;
    };
    double acc[R];
#pragma unroll
    for (int a = 0; a < R; ++a) acc[a] = 0.0;
    {
        for (int kb = 0; kb < m; kb += 64) {
            double vv[RC], xv[C];
            load(kb, vv, xv);
#pragma unroll
            for (int a = 0; a < R; ++a)
#pragma unroll
                for (int b = 0; b < C; ++b) acc[a] += vv[a * C + b] * xv[b];
        }
    }
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc[a] += __shfl_xor(acc[a], o, 64);
    if (lane < R) {
        double mine = acc[0];
#pragma unroll
        for (int a = 1; a < R; ++a)
            if (lane == a) mine = acc[a];
        y[i * R + lane] = mine;
    }
}


// Node-block SpMV with x staged in LDS (3x3 chunked structured rows, the
// box-mesh K): the WV consecutive rows of a workgroup read nearly the same x
// columns (their lattice boxes are shifted copies), so the workgroup loads
// the union of its rows' boxes once -- coalesced x-line segments -- and every
// wave reads its x entries from LDS instead of gathering them through the
// L1/L2 (3 gathers per block).  A workgroup whose union exceeds XL_CAP nodes
// or 21 nodes along x (its rows wrap into the next lattice line, or straddle
// the two RowMap ranges) gathers from global memory as before.  Row indices
// are read-first-lane scalars, so the row set-up runs on the scalar unit.
// Same products in the same order as k_nb_spmv: bitwise identical.
// Config 2: 0.730 -> 0.708 ms per SpMV, 736.5 -> 716.5 us per CG iteration;
// a variant with two union boxes for wrapping workgroups and one that loads
// the first value pass before the fill were slower (profiles/r02/xl_*.jsonl,
// cg_xl_*.jsonl).
constexpr int XL_CAP = 16 * 9 * 9;
template <int WV>
__global__ __launch_bounds__(64 * WV, 8) void k_nb_spmv_xl(RowMap rm, const int *__restrict__ rowptr,
                                                          const int *__restrict__ rowcnt,
                                                          const int *__restrict__ rowbox, int lx, int lxy,
                                                          const int64_t *__restrict__ vptr,
                                                          const double *__restrict__ val,
                                                          const double *__restrict__ x, double *__restrict__ y,
                                                          const int *__restrict__ istate, int xcd_chunk)
{
    constexpr int R = 3, C = 3, RC = 9;
    extern __shared__ double xs[];
    __shared__ int ub[WV][6];
    // the solve has ended (reason word set): every kernel a no-op.  Loaded
    // with the row's descriptors and tested before its value loads.
    const int stop = istate ? istate[I_REASON] : 0;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t blk = xcd_block(xcd_chunk);
    const int64_t nr = rm.na + rm.nb;
    const int64_t r = blk * WV + w;
    const bool live = r < nr;
    const int64_t i = !live ? 0 : (r < rm.na ? rm.a0 + r : rm.b0 + (r - rm.na));
    int m = 0, mp = 0, bbase = 0, bnx = 1, bny = 1, bnz = 1;
    const double *v = val;
    if (live) {
        const int b0 = rowptr[i];
        mp = rowptr[i + 1] - b0;
        m = rowcnt ? rowcnt[i] : mp;
        v = val + vptr[i];
        bbase = rowbox[2 * i];
        const int d = rowbox[2 * i + 1];
        bnx = d & 255;
        bny = (d >> 8) & 255;
        bnz = (d >> 16) & 255;
    }
    if (stop) return;  // (uniform: whole workgroup)
    const int cz = bbase / lxy, cy = (bbase - cz * lxy) / lx, cx = bbase - cz * lxy - cy * lx;
    if (lane == 0) {
        ub[w][0] = live ? cx : INT_MAX;
        ub[w][1] = live ? cy : INT_MAX;
        ub[w][2] = live ? cz : INT_MAX;
        ub[w][3] = live ? cx + bnx : INT_MIN;
        ub[w][4] = live ? cy + bny : INT_MIN;
        ub[w][5] = live ? cz + bnz : INT_MIN;
    }
    const int bnxy = bnx * bny;
    const int q16 = m & ~15;
    auto loadv = [&](int kb, double *vv) {
        const int k = kb + lane;
        if (kb + 64 <= q16) {
            const double *p = v + (k >> 4) * (RC * 16) + (k & 15);
#pragma unroll
            for (int t = 0; t < RC; ++t) vv[t] = __builtin_nontemporal_load(p + t * 16);
        } else if (k < m) {
            const int64_t o0 = vofs(1, RC, 0, k, m, mp);
            const int64_t st = k < q16 ? 16 : m - q16;
#pragma unroll
            for (int t = 0; t < RC; ++t) vv[t] = __builtin_nontemporal_load(v + o0 + t * st);
        } else {
#pragma unroll
            for (int t = 0; t < RC; ++t) vv[t] = 0.0;
        }
    };
    __syncthreads();
    int ox = INT_MAX, oy = INT_MAX, oz = INT_MAX, ex = INT_MIN, ey = INT_MIN, ez = INT_MIN;
#pragma unroll
    for (int q = 0; q < WV; ++q) {
        ox = min(ox, ub[q][0]);
        oy = min(oy, ub[q][1]);
        oz = min(oz, ub[q][2]);
        ex = max(ex, ub[q][3]);
        ey = max(ey, ub[q][4]);
        ez = max(ez, ub[q][5]);
    }
    ox = __builtin_amdgcn_readfirstlane(ox);
    oy = __builtin_amdgcn_readfirstlane(oy);
    oz = __builtin_amdgcn_readfirstlane(oz);
    ex = __builtin_amdgcn_readfirstlane(ex);
    ey = __builtin_amdgcn_readfirstlane(ey);
    ez = __builtin_amdgcn_readfirstlane(ez);
    const int UX = ex - ox, UY = ey - oy, UZ = ez - oz;
    const bool lds_x = (int64_t)UX * UY * UZ <= XL_CAP && UX * 3 <= 64;
    if (lds_x) {
        for (int seg = w; seg < UY * UZ; seg += WV) {
            const int uz = seg / UY, uy = seg - uz * UY;
            if (lane < UX * 3)
                xs[seg * UX * 3 + lane] = x[(int64_t)(ox + lx * (oy + uy) + lxy * (oz + uz)) * 3 + lane];
        }
    }
    __syncthreads();
    if (!live) return;
    double acc[R] = {0.0, 0.0, 0.0};
    auto rowloop = [&](auto xat) {
        for (int kb = 0; kb < m; kb += 64) {
            double vv[RC];
            loadv(kb, vv);
            const int k = kb + lane;
            if (k < m) {
                const int kz = k / bnxy, rem = k - kz * bnxy, ky = rem / bnx, kx = rem - ky * bnx;
#pragma unroll
                for (int a = 0; a < R; ++a)
#pragma unroll
                    for (int b = 0; b < C; ++b) acc[a] += vv[a * C + b] * xat(kx, ky, kz, b);
            }
        }
    };
    if (lds_x) {
        const int sy = UX * 3, sz = UX * UY * 3;
        const double *xl = xs + (cx - ox) * 3 + sy * (cy - oy) + sz * (cz - oz);
        rowloop([&](int kx, int ky, int kz, int b) { return xl[kx * 3 + sy * ky + sz * kz + b]; });
    } else {
        const double *xg = x + (int64_t)bbase * 3;
        rowloop([&](int kx, int ky, int kz, int b) { return xg[(int64_t)(kx + lx * ky + lxy * kz) * 3 + b]; });
    }
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc[a] += __shfl_xor(acc[a], o, 64);
    if (lane < R) {
        double mine = acc[0];
#pragma unroll
        for (int a = 1; a < R; ++a)
            if (lane == a) mine = acc[a];
        y[i * R + lane] = mine;
    }
}


// Node-block SpMV through per-group column dictionaries (unstructured 3x3
// chunked rows, 8 waves): the DICT_GROUP consecutive rows of a workgroup share
// most of their columns (union = 25 % of their blocks on the 1M-DoF Gmsh
// mesh, at most 1,053 nodes), so the workgroup gathers its group's distinct
// x nodes into LDS once (sorted node ids: 24-B records, mostly adjacent) and
// every block reads x from LDS through a 2-byte dictionary position instead
// of a 4-byte column (the bcol stream is not read).  Groups are aligned to
// DICT_GROUP rows in local row numbering; a RowMap range covers the groups
// that intersect it (waves outside the range idle), so the N > 1 split
// (interior rows, then ghost-dependent rows) reuses the same dictionaries.  A
// group whose dictionary exceeds DICT_CAP nodes reads x through it from
// global memory.  Same products in the same order as k_nb_spmv: bitwise
// identical.  xlo / xhi: the ext node range the fill may read -- the interior
// launch of an overlapped N > 1 SpMV passes the owned range, so no workgroup
// reads a ghost x entry while the comm stream is receiving it (the group's
// masked rows outside the range would not have used it; those slots read 0).
constexpr int DICT_GROUP = 8;
constexpr int DICT_CAP = 16 * 9 * 9;
__global__ __launch_bounds__(64 * DICT_GROUP, 8) void k_nb_spmv_dict(
    RowMap rm, int64_t ga0, int64_t nga, int64_t gb0, int64_t ngb, const int *__restrict__ rowptr,
    const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr, const uint16_t *__restrict__ lid,
    const int *__restrict__ dptr, const int *__restrict__ dict, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, const int *__restrict__ istate, int xcd_chunk, int64_t xlo,
    int64_t xhi)
{
    constexpr int R = 3, C = 3, RC = 9;
    extern __shared__ double xs[];
    // the solve has ended (reason word set): every kernel a no-op.  Loaded
    // with the row's descriptors and tested before its value loads.
    const int stop = istate ? istate[I_REASON] : 0;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t blk = xcd_block(xcd_chunk);
    if (blk >= nga + ngb) return;  // whole workgroup
    const bool in_a = blk < nga;
    const int64_t g = in_a ? ga0 + blk : gb0 + (blk - nga);
    const int64_t lo = in_a ? rm.a0 : rm.b0, hi = in_a ? rm.a0 + rm.na : rm.b0 + rm.nb;
    const int64_t i = g * DICT_GROUP + w;
    const bool live = i >= lo && i < hi;
    const int d0 = dptr[g], U = dptr[g + 1] - d0;
    if (stop) return;  // (uniform: whole workgroup)
    const bool lds_x = U <= DICT_CAP;
    if (lds_x)
        for (int t = threadIdx.x; t < 3 * U; t += 64 * DICT_GROUP) {
            const int e = t / 3;
            const int64_t node = dict[d0 + e];
            xs[t] = node >= xlo && node < xhi ? x[node * 3 + (t - 3 * e)] : 0.0;
        }
    __syncthreads();
    if (!live) return;
    const int b0 = rowptr[i], mp = rowptr[i + 1] - b0, m = rowcnt ? rowcnt[i] : mp;
    const double *v = val + vptr[i];
    const uint16_t *lrow = lid + b0;
    const int q16 = m & ~15;
    double acc[R] = {0.0, 0.0, 0.0};
    auto rowloop = [&](auto xat) {
        for (int kb = 0; kb < m; kb += 64) {
            const int k = kb + lane;
            double vv[RC];
            if (kb + 64 <= q16) {
                const double *p = v + (k >> 4) * (RC * 16) + (k & 15);
#pragma unroll
                for (int t = 0; t < RC; ++t) vv[t] = __builtin_nontemporal_load(p + t * 16);
            } else if (k < m) {
                const int64_t o0 = vofs(1, RC, 0, k, m, mp);
                const int64_t st = k < q16 ? 16 : m - q16;
#pragma unroll
                for (int t = 0; t < RC; ++t) vv[t] = __builtin_nontemporal_load(v + o0 + t * st);
            }
            if (k < m) {
                const int l = __builtin_nontemporal_load(lrow + k);
#pragma unroll
                for (int a = 0; a < R; ++a)
#pragma unroll
                    for (int b = 0; b < C; ++b) acc[a] += vv[a * C + b] * xat(l, b);
            }
        }
    };
    if (lds_x) rowloop([&](int l, int b) { return xs[l * 3 + b]; });
    else rowloop([&](int l, int b) { return x[(int64_t)dict[d0 + l] * 3 + b]; });
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc[a] += __shfl_xor(acc[a], o, 64);
    if (lane < R) {
        double mine = acc[0];
#pragma unroll
        for (int a = 1; a < R; ++a)
            if (lane == a) mine = acc[a];
        y[i * R + lane] = mine;
    }
}

// Scalar CSR SpMV (MatMult_SeqAIJ): one wavefront per row.  A pass covers
// 64*U entries from the row start rounded down to 32 entries, so every col
// load (32 int32 = 128 B) and every val load (16 doubles = 128 B) covers whole
// cache lines instead of straddling the neighbouring row's, and U independent
// (col, val) load pairs per lane are in flight before the dependent x gathers
// (one pair per pass leaves the wave latency bound).  Lanes outside [s, e)
// load nothing and add nothing.
template <int U, int WV>
__global__ __launch_bounds__(64 * WV) void k_aij_spmv(int64_t nrows, const int64_t *__restrict__ ptr,
                                                      const int *__restrict__ col,
                                                      const double *__restrict__ val,
                                                      const double *__restrict__ x, double *__restrict__ y,
                                                      const int *__restrict__ istate, int xcd_chunk)
{
    // the solve has ended (reason word set): every kernel a no-op.  Loaded
    // with the row's descriptors and tested before its value loads.
    const int stop = istate ? istate[I_REASON] : 0;
    const int lane = threadIdx.x & 63;
    const int64_t i = xcd_block(xcd_chunk) * WV + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (i >= nrows) return;
    const int64_t s = ptr[i], e = ptr[i + 1];
    if (stop) return;
    double acc = 0.0;
    for (int64_t k0 = s & ~(int64_t)31; k0 < e; k0 += 64 * U) {
        int c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = k0 + u * 64 + lane;
            const bool on = k >= s && k < e;
            c[u] = on ? ntload(col + k) : -1;
            v[u] = on ? ntload(val + k) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (c[u] >= 0) acc += v[u] * x[c[u]];
    }
    acc = wsum(acc);
    if (lane == 0) y[i] = acc;
}

// diagonal position of each node row (for Jacobi / get_diagonal)
__global__ void k_diagpos(int64_t nrows, int64_t row_off, const int *__restrict__ rowptr,
                          const int *__restrict__ rowcnt, const int *__restrict__ bcol, int *__restrict__ pos)
{
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    int lo = rowptr[i], hi = lo + (rowcnt ? rowcnt[i] : rowptr[i + 1] - lo) - 1, want = (int)(i + row_off), found = -1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        int c = bcol[mid];
        if (c == want) {
            found = mid;
            break;
        }
        if (c < want) lo = mid + 1;
        else hi = mid - 1;
    }
    pos[i] = found < 0 ? -1 : found - rowptr[i];
}

template <int R, int C>
__global__ void k_nb_scale(int64_t nrows, const int *__restrict__ rowptr, const int *__restrict__ rowcnt,
                           const int64_t *__restrict__ vptr, int lay, const int *__restrict__ bcol,
                           double *__restrict__ val, const double *__restrict__ L, const double *__restrict__ Rx)
{
    const int lane = threadIdx.x & 63;
    const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (i >= nrows) return;
    const int b0 = rowptr[i], mp = rowptr[i + 1] - b0, m = rowcnt ? rowcnt[i] : mp;
    double *v = val + vptr[i];
    for (int k = lane; k < m; k += 64) {
        const int64_t j = bcol[b0 + k];
        for (int a = 0; a < R; ++a)
            for (int b = 0; b < C; ++b) {
                double s = 1.0;
                if (L) s *= L[i * R + a];
                if (Rx) s *= Rx[j * C + b];
                v[vofs(lay, R * C, a * C + b, k, m, mp)] *= s;
            }
    }
}

__global__ void k_nb_diag(int64_t nrows, int R, int C, const int *__restrict__ rowptr,
                          const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr, int lay,
                          const int *__restrict__ pos, const double *__restrict__ val, double *__restrict__ d)
{
    int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= nrows * R) return;
    int64_t i = t / R;
    int a = (int)(t % R);
    const int b0 = rowptr[i], mp = rowptr[i + 1] - b0, m = rowcnt ? rowcnt[i] : mp;
    d[t] = pos[i] < 0 ? 0.0 : val[vptr[i] + vofs(lay, R * C, a * C + a, pos[i], m, mp)];
}

__global__ void k_aij_scale(int64_t nrows, const int64_t *__restrict__ ptr, const int *__restrict__ col,
                            double *__restrict__ val, const double *__restrict__ L,
                            const double *__restrict__ Rx)
{
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
        double s = 1.0;
        if (L) s *= L[i];
        if (Rx) s *= Rx[col[k]];
        val[k] *= s;
    }
}

__global__ void k_aij_diag(int64_t nrows, int64_t col_off, const int64_t *__restrict__ ptr,
                           const int *__restrict__ col, const double *__restrict__ val, double *__restrict__ d)
{
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    double v = 0.0;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
        if (col[k] == i + col_off) v = val[k];
    d[i] = v;
}

__global__ void k_axpy_same(int64_t n, double a, const double *__restrict__ x, double *__restrict__ y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] += a * x[i];
}

// Column dictionaries of an unstructured node-block matrix (k_nb_spmv_dict):
// built on the host from the device pattern, groups split over threads.
int nb_build_dict(kle_mat *A)
{
    const int64_t nrows = A->nrows, ng = (nrows + DICT_GROUP - 1) / DICT_GROUP;
    std::vector<int> rp(nrows + 1), cnt, bcol(std::max<int64_t>(A->nblocks, 1));
    KLE_HIP(hipMemcpy(rp.data(), A->d_rowptr, sizeof(int) * (nrows + 1), hipMemcpyDeviceToHost));
    if (A->d_rowcnt) {
        cnt.resize(nrows);
        KLE_HIP(hipMemcpy(cnt.data(), A->d_rowcnt, sizeof(int) * nrows, hipMemcpyDeviceToHost));
    }
    KLE_HIP(hipMemcpy(bcol.data(), A->d_bcol, sizeof(int) * bcol.size(), hipMemcpyDeviceToHost));
    const int64_t ncol = A->ext_nodes;
    std::vector<int> dptr(ng + 1, 0);
    std::vector<uint16_t> lid(bcol.size(), 0);
    std::vector<int> dict;
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    auto rows_of = [&](int64_t g, int64_t &r0, int64_t &r1) {
        r0 = g * DICT_GROUP;
        r1 = std::min(nrows, r0 + DICT_GROUP);
    };
    auto len = [&](int64_t r) { return A->d_rowcnt ? cnt[r] : rp[r + 1] - rp[r]; };
    // pass 1: distinct columns per group
    std::vector<int> usz(ng, 0);
    std::atomic<bool> bad{false};
    auto pass1 = [&](int t) {
        std::vector<int> stamp(ncol, -1);
        for (int64_t g = t; g < ng; g += nt) {
            int64_t r0, r1;
            rows_of(g, r0, r1);
            int u = 0;
            for (int64_t r = r0; r < r1; ++r)
                for (int k = 0; k < len(r); ++k) {
                    const int c = bcol[rp[r] + k];
                    if (c < 0 || c >= ncol) { bad = true; continue; }
                    if (stamp[c] != (int)g) {
                        stamp[c] = (int)g;
                        ++u;
                    }
                }
            usz[g] = u;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(pass1, t);
        for (auto &x : th) x.join();
    }
    KLE_ARG(!bad, "column out of range in the node-block pattern");
    int64_t total = 0;
    for (int64_t g = 0; g < ng; ++g) {
        if (usz[g] > 65535) return 0;  // positions would not fit 16 bits: keep the column stream
        total += usz[g];
        if (total > INT_MAX) return 0;  // int32 dictionary offsets
        dptr[g + 1] = (int)total;
    }
    dict.resize(std::max(dptr[ng], 1));
    auto pass2 = [&](int t) {
        std::vector<int> pos(ncol, 0), list;
        for (int64_t g = t; g < ng; g += nt) {
            int64_t r0, r1;
            rows_of(g, r0, r1);
            list.clear();
            for (int64_t r = r0; r < r1; ++r)
                for (int k = 0; k < len(r); ++k) list.push_back(bcol[rp[r] + k]);
            std::sort(list.begin(), list.end());
            list.erase(std::unique(list.begin(), list.end()), list.end());
            for (size_t j = 0; j < list.size(); ++j) {
                pos[list[j]] = (int)j;
                dict[dptr[g] + j] = list[j];
            }
            for (int64_t r = r0; r < r1; ++r)
                for (int k = 0; k < len(r); ++k) lid[rp[r] + k] = (uint16_t)pos[bcol[rp[r] + k]];
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(pass2, t);
        for (auto &x : th) x.join();
    }
    A->dict_len = dptr[ng];
    if (hipMalloc(&A->d_dptr, sizeof(int) * (ng + 1)) != hipSuccess ||
        hipMalloc(&A->d_dict, sizeof(int) * dict.size()) != hipSuccess ||
        hipMalloc(&A->d_lid, sizeof(uint16_t) * lid.size()) != hipSuccess)
        return fail(KLE_ERR_MEM, "out of device memory for column dictionaries");
    KLE_TRY(h2d(A->d_dptr, dptr.data(), sizeof(int) * (ng + 1)));
    KLE_TRY(h2d(A->d_dict, dict.data(), sizeof(int) * dict.size()));
    KLE_TRY(h2d(A->d_lid, lid.data(), sizeof(uint16_t) * lid.size()));
    return 0;
}

bool spmv_uses_comm_stream(const kle_mat *A, const kle_vec *x)
{
    // (the symmetric SpMV's two halos run on the comm stream whatever the
    // slab's interior: sym_spmv; the graph symmetric SpMV's with overlap on:
    // gsym_spmv)
    if (A->kind == 0 && A->d_sval && g_tune.spmv_sym && A->sym_graph)
        return A->ctx->nranks > 1 && A->halo_overlap != 0;
    return A->kind == 0 && A->ctx->nranks > 1 && A->halo_overlap &&
           (A->int_lo < A->int_hi || (A->d_sval && g_tune.spmv_sym)) &&
           (x->lo_rank >= 0 || x->hi_rank >= 0 || (x->plan && !x->plan->peers.empty()));
}

// Waves (rows) per workgroup: 8 for 3x3 chunked matrices of >= 64k node rows
// -- consecutive rows of one workgroup share most x columns in the CU's L1:
// config 2 +2.5 %, unstructured 1M mesh +2 %; 4 elsewhere (0.5 % ahead on the
// 1/8 slab); profiles/r01/spmv_waves_ab.jsonl.  With 8 waves, structured rows
// run k_nb_spmv_xl (x in LDS).  Below 64k rows 4 plain waves stay: alone the
// 8-wave LDS kernel is faster on the 1/8 slab (71.3 vs 73.4 us), inside the
// pipelined CG loop 1 % slower (79.6 vs 78.7 us per iteration,
// profiles/r02/cg_xl_eighth.jsonl).  kle_set_tuning("spmv_waves") overrides.
static int spmv_waves(const kle_mat *A)
{
    if (!(A->R == 3 && A->C == 3 && A->vlayout == 1)) return SPMV_WAVES;
    return g_tune.spmv_waves ? g_tune.spmv_waves : (A->nrows >= 64000 ? 8 : SPMV_WAVES);
}

template <int R, int C, int LAY, bool STRUCT>
static void launch_nb_lay(const kle_mat *A, RowMap rm, int wv, const int *rbox, const kle_vec *x, kle_vec *y,
                          const int *istate, hipStream_t st)
{
    const int64_t nr = rm.na + rm.nb;
    // While comm-stream kernels (halo, reductions, allreduce; N > 1 overlap)
    // run beside this SpMV, 4-wave workgroups reserve 21 KB of (unused) LDS:
    // 7 instead of 8 fit per CU, so the side kernels find room at once instead
    // of waiting for the SpMV grid to drain.  Measured on one GPU with a
    // reduction beside the SpMV of a 1/8 slab: 93.4 -> 90.7 us per iteration,
    // the capped SpMV itself no slower (profiles/r02/lds_cap_*.jsonl).
    // kle_set_tuning("spmv_dyn_lds") overrides.
    const size_t lds = g_tune.spmv_dyn_lds >= 0 ? (size_t)g_tune.spmv_dyn_lds
                                                 : (A->ctx->side_busy && wv != 8 ? 21504 : 0);
    // x in LDS where 8 rows' union box fits XL_CAP (p <= 4: 16 x 9 x 9 nodes)
    const bool xl = R == 3 && C == 3 && LAY == 1 && STRUCT && wv == 8 && g_tune.spmv_x_lds &&
                    (7 + A->box_max) * A->box_max * A->box_max <= XL_CAP;
    if (xl) {
        hipLaunchKernelGGL((k_nb_spmv_xl<8>), dim3(grid_for(nr, 8, 1 << 30)), dim3(512),
                           lds + XL_CAP * 3 * sizeof(double), st, rm, A->d_rowptr, A->d_rowcnt, rbox,
                           (int)A->box_lx, (int)A->box_lxy, A->d_vptr, A->d_val, x->base, y->d, istate,
                           g_tune.spmv_xcd_chunk);
    } else if (R == 3 && C == 3 && LAY == 1 && !STRUCT && wv == 8 && A->d_lid && g_tune.spmv_dict) {
        // dictionary groups intersecting each RowMap range
        auto groups = [](int64_t a0, int64_t na, int64_t &g0, int64_t &ng) {
            g0 = a0 / DICT_GROUP;
            ng = na > 0 ? (a0 + na + DICT_GROUP - 1) / DICT_GROUP - g0 : 0;
        };
        int64_t ga0, nga, gb0, ngb;
        groups(rm.a0, rm.na, ga0, nga);
        groups(rm.b0, rm.nb, gb0, ngb);
        // rows [int_lo, int_hi) read no ghost column: their launch reads owned x only
        const bool own_only = rm.nb == 0 && rm.a0 >= A->int_lo && rm.a0 + rm.na <= A->int_hi;
        const int64_t xlo = own_only ? A->ghost_lo / C : 0, xhi = own_only ? xlo + A->n_local / C : INT64_MAX;
        hipLaunchKernelGGL(k_nb_spmv_dict, dim3((unsigned)(nga + ngb)), dim3(64 * DICT_GROUP),
                           lds + DICT_CAP * 3 * sizeof(double), st, rm, ga0, nga, gb0, ngb, A->d_rowptr, A->d_rowcnt,
                           A->d_vptr, A->d_lid, A->d_dptr, A->d_dict, A->d_val, x->base, y->d, istate,
                           g_tune.spmv_xcd_chunk, xlo, xhi);
    } else if (R == 3 && C == 3 && LAY == 1 && wv == 8)
        hipLaunchKernelGGL((k_nb_spmv<R, C, LAY, STRUCT, 8>), dim3(grid_for(nr, 8, 1 << 30)), dim3(512), lds, st, rm,
                           A->d_rowptr, A->d_rowcnt, rbox, (int)A->box_lx, (int)A->box_lxy, A->d_vptr, A->d_bcol,
                           A->d_val, x->base, y->d, istate, g_tune.spmv_xcd_chunk);
    else
        hipLaunchKernelGGL((k_nb_spmv<R, C, LAY, STRUCT, SPMV_WAVES>), dim3(grid_for(nr, SPMV_WAVES, 1 << 30)),
                           dim3(SPMV_BLOCK), lds, st, rm, A->d_rowptr, A->d_rowcnt, rbox, (int)A->box_lx,
                           (int)A->box_lxy, A->d_vptr, A->d_bcol, A->d_val, x->base, y->d, istate,
                           g_tune.spmv_xcd_chunk);
}

template <int R, int C>
static void launch_nb(const kle_mat *A, RowMap rm, const int *rbox, const kle_vec *x, kle_vec *y,
                      const int *istate, hipStream_t st)
{
    if (rm.na + rm.nb <= 0) return;
    const int wv = spmv_waves(A);
    if (A->vlayout == 1) {
        if (rbox) launch_nb_lay<R, C, 1, true>(A, rm, wv, rbox, x, y, istate, st);
        else launch_nb_lay<R, C, 1, false>(A, rm, wv, rbox, x, y, istate, st);
    } else {
        if (rbox) launch_nb_lay<R, C, 0, true>(A, rm, wv, rbox, x, y, istate, st);
        else launch_nb_lay<R, C, 0, false>(A, rm, wv, rbox, x, y, istate, st);
    }
}

static int launch_nb_shape(const kle_mat *A, RowMap rm, const int *rbox, const kle_vec *x, kle_vec *y,
                           const int *istate, hipStream_t st)
{
#define NB_SHAPE(RR, CC)                                                  \
    if (A->R == RR && A->C == CC) {                                       \
        launch_nb<RR, CC>(A, rm, rbox, x, y, istate, st);                 \
        KLE_HIP(hipGetLastError());                                       \
        return 0;                                                         \
    }
    NB_SHAPE(3, 3) NB_SHAPE(6, 3) NB_SHAPE(3, 6) NB_SHAPE(2, 2) NB_SHAPE(2, 1) NB_SHAPE(1, 2) NB_SHAPE(3, 1)
    NB_SHAPE(1, 3) NB_SHAPE(3, 2) NB_SHAPE(2, 3) NB_SHAPE(1, 1)
#undef NB_SHAPE
    return fail(KLE_ERR_SUP, "no SpMV kernel for %dx%d blocks", A->R, A->C);
}

// Whether A's product runs the box bricks, whose owned rows' gather a
// consumer may take over (spmv_split; k_pipe_iter_g)
bool spmv_can_split(const kle_mat *A)
{
    return A->kind == 0 && A->d_sval && g_tune.spmv_sym && A->sym_brick && !A->sym_graph && A->nbricks > 0;
}

// y = A x without the owned rows' gather and the received reverse-halo sums
// (kle_brick.hip brick_spmv split): the consumer adds them (BrickGather), or
// brick_gather_rest does.  Only where spmv_can_split.
int spmv_split(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart)
{
    KLE_ARG(spmv_can_split(A), "split product: not a box-brick matrix");
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(A->ctx->tic("spmv", &ev));
    KLE_TRY(brick_spmv(A, x, y, istate, dpart, true));
    KLE_TRY(A->ctx->toc("spmv", &ev));
    return 0;
}

int spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate)
{
    kle_ctx *c = A->ctx;
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (A->kind == 0 && A->d_sval && g_tune.spmv_sym) {
        // symmetric storage (both halos of N > 1 inside)
        KLE_TRY(c->tic("spmv", &ev));
        KLE_TRY(sym_spmv(A, x, y, istate));
        KLE_TRY(c->toc("spmv", &ev));
        return 0;
    }
    if (A->kind == 0) {
        // N > 1: rows [int_lo, int_hi) read no ghost entry, so they run while the
        // halo is in flight on the comm stream; the ghost-dependent rows follow
        const bool overlap = spmv_uses_comm_stream(A, x);
        if (c->nranks > 1 && !overlap)
            KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank,
                                  x->send_lo, x->send_hi, nullptr, x->plan.get()));
        KLE_TRY(c->tic("spmv", &ev));
        const int *rbox = A->spmv_struct ? A->d_rowbox : nullptr;
        if (!overlap) {
            KLE_TRY(launch_nb_shape(A, RowMap{0, A->nrows, 0, 0}, rbox, x, y, istate, c->stream));
        } else {
            SideBusy busy(c);  // the halo (and, in pipecg, the reduction) run beside both launches
            KLE_HIP(hipEventRecord(c->ev_x_ready, c->stream));
            KLE_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_x_ready, 0));
            KLE_TRY(launch_nb_shape(A, RowMap{A->int_lo, A->int_hi - A->int_lo, 0, 0}, rbox, x, y, istate,
                                    c->stream));
            // interior rows are queued; exchange the halo beside them
            KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank,
                                  x->send_lo, x->send_hi, c->comm_stream, x->plan.get()));
            KLE_HIP(hipEventRecord(c->ev_halo_done, c->comm_stream));
            KLE_HIP(hipStreamWaitEvent(c->stream, c->ev_halo_done, 0));
            KLE_TRY(launch_nb_shape(A, RowMap{0, A->int_lo, A->int_hi, A->nrows - A->int_hi}, rbox, x, y, istate,
                                    c->stream));
        }
        KLE_TRY(c->toc("spmv", &ev));
        return 0;
    }
    // 8 load pairs in flight per lane, 4 rows per workgroup: 5.50 TB/s at config 2
    // vs 5.45 (16 pairs), 5.45 (8 rows per workgroup), 4.94 (4 pairs), 3.99 TB/s
    // (1 pair): profiles/r02/aij_ab_*.jsonl
    KLE_TRY(c->tic("spmv", &ev));
    hipLaunchKernelGGL((k_aij_spmv<8, 4>), dim3(grid_for(A->m_local, 4, 1 << 30)), dim3(256), 0, c->stream,
                       A->m_local, A->d_aptr, A->d_acol, A->d_aval, x->d, y->d, istate, g_tune.spmv_xcd_chunk);
    KLE_HIP(hipGetLastError());
    KLE_TRY(c->toc("spmv", &ev));
    return 0;
}

int spmv_dot_parts(const kle_mat *A)
{
    return A->kind == 0 && A->d_sval && g_tune.spmv_sym ? sym_dot_parts(A) : 0;
}

int spmv_dot(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart, int *nparts)
{
    *nparts = spmv_dot_parts(A);
    if (!*nparts) return spmv(A, x, y, istate);
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(A->ctx->tic("spmv", &ev));
    KLE_TRY(sym_spmv(A, x, y, istate, dpart));
    KLE_TRY(A->ctx->toc("spmv", &ev));
    return 0;
}

static int check_mult_layout(const kle_mat *A, const kle_vec *x, const kle_vec *y)
{
    if (A->kind == 0) {
        if (x->n_local != A->n_local || x->ghost_lo != A->ghost_lo || x->ghost_hi != A->ghost_hi)
            return fail(KLE_ERR_SIZ, "x layout does not match the matrix column space "
                                     "(need a mesh vector with bs=%d)", A->C);
    } else if (x->n_local != A->n_local) {
        return fail(KLE_ERR_SIZ, "x has %lld local entries, matrix has %lld columns", (long long)x->n_local,
                    (long long)A->n_local);
    }
    if (y->n_local != A->m_local)
        return fail(KLE_ERR_SIZ, "y has %lld local entries, matrix has %lld rows", (long long)y->n_local,
                    (long long)A->m_local);
    return 0;
}

// host copy of an nb matrix
// Does PETSc hold entry (row node i (owned-local), comp a) x (col node jl
// (ext-local), comp b)?  No-slip matrices keep DoF-level patterns.
static bool nb_entry_exists(const kle_mat *A, int64_t i, int a, int64_t jl, int b)
{
    if (A->mask_rule == MASK_NONE) return true;
    const int64_t il = A->node_begin - A->ext_begin + i;
    const int rc = A->dof_cls[il * A->R + a];
    const int cc = A->mask_rule == MASK_TANG_ROWS ? DOF_FREE : A->dof_cls[jl * A->C + b];
    return mask_entry(A->mask_rule, rc, cc, jl == il && a == b);
}

struct NBHost {
    std::vector<int> rp, bc, cnt;
    std::vector<int64_t> vp;
    std::vector<double> v;
    // entry t of block k in row i
    double at(const kle_mat *A, int64_t i, int t, int k) const
    {
        return v[vp[i] + vofs(A->vlayout, A->R * A->C, t, k, cnt[i], rp[i + 1] - rp[i])];
    }
};

static int nb_download(const kle_mat *A, NBHost &h)
{
    h.rp.resize(A->nrows + 1);
    h.bc.resize(std::max<int64_t>(A->nblocks, 1));
    h.v.resize(std::max<int64_t>(A->nvals, 1));
    h.vp.resize(A->nrows + 1);
    KLE_HIP(hipMemcpy(h.vp.data(), A->d_vptr, sizeof(int64_t) * (A->nrows + 1), hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(h.rp.data(), A->d_rowptr, sizeof(int) * (A->nrows + 1), hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(h.bc.data(), A->d_bcol, sizeof(int) * h.bc.size(), hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(h.v.data(), A->d_val, sizeof(double) * h.v.size(), hipMemcpyDeviceToHost));
    h.cnt.resize(A->nrows);
    if (A->d_rowcnt) KLE_HIP(hipMemcpy(h.cnt.data(), A->d_rowcnt, sizeof(int) * A->nrows, hipMemcpyDeviceToHost));
    else
        for (int64_t i = 0; i < A->nrows; ++i) h.cnt[i] = h.rp[i + 1] - h.rp[i];
    return 0;
}

static int aij_upload(kle_mat *A)
{
    kle_ctx *c = A->ctx;
    hipFree(A->d_aptr);
    hipFree(A->d_acol);
    hipFree(A->d_aval);
    A->d_aptr = nullptr;
    A->d_acol = nullptr;
    A->d_aval = nullptr;
    A->nnz = A->h_ptr.back();
    std::vector<int> c32(std::max<int64_t>(A->nnz, 1));
    for (int64_t k = 0; k < A->nnz; ++k) c32[k] = (int)(A->h_col[k] - A->col_lo);
    KLE_HIP(hipMalloc(&A->d_aptr, sizeof(int64_t) * A->h_ptr.size()));
    KLE_HIP(hipMalloc(&A->d_acol, sizeof(int) * c32.size()));
    if (big_alloc(reinterpret_cast<void **>(&A->d_aval), sizeof(double) * std::max<int64_t>(A->nnz, 1)) < 0)
        return fail(KLE_ERR_MEM, "out of device memory for the AIJ values");
    KLE_HIP(hipMemcpyAsync(A->d_aptr, A->h_ptr.data(), sizeof(int64_t) * A->h_ptr.size(), hipMemcpyHostToDevice, c->stream));
    KLE_HIP(hipMemcpyAsync(A->d_acol, c32.data(), sizeof(int) * c32.size(), hipMemcpyHostToDevice, c->stream));
    if (A->nnz)
        KLE_HIP(hipMemcpyAsync(A->d_aval, A->h_val.data(), sizeof(double) * A->nnz, hipMemcpyHostToDevice, c->stream));
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

}  // namespace kle

using namespace kle;

extern "C" {

int kle_mat_create_aij(kle_ctx *ctx, int64_t m_local, int64_t n_local, int64_t m_global, int64_t n_global,
                       const int32_t *d_nnz, const int32_t *o_nnz, kle_mat **out)
{
    KLE_ARG(ctx && out, "null arg");
    KLE_ARG(m_local >= 0 && n_local >= 0, "negative size");
    int64_t row_lo = 0, col_lo = 0;
    if (ctx->nranks > 1) {
        // a distributed generic AIJ is supported only without entries: the
        // preallocated-but-never-filled matrices of the reference (MatFS.Rd,
        // mat_fs.py:54-94) -- its product is zero and needs no halo
        bool empty = d_nnz != nullptr;
        for (int64_t r = 0; empty && r < m_local; ++r) empty = d_nnz[r] == 0 && (!o_nnz || o_nnz[r] == 0);
        if (!empty) return fail(KLE_ERR_SUP, "generic AIJ is single-rank; use kle_assemble_kle for MPI layouts");
        std::vector<int64_t> ms(ctx->nranks), ns(ctx->nranks);
        KLE_TRY(allgather_i64(ctx, m_local, ms));
        KLE_TRY(allgather_i64(ctx, n_local, ns));
        int64_t mt = 0, nt = 0;
        for (int r = 0; r < ctx->nranks; ++r) {
            if (r == ctx->rank) {
                row_lo = mt;
                col_lo = nt;
            }
            mt += ms[r];
            nt += ns[r];
        }
        if (m_global < 0) m_global = mt;
        if (n_global < 0) n_global = nt;
        KLE_ARG(m_global == mt && n_global == nt, "global sizes do not match the sum of local sizes");
    } else {
        if (m_global < 0) m_global = m_local;
        if (n_global < 0) n_global = n_local;
        KLE_ARG(m_global == m_local && n_global == n_local, "single rank: global size must equal local size");
    }
    kle_mat *A = new kle_mat;
    A->row_lo = row_lo;
    A->col_lo = col_lo;
    A->empty_only = ctx->nranks > 1;
    A->ctx = ctx;
    A->kind = 1;
    A->m_local = m_local;
    A->n_local = n_local;
    A->m_global = m_global;
    A->n_global = n_global;
    A->stash.resize(m_local);
    if (d_nnz) A->d_nnz_hint.assign(d_nnz, d_nnz + m_local);
    (void)o_nnz;
    *out = A;
    return 0;
}

int kle_mat_create_aij_csr(kle_ctx *ctx, int64_t m, int64_t n, const int64_t *indptr, const int64_t *indices,
                           const double *data, kle_mat **out)
{
    KLE_ARG(ctx && indptr && out, "null arg");
    KLE_ARG(indptr[0] == 0, "indptr[0] must be 0");
    for (int64_t r = 0; r < m; ++r) {
        KLE_ARG(indptr[r + 1] >= indptr[r], "indptr not monotone at row %lld", (long long)r);
        for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) {
            KLE_ARG(indices[k] >= 0 && indices[k] < n, "column %lld out of range", (long long)indices[k]);
            KLE_ARG(k == indptr[r] || indices[k] > indices[k - 1], "columns of row %lld not strictly ascending",
                    (long long)r);
        }
    }
    kle_mat *A;
    KLE_TRY(kle_mat_create_aij(ctx, m, n, m, n, nullptr, nullptr, &A));
    const int64_t z = indptr[m];
    A->h_ptr.assign(indptr, indptr + m + 1);
    A->h_col.assign(indices, indices + z);
    A->h_val.assign(data, data + z);
    A->assembled = true;
    A->stash.clear();
    int rc = aij_upload(A);
    if (rc) {
        kle_mat_destroy(A);
        return rc;
    }
    *out = A;
    return 0;
}

int kle_mat_set_values(kle_mat *A, int32_t nr, const int64_t *rows, int32_t nc, const int64_t *cols,
                       const double *v, int addv)
{
    if (A) sym_drop(A);
    KLE_ARG(A && rows && cols && v, "null arg");
    if (A->kind != 1) return fail(KLE_ERR_SUP, "setValues on a node-block matrix: assemble with kle_assemble_kle");
    for (int32_t r = 0; r < nr; ++r) {
        const int64_t row = rows[r] - A->row_lo;
        if (rows[r] < 0) continue;  // PETSc ignores negative indices
        if (row < 0 || row >= A->m_local)
            return fail(KLE_ERR_OUTOFRANGE, "row %lld out of range [0,%lld)", (long long)rows[r], (long long)A->m_local);
        for (int32_t c = 0; c < nc; ++c) {
            if (cols[c] < 0) continue;
            if (cols[c] >= A->n_global)
                return fail(KLE_ERR_OUTOFRANGE, "column %lld out of range", (long long)cols[c]);
            const double val = v[(int64_t)r * nc + c];
            if (A->empty_only)
                return fail(KLE_ERR_NEWNZ, "new nonzero at (%lld,%lld) caused a malloc (matrix preallocated empty)",
                            (long long)rows[r], (long long)cols[c]);
            if (!A->assembled) {
                A->stash[row].push_back({cols[c], val, addv ? 1 : 0});
            } else {
                auto b = A->h_col.begin() + A->h_ptr[row], e = A->h_col.begin() + A->h_ptr[row + 1];
                auto it = std::lower_bound(b, e, cols[c]);
                if (it == e || *it != cols[c])
                    return fail(KLE_ERR_NEWNZ, "new nonzero at (%lld,%lld) caused a malloc", (long long)rows[r],
                                (long long)cols[c]);
                double &slot = A->h_val[it - A->h_col.begin()];
                slot = addv ? slot + val : val;
                A->dirty = true;
            }
        }
    }
    return 0;
}

int kle_mat_assemble(kle_mat *A)
{
    if (A) sym_drop(A);
    KLE_ARG(A, "null mat");
    if (A->kind != 1) return 0;
    if (!A->assembled) {
        // build the pattern: entries in call order, ADD sums from 0 in that
        // order, INSERT overwrites (MatSetValues_SeqAIJ semantics)
        A->h_ptr.assign(A->m_local + 1, 0);
        A->h_col.clear();
        A->h_val.clear();
        for (int64_t r = 0; r < A->m_local; ++r) {
            std::map<int64_t, double> row;
            for (auto &en : A->stash[r]) {
                if (en.add) row[en.col] += en.v;
                else row[en.col] = en.v;
            }
            for (auto &kv : row) {
                A->h_col.push_back(kv.first);
                A->h_val.push_back(kv.second);
            }
            A->h_ptr[r + 1] = (int64_t)A->h_col.size();
            std::vector<kle_mat::StashEnt>().swap(A->stash[r]);
        }
        A->assembled = true;
        return aij_upload(A);
    }
    if (A->dirty) {
        KLE_TRY(h2d(A->d_aval, A->h_val.data(), sizeof(double) * A->nnz));
        A->dirty = false;
    }
    return 0;
}

int kle_mat_destroy(kle_mat *A)
{
    if (!A) return 0;
    hipFree(A->d_rowcnt);
    hipFree(A->d_rowbox);
    hipFree(A->d_vptr);
    hipFree(A->d_rowptr);
    hipFree(A->d_bcol);
    hipFree(A->d_dptr);
    hipFree(A->d_dict);
    hipFree(A->d_lid);
    hipFree(A->d_val);
    sym_drop(A);
    hipFree(A->d_aptr);
    hipFree(A->d_acol);
    hipFree(A->d_aval);
    delete A;
    return 0;
}

int kle_mat_get_local_size(const kle_mat *A, int64_t *m, int64_t *n)
{
    KLE_ARG(A && m && n, "null arg");
    *m = A->m_local;
    *n = A->n_local;
    return 0;
}

int kle_mat_get_size(const kle_mat *A, int64_t *m, int64_t *n)
{
    KLE_ARG(A, "null mat");
    if (m) *m = A->m_global;
    if (n) *n = A->n_global;
    return 0;
}

int kle_mat_get_ownership_range(const kle_mat *A, int64_t *lo, int64_t *hi)
{
    KLE_ARG(A && lo && hi, "null arg");
    *lo = A->row_lo;
    *hi = A->row_lo + A->m_local;
    return 0;
}

int kle_mat_get_info(const kle_mat *A, kle_mat_info *info)
{
    KLE_ARG(A && info, "null arg");
    kle_mat_info r{};
    r.m_global = A->m_global;
    r.n_global = A->n_global;
    r.m_local = A->m_local;
    r.n_local = A->n_local;
    KLE_TRY(kle_mat_get_local_nnz(A, &r.nz_used));
    r.format = A->kind;
    r.block_rows = A->kind == 0 ? A->R : 1;
    r.block_cols = A->kind == 0 ? A->C : 1;
    KLE_TRY(kle_mat_spmv_bytes(A, &r.spmv_bytes));
    *info = r;
    return 0;
}

int kle_mat_get_local_nnz(const kle_mat *A, int64_t *nnz)
{
    KLE_ARG(A && nnz, "null arg");
    if (A->kind == 1) {
        *nnz = A->nnz;
        return 0;
    }
    int64_t m, z;
    KLE_TRY(kle_mat_get_csr_size(A, &m, &z));
    *nnz = z;
    return 0;
}

int kle_mat_mult(kle_mat *A, kle_vec *x, kle_vec *y)
{
    KLE_ARG(A && x && y, "null arg");
    if (A->kind == 1 && !A->assembled) return fail(KLE_ERR_STATE, "matrix not assembled");
    KLE_TRY(check_mult_layout(A, x, y));
    return spmv(A, x, y, nullptr);
}

int kle_mat_mult_add(kle_mat *A, kle_vec *x, kle_vec *y, kle_vec *z)
{
    KLE_ARG(A && x && y && z, "null arg");
    kle_vec *t;
    KLE_TRY(kle_vec_duplicate(z, &t));
    KLE_TRY(kle_mat_mult(A, x, t));
    KLE_TRY(kle_vec_waxpy(z, 1.0, t, y));
    KLE_HIP(hipStreamSynchronize(A->ctx->stream));
    kle_vec_destroy(t);
    return 0;
}

int kle_mat_diagonal_scale(kle_mat *A, const kle_vec *L, const kle_vec *Rv)
{
    KLE_ARG(A, "null mat");
    sym_drop(A);  // the symmetric copy no longer describes the values
    kle_ctx *c = A->ctx;
    if (L && L->n_local != A->m_local) return fail(KLE_ERR_SIZ, "left scaling vector size mismatch");
    if (A->kind == 0) {
        const double *rx = nullptr;
        if (Rv) {
            if (Rv->n_local != A->n_local || Rv->ghost_lo != A->ghost_lo || Rv->ghost_hi != A->ghost_hi)
                return fail(KLE_ERR_SIZ, "right scaling vector must be a ghosted mesh vector of the column space");
            KLE_TRY(halo_exchange(c, Rv->base, Rv->ghost_lo, Rv->n_local, Rv->ghost_hi, Rv->lo_rank, Rv->hi_rank,
                                  Rv->send_lo, Rv->send_hi, nullptr, Rv->plan.get()));
            rx = Rv->base;
        }
        const int64_t th = A->nrows * 64;
#define SC_CASE(RR, CC)                                                                                    \
    if (A->R == RR && A->C == CC)                                                                          \
        hipLaunchKernelGGL((k_nb_scale<RR, CC>), dim3((th + 255) / 256), dim3(256), 0, c->stream, A->nrows, \
                           A->d_rowptr, A->d_rowcnt, A->d_vptr, A->vlayout, A->d_bcol, A->d_val,           \
                           L ? L->d : nullptr, rx);                                                        \
    else
        SC_CASE(3, 3) SC_CASE(2, 2) SC_CASE(2, 1) SC_CASE(1, 2) SC_CASE(3, 1) SC_CASE(1, 3) SC_CASE(6, 3)
        SC_CASE(3, 6) SC_CASE(1, 1) return fail(KLE_ERR_SUP, "no scale kernel for %dx%d", A->R, A->C);
#undef SC_CASE
    } else {
        if (Rv && Rv->n_local != A->n_local) return fail(KLE_ERR_SIZ, "right scaling vector size mismatch");
        hipLaunchKernelGGL(k_aij_scale, dim3((A->m_local + 255) / 256), dim3(256), 0, c->stream, A->m_local,
                           A->d_aptr, A->d_acol, A->d_aval, L ? L->d : nullptr, Rv ? Rv->d : nullptr);
        // keep the host mirror in step for later setValues
        KLE_HIP(hipMemcpyAsync(A->h_val.data(), A->d_aval, sizeof(double) * A->nnz, hipMemcpyDeviceToHost, c->stream));
    }
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int kle_mat_get_diagonal(const kle_mat *A, kle_vec *d)
{
    KLE_ARG(A && d, "null arg");
    KLE_ARG(d->n_local == A->m_local, "diagonal vector size mismatch");
    kle_ctx *c = A->ctx;
    if (A->kind == 0) {
        KLE_ARG(A->R == A->C, "get_diagonal needs square blocks");
        int *pos;
        KLE_HIP(hipMalloc(&pos, sizeof(int) * std::max<int64_t>(A->nrows, 1)));
        hipLaunchKernelGGL(k_diagpos, dim3((A->nrows + 255) / 256), dim3(256), 0, c->stream, A->nrows,
                           A->node_begin - A->ext_begin, A->d_rowptr, A->d_rowcnt, A->d_bcol, pos);
        hipLaunchKernelGGL(k_nb_diag, dim3((A->nrows * A->R + 255) / 256), dim3(256), 0, c->stream, A->nrows, A->R,
                           A->C, A->d_rowptr, A->d_rowcnt, A->d_vptr, A->vlayout, pos, A->d_val, d->d);
        KLE_HIP(hipGetLastError());
        KLE_HIP(hipStreamSynchronize(c->stream));
        hipFree(pos);
        return 0;
    }
    hipLaunchKernelGGL(k_aij_diag, dim3((A->m_local + 255) / 256), dim3(256), 0, c->stream, A->m_local, A->row_lo - A->col_lo,
                       A->d_aptr, A->d_acol, A->d_aval, d->d);
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int kle_mat_get_csr_size(const kle_mat *A, int64_t *m_local, int64_t *nnz)
{
    KLE_ARG(A && m_local && nnz, "null arg");
    *m_local = A->m_local;
    if (A->kind == 1) {
        *nnz = A->assembled ? A->nnz : 0;
        return 0;
    }
    if (A->mask_rule != MASK_NONE) {
        NBHost h;
        KLE_TRY(nb_download(A, h));
        int64_t z = 0;
        for (int64_t i = 0; i < A->nrows; ++i)
            for (int a = 0; a < A->R; ++a)
                for (int k = 0; k < h.cnt[i]; ++k)
                    for (int b = 0; b < A->C; ++b) z += nb_entry_exists(A, i, a, h.bc[h.rp[i] + k], b);
        *nnz = z;
        return 0;
    }
    std::vector<int> rp(A->nrows + 1), cnt(A->nrows);
    KLE_HIP(hipMemcpy(rp.data(), A->d_rowptr, sizeof(int) * (A->nrows + 1), hipMemcpyDeviceToHost));
    if (A->d_rowcnt) KLE_HIP(hipMemcpy(cnt.data(), A->d_rowcnt, sizeof(int) * A->nrows, hipMemcpyDeviceToHost));
    else
        for (int64_t i = 0; i < A->nrows; ++i) cnt[i] = rp[i + 1] - rp[i];
    int64_t z = 0;
    for (int64_t i = 0; i < A->nrows; ++i)
        z += A->diag_only_row[i] ? std::min(A->R, A->C) : (int64_t)cnt[i] * A->R * A->C;
    *nnz = z;
    return 0;
}

int kle_mat_get_row(const kle_mat *A, int64_t row, int64_t *ncols, int64_t *cols, double *vals)
{
    KLE_ARG(A && ncols, "null arg");
    KLE_ARG(row >= A->row_lo && row < A->row_lo + A->m_local, "row %lld not owned", (long long)row);
    const int64_t lr = row - A->row_lo;
    std::vector<int64_t> c;
    std::vector<double> v;
    if (A->kind == 1) {
        KLE_ARG(A->assembled, "matrix not assembled");
        const int64_t b = A->h_ptr[lr], e = A->h_ptr[lr + 1];
        c.assign(A->h_col.begin() + b, A->h_col.begin() + e);
        v.resize(e - b);
        if (e > b) KLE_HIP(hipMemcpy(v.data(), A->d_aval + b, sizeof(double) * (e - b), hipMemcpyDeviceToHost));
    } else {
        const int R = A->R, C = A->C;
        const int64_t i = lr / R;
        const int a = (int)(lr % R);
        int rp[2], cnt = 0;
        KLE_HIP(hipMemcpy(rp, A->d_rowptr + i, sizeof(int) * 2, hipMemcpyDeviceToHost));
        if (A->d_rowcnt) KLE_HIP(hipMemcpy(&cnt, A->d_rowcnt + i, sizeof(int), hipMemcpyDeviceToHost));
        else cnt = rp[1] - rp[0];
        const int mp = rp[1] - rp[0];
        std::vector<int> bc(std::max(cnt, 1));
        int64_t vp[2];
        KLE_HIP(hipMemcpy(vp, A->d_vptr + i, sizeof(int64_t) * 2, hipMemcpyDeviceToHost));
        std::vector<double> rowv(std::max<int64_t>(vp[1] - vp[0], 1));
        if (cnt) KLE_HIP(hipMemcpy(bc.data(), A->d_bcol + rp[0], sizeof(int) * cnt, hipMemcpyDeviceToHost));
        if (vp[1] > vp[0])
            KLE_HIP(hipMemcpy(rowv.data(), A->d_val + vp[0], sizeof(double) * (vp[1] - vp[0]), hipMemcpyDeviceToHost));
        auto val_at = [&](int t, int kk) { return rowv[vofs(A->vlayout, R * C, t, kk, cnt, mp)]; };
        if (A->diag_only_row[i]) {
            if (a < C) {
                c.push_back((A->node_begin + i) * C + a);
                v.push_back(val_at(a * C + a, 0));
            }
        } else {
            for (int k = 0; k < cnt; ++k)
                for (int b = 0; b < C; ++b) {
                    if (A->mask_rule != MASK_NONE && !nb_entry_exists(A, i, a, bc[k], b)) continue;
                    c.push_back((A->ext_gid.empty() ? A->ext_begin + bc[k] : A->ext_gid[bc[k]]) * C + b);
                    v.push_back(val_at(a * C + b, k));
                }
        }
    }
    *ncols = (int64_t)c.size();
    if (cols) std::copy(c.begin(), c.end(), cols);
    if (vals) std::copy(v.begin(), v.end(), vals);
    return 0;
}

int kle_mat_get_csr(const kle_mat *A, int64_t *indptr, int64_t *indices, double *data)
{
    KLE_ARG(A && indptr && indices && data, "null arg");
    if (A->kind == 1) {
        KLE_HIP(hipMemcpy(data, A->d_aval, sizeof(double) * A->nnz, hipMemcpyDeviceToHost));
        memcpy(indptr, A->h_ptr.data(), sizeof(int64_t) * (A->m_local + 1));
        memcpy(indices, A->h_col.data(), sizeof(int64_t) * A->nnz);
        return 0;
    }
    NBHost h;
    KLE_TRY(nb_download(A, h));
    const int R = A->R, C = A->C;
    int64_t z = 0;
    indptr[0] = 0;
    for (int64_t i = 0; i < A->nrows; ++i) {
        const int b0 = h.rp[i], m = h.cnt[i];
        for (int a = 0; a < R; ++a) {
            if (A->diag_only_row[i]) {
                // Dirichlet row: PETSc stores the diagonal only (mat_fs.py:44-45,115-120)
                if (a < C) {
                    indices[z] = (A->node_begin + i) * C + a;
                    data[z++] = h.at(A, i, a * C + a, 0);
                }
            } else {
                for (int k = 0; k < m; ++k)
                    for (int b = 0; b < C; ++b) {
                        if (A->mask_rule != MASK_NONE && !nb_entry_exists(A, i, a, h.bc[b0 + k], b)) continue;
                        indices[z] = (A->ext_gid.empty() ? A->ext_begin + h.bc[b0 + k] : A->ext_gid[h.bc[b0 + k]]) * C + b;
                        data[z++] = h.at(A, i, a * C + b, k);
                    }
            }
            indptr[i * R + a + 1] = z;
        }
    }
    return 0;
}

int kle_mat_convert_aij(const kle_mat *A, kle_mat **out)
{
    KLE_ARG(A && out, "null arg");
    KLE_ARG(A->ctx->nranks == 1, "convert_aij is single-rank");
    int64_t m, z;
    KLE_TRY(kle_mat_get_csr_size(A, &m, &z));
    kle_mat *B;
    KLE_TRY(kle_mat_create_aij(A->ctx, A->m_local, A->n_local, A->m_global, A->n_global, nullptr, nullptr, &B));
    B->h_ptr.resize(m + 1);
    B->h_col.resize(std::max<int64_t>(z, 1));
    B->h_val.resize(std::max<int64_t>(z, 1));
    KLE_TRY(kle_mat_get_csr(A, B->h_ptr.data(), B->h_col.data(), B->h_val.data()));
    B->h_col.resize(z);
    B->h_val.resize(z);
    B->assembled = true;
    B->stash.clear();
    KLE_TRY(aij_upload(B));
    *out = B;
    return 0;
}

int kle_mat_axpy(kle_mat *Y, double a, const kle_mat *X)
{
    KLE_ARG(Y && X, "null arg");
    sym_drop(Y);
    KLE_ARG(Y->kind == X->kind && Y->m_local == X->m_local && Y->n_local == X->n_local, "layout mismatch");
    kle_ctx *c = Y->ctx;
    if (Y->kind == 0) {
        KLE_ARG(Y->R == X->R && Y->C == X->C && Y->nblocks == X->nblocks, "axpy needs the same pattern");
        NBHost hy, hx;
        KLE_TRY(nb_download(Y, hy));
        KLE_TRY(nb_download(X, hx));
        if (hy.rp != hx.rp || hy.bc != hx.bc || hy.cnt != hx.cnt || hy.vp != hx.vp || Y->vlayout != X->vlayout)
            return fail(KLE_ERR_SUP, "axpy needs the same pattern");
        const int64_t n = Y->nvals;
        hipLaunchKernelGGL(k_axpy_same, dim3(grid_for(n, 256, 2048)), dim3(256), 0, c->stream, n, a, X->d_val, Y->d_val);
        KLE_HIP(hipGetLastError());
        KLE_HIP(hipStreamSynchronize(c->stream));
        return 0;
    }
    // aij: subset pattern, merged on the host (setup-time operation)
    for (int64_t r = 0; r < X->m_local; ++r)
        for (int64_t k = X->h_ptr[r]; k < X->h_ptr[r + 1]; ++k) {
            auto b = Y->h_col.begin() + Y->h_ptr[r], e = Y->h_col.begin() + Y->h_ptr[r + 1];
            auto it = std::lower_bound(b, e, X->h_col[k]);
            if (it == e || *it != X->h_col[k]) return fail(KLE_ERR_SUP, "axpy: X pattern not a subset of Y");
        }
    std::vector<double> xv(std::max<int64_t>(X->nnz, 1));
    KLE_HIP(hipMemcpy(Y->h_val.data(), Y->d_aval, sizeof(double) * Y->nnz, hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(xv.data(), X->d_aval, sizeof(double) * X->nnz, hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < X->m_local; ++r)
        for (int64_t k = X->h_ptr[r]; k < X->h_ptr[r + 1]; ++k) {
            auto b = Y->h_col.begin() + Y->h_ptr[r], e = Y->h_col.begin() + Y->h_ptr[r + 1];
            auto it = std::lower_bound(b, e, X->h_col[k]);
            Y->h_val[it - Y->h_col.begin()] += a * xv[k];
        }
    KLE_TRY(h2d(Y->d_aval, Y->h_val.data(), sizeof(double) * Y->nnz));
    return 0;
}

int kle_mat_duplicate(const kle_mat *A, int copy_values, kle_mat **out)
{
    KLE_ARG(A && out, "null arg");
    kle_mat *B = new kle_mat(*A);
    B->d_rowcnt = nullptr;
    B->d_rowbox = nullptr;
    B->d_vptr = nullptr;
    B->d_rowptr = nullptr;
    B->d_bcol = nullptr;
    B->d_dptr = nullptr;
    B->d_dict = nullptr;
    B->d_lid = nullptr;
    B->d_val = nullptr;
    B->d_aptr = nullptr;
    B->d_acol = nullptr;
    B->d_aval = nullptr;
    // the symmetric copy is A's own: B starts on full storage (rebuilt below
    // from the copied values when A had one)
    sym_forget(B);
    if (A->kind == 0) {
        const size_t nv = std::max<int64_t>(A->nvals, 1);
        KLE_HIP(hipMalloc(&B->d_rowptr, sizeof(int) * (A->nrows + 1)));
        KLE_HIP(hipMalloc(&B->d_bcol, sizeof(int) * std::max<int64_t>(A->nblocks, 1)));
        KLE_HIP(hipMalloc(&B->d_val, sizeof(double) * nv));
        KLE_HIP(hipMemcpy(B->d_rowptr, A->d_rowptr, sizeof(int) * (A->nrows + 1), hipMemcpyDeviceToDevice));
        if (A->d_rowcnt) {
            KLE_HIP(hipMalloc(&B->d_rowcnt, sizeof(int) * std::max<int64_t>(A->nrows, 1)));
            KLE_HIP(hipMemcpy(B->d_rowcnt, A->d_rowcnt, sizeof(int) * A->nrows, hipMemcpyDeviceToDevice));
        }
        KLE_HIP(hipMalloc(&B->d_vptr, sizeof(int64_t) * (A->nrows + 1)));
        KLE_HIP(hipMemcpy(B->d_vptr, A->d_vptr, sizeof(int64_t) * (A->nrows + 1), hipMemcpyDeviceToDevice));
        if (A->d_rowbox) {
            KLE_HIP(hipMalloc(&B->d_rowbox, sizeof(int) * 2 * std::max<int64_t>(A->nrows, 1)));
            KLE_HIP(hipMemcpy(B->d_rowbox, A->d_rowbox, sizeof(int) * 2 * A->nrows, hipMemcpyDeviceToDevice));
        }
        KLE_HIP(hipMemcpy(B->d_bcol, A->d_bcol, sizeof(int) * std::max<int64_t>(A->nblocks, 1), hipMemcpyDeviceToDevice));
        if (A->d_lid) {
            const int64_t ng = (A->nrows + DICT_GROUP - 1) / DICT_GROUP;
            KLE_HIP(hipMalloc(&B->d_dptr, sizeof(int) * (ng + 1)));
            KLE_HIP(hipMalloc(&B->d_dict, sizeof(int) * std::max<int64_t>(A->dict_len, 1)));
            KLE_HIP(hipMalloc(&B->d_lid, sizeof(uint16_t) * std::max<int64_t>(A->nblocks, 1)));
            KLE_HIP(hipMemcpy(B->d_dptr, A->d_dptr, sizeof(int) * (ng + 1), hipMemcpyDeviceToDevice));
            KLE_HIP(hipMemcpy(B->d_dict, A->d_dict, sizeof(int) * std::max<int64_t>(A->dict_len, 1),
                              hipMemcpyDeviceToDevice));
            KLE_HIP(hipMemcpy(B->d_lid, A->d_lid, sizeof(uint16_t) * std::max<int64_t>(A->nblocks, 1),
                              hipMemcpyDeviceToDevice));
        }
        if (copy_values) KLE_HIP(hipMemcpy(B->d_val, A->d_val, sizeof(double) * nv, hipMemcpyDeviceToDevice));
        else KLE_HIP(hipMemset(B->d_val, 0, sizeof(double) * nv));
        if (copy_values && A->d_sval) KLE_TRY(sym_build(B));
    } else {
        if (!copy_values) std::fill(B->h_val.begin(), B->h_val.end(), 0.0);
        if (A->assembled) {
            if (copy_values) KLE_HIP(hipMemcpy(B->h_val.data(), A->d_aval, sizeof(double) * A->nnz, hipMemcpyDeviceToHost));
            KLE_TRY(aij_upload(B));
        }
    }
    *out = B;
    return 0;
}

int kle_get_nb_pad(void) { return g_nb_pad; }

int kle_set_nb_layout(int layout)
{
    KLE_ARG(layout == 0 || layout == 1, "layout must be 0 (padded streams) or 1 (16-block chunks)");
    g_nb_layout = layout;
    return 0;
}

int kle_get_nb_layout(void) { return g_nb_layout; }

int kle_mat_set_spmv_structured(kle_mat *A, int on)
{
    KLE_ARG(A, "null matrix");
    A->spmv_struct = on != 0;
    return 0;
}

int kle_mat_move_values(kle_mat *A, long long shift, int fresh)
{
    using namespace kle;
    KLE_ARG(A && A->d_sval, "no symmetric storage");
    KLE_ARG(shift >= 0 && shift % 8 == 0 && shift <= (1ll << 30), "shift: a multiple of 8 bytes in [0, 1 GiB]");
    const size_t bytes = sizeof(double) * (size_t)std::max<int64_t>(A->snvals, 1);
    if (!fresh && A->sval_raw && (size_t)shift + bytes <= A->sval_cap) {
        // the same allocation (the same physical pages), another offset:
        // through a scratch copy (the ranges may overlap)
        double *tmp = nullptr;
        if (hipMalloc(&tmp, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return fail(KLE_ERR_MEM, "out of device memory for the move's scratch copy");
        }
        KLE_HIP(hipStreamSynchronize(A->ctx->stream));
        KLE_HIP(hipMemcpy(tmp, A->d_sval, bytes, hipMemcpyDeviceToDevice));
        double *nv = reinterpret_cast<double *>(static_cast<char *>(A->sval_raw) + shift);
        KLE_HIP(hipMemcpy(nv, tmp, bytes, hipMemcpyDeviceToDevice));
        KLE_HIP(hipFree(tmp));
        A->d_sval = nv;
        return 0;
    }
    if (!fresh) shift = 0;  // (a new allocation with room for later offsets: shift applies from the next call)
    const size_t cap = bytes + (size_t)(fresh ? shift : (8ll << 20));
    double *old = A->d_sval;
    void *old_raw = A->sval_raw ? A->sval_raw : A->d_sval;
    KLE_HIP(hipStreamSynchronize(A->ctx->stream));
    if (sval_alloc(A, cap)) {  // (the same allocator as the build's)
        A->d_sval = old;
        A->sval_raw = old_raw == old ? nullptr : old_raw;
        return fail(KLE_ERR_MEM, "out of device memory for the moved values (%zu bytes)", cap);
    }
    A->sval_cap = cap;
    char *raw = reinterpret_cast<char *>(A->d_sval);
    double *nv = reinterpret_cast<double *>(raw + shift);
    KLE_HIP(hipMemcpy(nv, old, bytes, hipMemcpyDeviceToDevice));
    KLE_HIP(hipFree(old_raw));
    A->sval_raw = raw;
    A->d_sval = nv;
    return 0;
}

int kle_mat_get_sym_bricks(const kle_mat *A, int *nbricks, int *dims, double *entries_per_row, double *model_us)
{
    KLE_ARG(A && nbricks && dims && entries_per_row && model_us, "null arg");
    const bool on = A->d_sval && A->sym_brick;
    *nbricks = on ? A->nbricks : 0;
    for (int k = 0; k < 3; ++k) dims[k] = on ? A->brick_dims[k] : 0;
    *entries_per_row = on && A->nrows ? (double)A->sws_entries / A->nrows : 0.0;
    *model_us = on ? A->brick_model_us : 0.0;
    return 0;
}

int kle_mat_set_symmetric(kle_mat *A, int on)
{
    KLE_ARG(A, "null matrix");
    if (!on) {
        sym_drop(A);
        return 0;
    }
    return sym_build(A);
}

int kle_mat_get_symmetric(const kle_mat *A, int *on)
{
    KLE_ARG(A && on, "null arg");
    *on = A->d_sval != nullptr;
    return 0;
}


int kle_mat_is_structured(const kle_mat *A, int *on)
{
    KLE_ARG(A && on, "null arg");
    *on = A->d_rowbox != nullptr;
    return 0;
}

int kle_mat_set_halo_overlap(kle_mat *A, int on)
{
    KLE_ARG(A, "null matrix");
    A->halo_overlap = on != 0;
    return 0;
}

int kle_set_nb_pad(int quantum)
{
    KLE_ARG(quantum >= 1 && quantum <= 64, "pad quantum must be in [1,64]");
    g_nb_pad = quantum;
    return 0;
}

int kle_mat_get_format(const kle_mat *A, char *buf, int buflen)
{
    KLE_ARG(A && buf && buflen > 3, "bad arg");
    snprintf(buf, buflen, "%s", A->kind == 0 ? "nb" : "aij");
    return 0;
}

int kle_mat_spmv_kernel(const kle_mat *A, char *buf, int buflen)
{
    KLE_ARG(A && buf && buflen > 0, "bad arg");
    std::string s;
    if (A->kind != 0) {
        s = "k_aij_spmv<8,4>";
    } else if (A->d_sval && g_tune.spmv_sym) {
        s = sym_kernel_name(A);
    } else {
        const int wv = spmv_waves(A), lay = A->vlayout;
        const bool st = A->spmv_struct && A->d_rowbox, n33 = A->R == 3 && A->C == 3 && lay == 1;
        if (n33 && st && wv == 8 && g_tune.spmv_x_lds && (7 + A->box_max) * A->box_max * A->box_max <= XL_CAP)
            s = "k_nb_spmv_xl<8>";
        else if (n33 && !st && wv == 8 && A->d_lid && g_tune.spmv_dict)
            s = "k_nb_spmv_dict";
        else
            s = "k_nb_spmv<" + std::to_string(A->R) + "," + std::to_string(A->C) + "," + std::to_string(lay) + "," +
                (st ? "true" : "false") + "," + std::to_string(n33 && wv == 8 ? 8 : SPMV_WAVES) + ">";
    }
    snprintf(buf, buflen, "%s", s.c_str());
    return 0;
}

int kle_mat_spmv_bytes(const kle_mat *A, double *bytes)
{
    KLE_ARG(A && bytes, "null arg");
    if (A->kind == 0 && A->d_sval && g_tune.spmv_sym) {
        *bytes = sym_spmv_bytes(A);
    } else if (A->kind == 0) {
        // bytes the SpMV must move: real blocks only (row padding is not counted);
        // the column stream unless the columns are computed from row boxes
        // (dictionary matrices: a 2-byte position per block plus the
        // dictionaries and their offsets instead of the column stream)
        const bool sb = A->spmv_struct && A->d_rowbox;
        const bool dict = !sb && A->d_lid && g_tune.spmv_dict;
        const double colb = sb ? 0.0 : dict ? 2.0 : 4.0;
        *bytes = (double)A->nblocks_real * (A->R * A->C * 8.0 + colb) + (A->nrows + 1) * 4.0 +
                 (A->d_rowcnt ? A->nrows * 4.0 : 0.0) + (sb ? A->nrows * 8.0 : 0.0) +
                 (dict ? A->dict_len * 4.0 + ((A->nrows + DICT_GROUP - 1) / DICT_GROUP + 1) * 4.0 : 0.0) +
                 (double)A->ext_nodes * A->C * 8.0 + (double)A->m_local * 8.0;
    } else {
        *bytes = (double)A->nnz * 12.0 + (A->m_local + 1) * 8.0 + A->n_local * 8.0 + A->m_local * 8.0;
    }
    return 0;
}

int kle_mat_time_local_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, int reps, double *ms)
{
    KLE_ARG(A && x && y && ms && reps >= 1, "bad arg");
    KLE_TRY(check_mult_layout(A, x, y));
    KLE_ARG(spmv_can_split(A), "local product timing: box-brick symmetric storage only");
    kle_ctx *c = A->ctx;
    hipEvent_t e0, e1;
    KLE_HIP(hipEventCreate(&e0));
    if (hipEventCreate(&e1) != hipSuccess) {
        hipEventDestroy(e0);
        return fail(KLE_ERR_DEVICE, "event create failed");
    }
    int rc = hipEventRecord(e0, c->stream) == hipSuccess ? 0 : fail(KLE_ERR_DEVICE, "event record failed");
    for (int i = 0; i < reps && !rc; ++i) rc = brick_spmv_local(A, x, y);
    float t = 0.0f;
    if (!rc && (hipEventRecord(e1, c->stream) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&t, e0, e1) != hipSuccess))
        rc = fail(KLE_ERR_DEVICE, "event timing failed");
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (rc) return rc;
    *ms = (double)t / reps;
    return 0;
}

}  // extern "C"
