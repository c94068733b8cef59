// kle_sym.hip -- symmetric (SBAIJ-style, upper-triangle) node-block storage of
// the KLE K and its SpMV kernels for gfx950 (kle_mat_set_symmetric =
// MatSetOption(MAT_SPD); K is SPD: MatFS.buildFS, mat_fs.py:150-192).
#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "kle_brick.hpp"
#include "kle_internal.hpp"
#include "kle_sym_dev.hpp"

namespace kle {

// ---------------------------------------------------------------------------
// Symmetric node-block storage (PETSc MATSBAIJ; kle_mat_set_symmetric): on a
// box lattice a structured row's columns are its box in lexicographic order,
// so the upper triangle j >= i of row i is the tail [k0, m) of that box from
// its own (diagonal) block on.  Only those blocks are stored (same 16-block
// chunk layout, rows 128-B aligned): 31.4 M of config 2's 62.4 M blocks.
//
// y = A x as one pass over the stored blocks: block (i, j) adds B x_j to row i
// and B^T x_i to row j.  A workgroup takes a tile of SYM_TX x SYM_TY rows of
// TZ lattice planes; every row it touches lies in the tile's region
// [x0-P, x0+TX+P) x [y0-P, y0+TY+P) x [z0, z0+TZ-1+P] (P = the largest
// row-box reach), accumulated in LDS and written as the tile's partial sums to
// a workspace; the gather kernel sums, per row, the partials of the (at most
// 2 x 2 x (P/TZ+2)) tiles whose regions contain it, in a fixed tile order.
// HBM: the stored values once (half of the full storage) + the partials
// written and read once.
constexpr int SYM_TX = 8;  // tile rows in x; TY x TZ (8 x 2, 4 x 4 or 2 x 4) per matrix: sym_TY, sym_TZ
constexpr int SYM_FILL = 12;  // x-fill loads per thread of k_nb_spmv_sym_xl (one pass over the region)

// Lattices: the rows are the owned Lx x Ly x Lz nodes; the columns add zo
// lattice planes of lower ghosts before them and hp of upper ghosts after
// them (slab partitions, N > 1: ext layout [lower ghosts | owned | upper]).
// Row boxes (d_rowbox) are in column (ext) coordinates.  The upper triangle
// of an owned row never reaches a lower ghost; the blocks that reach upper
// ghosts add their transposed parts to ghost rows, whose partials go back to
// the owner (sym_spmv's reverse halo).
// Region of a tile: [x0 - PX, x0 - PX + RX) x [y0 - PY, y0 - PY + RY) x
// [z0, z0 + RZ) -- the bounding box, over all tiles, of the rows' upper
// triangles relative to their tile's origin (sym_build).  On element-aligned
// tiles an upper triangle reaches back p nodes in x and y (from the planes
// above) but forward only to the next element boundary, one node past the
// tile: 13 x 9 x 5 nodes for 8 x 4 x 4 tiles at p = 4, not (8 + 2p) x (4 + 2p)
// x (4 + p) = 1536.
struct SymGeo {
    int Lx, Ly, Lz, P, TX, TY, TZ, PX, PY, RX, RY, RZ, ntx, nty, ntz, zo, hp;
    int WN;  // per-component stride of a tile's partials in the workspace (>= RX RY RZ)
};

__device__ __forceinline__ void sym_box(const int *__restrict__ rowbox, int64_t i, int Lx, int64_t Lxy, int &bx,
                                        int &by, int &bz, int &bnx, int &bny, int &bnz)
{
    const int64_t base = rowbox[2 * i];
    const int d = rowbox[2 * i + 1];
    bz = (int)(base / Lxy);
    const int64_t r = base - (int64_t)bz * Lxy;
    by = (int)(r / Lx);
    bx = (int)(r - (int64_t)by * Lx);
    bnx = d & 255;
    bny = (d >> 8) & 255;
    bnz = (d >> 16) & 255;
}

// Copy each row's upper tail into the symmetric layout and measure
// max |B_ij - B_ji^T| per row (the stored triangle must describe the matrix).
__global__ __launch_bounds__(256) void k_sym_build(int64_t nrows, int Lx, int Ly, int zo, const int *__restrict__ rowptr,
                                                   const int *__restrict__ rowcnt, const int *__restrict__ rowbox,
                                                   const int64_t *__restrict__ vptr, const double *__restrict__ val,
                                                   const int64_t *__restrict__ svptr, double *__restrict__ sval,
                                                   double *__restrict__ rowdiff, double *__restrict__ rowmax)
{
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= nrows) return;
    const int64_t Lxy = (int64_t)Lx * Ly;
    const int z = (int)(i / Lxy), y = (int)((i - z * Lxy) / Lx), x = (int)(i - z * Lxy - (int64_t)y * Lx);
    int bx, by, bz, bnx, bny, bnz;
    sym_box(rowbox, i, Lx, Lxy, bx, by, bz, bnx, bny, bnz);
    bz -= zo;  // (owned coordinates)
    const int m = rowcnt ? rowcnt[i] : rowptr[i + 1] - rowptr[i], mp = rowptr[i + 1] - rowptr[i];
    const int k0 = (x - bx) + bnx * ((y - by) + bny * (z - bz));
    const int mu = m - k0;
    const double *v = val + vptr[i];
    double *sv = sval + svptr[i];
    double dmax = 0.0, vmax = 0.0;
    for (int kk = lane; kk < mu; kk += 64) {
        const int k = k0 + kk;
        double b[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            b[t] = v[vofs(1, 9, t, k, m, mp)];
            sv[vofs(1, 9, t, kk, mu, mu)] = b[t];
            vmax = fmax(vmax, fabs(b[t]));
        }
        if (kk == 0) continue;
        const int bnxy = bnx * bny;
        const int kz = k / bnxy, ky = (k - kz * bnxy) / bnx, kx = k - kz * bnxy - ky * bnx;
        const int64_t j = (bx + kx) + (int64_t)Lx * (by + ky) + Lxy * (bz + kz);
        if (j >= nrows) continue;  // an upper ghost row (N > 1): sym_build checks those by a product
        int cx, cy, cz, cnx, cny, cnz;
        sym_box(rowbox, j, Lx, Lxy, cx, cy, cz, cnx, cny, cnz);
        cz -= zo;
        if (x < cx || x >= cx + cnx || y < cy || y >= cy + cny || z < cz || z >= cz + cnz) {
            dmax = INFINITY;  // (i, j) stored but (j, i) not in the pattern
            continue;
        }
        const int mj = rowcnt ? rowcnt[j] : rowptr[j + 1] - rowptr[j], mpj = rowptr[j + 1] - rowptr[j];
        const int kj = (x - cx) + cnx * ((y - cy) + cny * (z - cz));
        const double *vj = val + vptr[j];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) dmax = fmax(dmax, fabs(b[a * 3 + c] - vj[vofs(1, 9, c * 3 + a, kj, mj, mpj)]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        dmax = fmax(dmax, __shfl_xor(dmax, o, 64));
        vmax = fmax(vmax, __shfl_xor(vmax, o, 64));
    }
    if (lane == 0) {
        rowdiff[i] = dmax;
        rowmax[i] = vmax;
    }
}

// Same tile pass with the wave's (row, 64-block pass) items flattened into one
// software-pipelined loop: the values and x entries of the next item are in
// flight while the current one is multiplied and accumulated (a wave's rows
// average 1.4 passes of 64 blocks, so one item at a time leaves it waiting
// on HBM latency at every row).
struct SymRow {
    const double *v;
    double x0, x1, x2;
    int bnx, bnxy, k0, mu, rx0, ry0, rz0, own;
    float ibnx, ibnxy;  // 1/bnx, 1/bnxy: quotients of block positions by float multiply + one fix-up
};

// ---------------------------------------------------------------------------
// Symmetric SpMV with x staged in LDS (round 3; default).  Every x entry the
// tile's blocks multiply lies in the tile's region -- the same region its
// transposed partials go to -- so the workgroup loads x of the whole region
// once, as coalesced lattice-line segments (16 nodes = 384 B per line at
// P = 4), and each block reads x_j from LDS at the region index it already
// computes for its transposed add: an item is 9 value loads (nontemporal,
// whole 128-B lines) instead of 9 + 3 x gathers through L1/L2/MALL.  The
// first item's value loads are issued before the x fill lands, so the tile
// prologue costs one memory round trip, not two.
//
// DET (bitwise reproducible): the transposed adds are exact int64 fixed-point
// sums (ds_add_u64).  Integer addition commutes, so the partials -- and y --
// do not depend on the order in which the waves' adds reach LDS.  Scale per
// tile S = 2^(61-E) with 2^E > W_t * max|x_i| (W_t, precomputed by
// k_sym_bound: the largest sum, over a region node, of the transposed row
// sums sum_a |B[a][b]| of the blocks that add to it; max|x_i| over the tile's
// rows from LDS), so no partial can exceed 2^61.  Each add is rounded to
// 2^(E-62) absolute (fp64 rounds a contribution of size max|B| max|x| to
// 2^-53 of it).  The direct row sums B x_j stay fp64 in registers (fixed-order
// DPP sum per row, one writer per row) and are added to the row's partial at
// the end.  Without DET the transposed adds are fp64 LDS atomics (ds_add_f64),
// equal to the full-storage product to rounding but run-dependent.
// A partial store with a cache policy (spmv_sym_stpol): 0 plain (write-back
// L2), 1 nontemporal, 2 sc1, 3 sc0 sc1 (write-through: the line leaves L2
// with the store instead of at its eviction under the value stream)
__device__ __forceinline__ void pst(double *p, double v, int pol)
{
    if (pol == 1)
        __builtin_nontemporal_store(v, p);
    else if (pol == 2)
        asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if (pol == 3)
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else
        *p = v;
}

// launch-local block -> work item: runs of ch consecutive items per XCD
// (workgroups are dealt round-robin over the 8 XCDs; kle_mat.hip xcd_block)
__device__ __forceinline__ int64_t gsym_block(int ch)
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

// SGPR cap: the HIP runtime admits workgroups per CU by its own register
// model, 512 SGPRs per SIMD / the kernel's SGPRs rounded up to 16 (the occupancy
// API and the dispatcher agree: 106 SGPRs -> 4 waves per SIMD = 2 of these
// 8-wave workgroups per CU, measured with the probe build's phase timestamps);
// at <= 80 it admits 6 waves per SIMD = 3 workgroups (75 VGPRs allow 6)
#ifndef SYM_XL_SGPRS
#define SYM_XL_SGPRS 80
#endif
template <int WV, bool DET, int TY, int TZ>
__global__ __launch_bounds__(64 * WV, 4) __attribute__((amdgpu_num_sgpr(SYM_XL_SGPRS))) void k_nb_spmv_sym_xl(SymGeo g, const int *__restrict__ srow,
                                                             const int64_t *__restrict__ svptr,
                                                             const double *__restrict__ sval,
                                                             const double *__restrict__ x, double *__restrict__ ws,
                                                             const int *__restrict__ tile_e,
                                                             const int *__restrict__ istate, int t0,
                                                             int early, int stpol, int xcd KLE_PROBE_PARAM)
{
    KLE_PROBE_CONST
    // LDS: x [3][RN] | y [3][RN + 64] (DET: int64; 64 dummy slots per
    // component take the adds of masked lanes) | direct row sums [3][TR]
    extern __shared__ double lds[];
    KLE_PROBE_TS(ts0)
    // the solve's reason word (nonzero: the solve has ended, every kernel is a
    // no-op): loaded first, tested once the tile's descriptor and x loads are
    // in flight, so its round trip overlaps theirs instead of delaying them
    const int stop = istate ? istate[I_REASON] : 0;
    static_assert(TY * TZ == 16 || TY * TZ == 8, "tiles of 128 or 64 rows");
    constexpr int TR = SYM_TX * TY * TZ, NT = 64 * WV;
    constexpr int NQ = SYM_TX * TY / WV;  // row slots per wave and plane
    constexpr int NS = NQ * TZ;               // row slots per wave
    const int RN = g.RX * g.RY * g.RZ, RS = RN + 64;
    double *xl = lds, *yl = lds + 3 * RN, *yd = lds + 3 * RN + 3 * RS;
    // (N > 1: tiles [t0, ...) of one launch; xcd > 0: runs of xcd tiles per XCD, spmv_sym_xcd)
    const int64_t t = gsym_block(xcd) + t0;
    const int tix = (int)(t % g.ntx);
    const int64_t q = t / g.ntx;
    const int tiy = (int)(q % g.nty), tz = (int)(q / g.nty) * TZ;
    const int x0 = tix * SYM_TX, y0 = tiy * TY, ox = x0 - g.PX, oy = y0 - g.PY;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t Lxy = (int64_t)g.Lx * g.Ly;
    const int nx = min(SYM_TX, g.Lx - x0);
    // slot s of wave w: plane tz + s / NQ; with u = s % NQ, lattice line
    // y0 + (w >> 3) + (WV >> 3) u and x offset (w + u) & 7 -- the 64 rows of a
    // plane once over the WV waves, every wave across lines and x classes
    // (the end-of-tile barrier waits for the slowest wave)
    auto slot_x = [&](int s) { return (w + s % NQ) & 7; };
    auto slot_y = [&](int s) { return (w >> 3) + (WV >> 3) * (s % NQ); };
    auto slot_ok = [&](int s) { return y0 + slot_y(s) < g.Ly && slot_x(s) < nx && tz + s / NQ < g.Lz; };
    auto next_slot = [&](int s) {
        while (s < NS && !slot_ok(s)) ++s;
        return s;
    };
    // Every global load below is unconditional (clamped to a valid address,
    // masked afterwards) and every use of a loaded value is too: a load or a
    // use under a branch makes the compiler's wait counting conservative, and
    // it then drains the whole load queue at every item.
    // 1. the wave's row descriptors (packed box, value offset): lane s holds slot s
    int pd, psl, psh;
    {
        const bool ok = lane < NS && slot_ok(lane);
        const int64_t i =
            ok ? x0 + slot_x(lane) + (int64_t)g.Lx * (y0 + slot_y(lane)) + Lxy * (tz + lane / NQ) : 0;
        pd = srow[i];
        const int64_t o = svptr[i];
        psl = (int)(uint32_t)o;
        psh = (int)(o >> 32);
    }
    // 2. x of the region, one pass (the launch guarantees NL <= FB * fstep):
    // line (ry, rz) is 3 RX contiguous doubles of x; thread -> a fixed
    // position in a line, lines fl0, fl0 + fstep, ...  Nodes outside the
    // lattice read as 0.
    const int L3 = 3 * g.RX, NL = g.RY * g.RZ;
    const int fc = threadIdx.x % L3, fl0 = threadIdx.x / L3, fstep = NT / L3;
    const int frx = fc / 3, fcc = fc - 3 * frx;
    const bool fx_ok = fl0 < fstep && ox + frx >= 0 && ox + frx < g.Lx;
    double fv[SYM_FILL];
#pragma unroll
    for (int f = 0; f < SYM_FILL; ++f) {
        const int l = fl0 + f * fstep;
        const int rz = l / g.RY, ry = l - rz * g.RY;
        const bool ok = fx_ok && l < NL && oy + ry >= 0 && oy + ry < g.Ly && tz + rz < g.Lz + g.hp;
        const int64_t node = ok ? (int64_t)(ox + frx) + (int64_t)g.Lx * (oy + ry) + Lxy * (g.zo + tz + rz) : 0;
        const double v = x[3 * node + fcc];
        fv[f] = ok ? v : 0.0;
    }
    if (__builtin_amdgcn_readfirstlane(stop) != 0) return;  // (nothing written yet)
    for (int k = threadIdx.x; k < 3 * RS; k += NT) yl[k] = 0.0;
    for (int k = threadIdx.x; k < 3 * TR; k += NT) yd[k] = 0.0;
    // a row from its packed descriptor (sym_row_desc): no divisions -- the
    // scalar unit is shared by the CU's waves, and 64-bit box arithmetic per
    // row cost as many instructions as the row's items
    auto slot_row = [&](int s, SymRow &R) {
        const int sx = slot_x(s), sy = slot_y(s), sz = s / NQ;  // the row in the tile
        const int d = __builtin_amdgcn_readlane(pd, s);
        const int dbx = d & 15, dby = (d >> 4) & 15, dbz = (d >> 8) & 15;
        R.bnx = (d >> 12) & 15;
        const int bny = (d >> 16) & 15, bnz = (d >> 20) & 15;
        R.bnxy = R.bnx * bny;
        R.ibnx = __builtin_amdgcn_rcpf((float)R.bnx);  // (sym_div fixes the quotient up)
        R.ibnxy = __builtin_amdgcn_rcpf((float)R.bnxy);
        R.k0 = dbx + R.bnx * (dby + bny * dbz);
        R.mu = R.bnxy * bnz - R.k0;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(psl, s);
        const int64_t hi = __builtin_amdgcn_readlane(psh, s);
        R.v = sval + ((hi << 32) | lo);
        R.rx0 = g.PX + sx - dbx;  // box corner in the region
        R.ry0 = g.PY + sy - dby;
        R.rz0 = sz - dbz;
        R.own = sx + SYM_TX * (sy + TY * sz);  // row slot in the tile
        const int ir = (sx + g.PX) + g.RX * ((sy + g.PY) + g.RY * sz);  // its region index
        R.x0 = uni_d(xl[ir]);  // (the first row re-reads these once the fill has landed)
        R.x1 = uni_d(xl[RN + ir]);
        R.x2 = uni_d(xl[2 * RN + ir]);
        // every field is wave-uniform: keep them in SGPRs, so moving a row
        // between the cur / nxt sets never touches VGPRs with loads in flight
        R.ibnx = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, R.ibnx)));
        R.ibnxy = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, R.ibnxy)));
        R.mu = __builtin_amdgcn_readfirstlane(R.mu);
        R.k0 = __builtin_amdgcn_readfirstlane(R.k0);
        R.bnx = __builtin_amdgcn_readfirstlane(R.bnx);
        R.bnxy = __builtin_amdgcn_readfirstlane(R.bnxy);
        R.rx0 = __builtin_amdgcn_readfirstlane(R.rx0);
        R.ry0 = __builtin_amdgcn_readfirstlane(R.ry0);
        R.rz0 = __builtin_amdgcn_readfirstlane(R.rz0);
        R.own = __builtin_amdgcn_readfirstlane(R.own);
    };
    // item = (row, pass kb): the values of its 64 blocks (lanes past the
    // row's end re-read its last block; their results go nowhere) and the
    // blocks' region index
    auto load_v = [&](const SymRow &R, int kb, double *vv, int &rr) {
        const int kk = min(kb + lane, R.mu - 1);
        const int q16 = R.mu & ~15;
        const bool ch = kk < q16;
        const int o0 = ch ? (kk >> 4) * 144 + (kk & 15) : q16 * 9 + (kk - q16);
        const int st = ch ? 16 : R.mu - q16;
        unsigned o[9];
#pragma unroll
        for (int s = 0; s < 9; ++s) o[s] = (unsigned)(o0 + s * st) * 8u;
        sym_ld9(vv, R.v, o);
        const int k = R.k0 + kk;
        const int kz = sym_div(k, R.bnxy, R.ibnxy), rem = k - kz * R.bnxy;
        const int ky = sym_div(rem, R.bnx, R.ibnx), kx = rem - ky * R.bnx;
        rr = (R.rx0 + kx) + g.RX * ((R.ry0 + ky) + g.RY * (R.rz0 + kz));
        if (probe & 16) rr = lane;  // (timing probe 16: no block -> region arithmetic)
    };
    auto load_x = [&](int rr, double *xv) {
        xv[0] = xl[rr];
        xv[1] = xl[RN + rr];
        xv[2] = xl[2 * RN + rr];
    };
    // 3. items = (row, pass of 64 blocks).  The issue cursor (row I, slot xi,
    // pass ki) runs one item in front of the compute cursor (row C, slot xc,
    // pass kc); past the wave's last item it stays there, re-reading it
    // (cache hits), so every step issues exactly 9 loads and the wait for the
    // item being summed is a fixed vmcnt(9).  (Two items ahead measured
    // slower in rounds 2 and 3.)  A wave without rows in
    // this tile (16-wave tiles on a lattice edge) loads a dummy item.
    int xi = next_slot(0), ki = 0;
    const bool any = xi < NS;
    bool idone = !any;
    SymRow I, C;
    if (any) {
        slot_row(xi, I);
    } else {
        I.v = sval;
        I.mu = 1;
        I.k0 = 0;
        I.bnx = I.bnxy = 1;
        I.ibnx = I.ibnxy = 1.0f;
        I.rx0 = I.ry0 = I.rz0 = 0;
    }
    auto issue_next = [&]() {
        if (idone) return;
        if (ki + 64 < I.mu) {
            ki += 64;
            return;
        }
        const int nx = next_slot(xi + 1);
        if (nx >= NS) {
            idone = true;
            return;
        }
        xi = nx;
        ki = 0;
        slot_row(xi, I);
    };
    double v0[9], v1[9];
    int r0, r1 = 0;
    // early: the first item's value loads go out with the x fill (they do not
    // read x), so the tile's first round trip overlaps the fill's
    if (early) load_v(I, ki, v0, r0);
#pragma unroll
    for (int f = 0; f < SYM_FILL; ++f) {
        const int l = fl0 + f * fstep;  // (unused slots store into a dummy y slot: no branch)
        xl[fl0 < fstep && l < NL ? fcc * RN + frx + g.RX * l : 4 * RN + lane] = fv[f];
    }
    if (!early) load_v(I, ki, v0, r0);  // in flight across the barrier
    __builtin_amdgcn_s_waitcnt(0xC07F);  // LDS stores done (lgkmcnt 0); the value loads stay in flight
    __builtin_amdgcn_s_barrier();
    KLE_PROBE_TS(ts1)
    double S = 1.0, invS = 1.0;
    if (DET) {
        // max |x_i| over the tile's rows (every wave computes it; max is exact)
        double m = 0.0;
        int bad = 0;
        for (int r = lane; r < TR; r += 64) {
            const int k = (g.PX + (r & 7)) + g.RX * ((g.PY + (r >> 3) % TY) + g.RY * (r / (SYM_TX * TY)));
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double a = fabs(xl[c * RN + k]);
                bad |= !(a <= 1.7976931348623157e308);
                m = fmax(m, a);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
        if (__ballot(bad)) {
            S = 0.0;  // non-finite x: the partials come out NaN, as a floating-point sum would
            invS = __builtin_nan("");
        } else if (m > 0.0) {
            int em;
            (void)frexp(m, &em);  // 2^em > m
            const int E = min(max(tile_e[t] + em, -960), 1020);
            S = ldexp(1.0, 61 - E);
            invS = ldexp(1.0, E - 61);
        }
    }
    if (any && !(probe & 128)) {  // (timing probe 128: no item loop)
        int xc = next_slot(0), kc = 0;
        slot_row(xc, C);  // (x_i from LDS, now that the fill has landed)
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
        // one item: issue the next item into vn, wait for vv (the next
        // item's loads stay in flight), sum it
        auto step = [&](double *vv, const int rr, double *vn, int &rn) {
            issue_next();
            load_v(I, ki, vn, rn);
            double xv[3];
            if (probe & 4)
                xv[0] = xv[1] = xv[2] = C.x0;
            else
                load_x(rr, xv);  // LDS latency overlaps the wait
            sym_wait9<9>(vv);
            // B x_j into the row, B^T x_i into row j (lanes past the row's end
            // and the diagonal block add into their dummy slot)
            const int kk = kc + lane;
            const bool live = kk < C.mu;
            const int rt = live && kk > 0 ? rr : RN + lane;
            const double s0 = vv[0] * xv[0] + vv[1] * xv[1] + vv[2] * xv[2];
            const double s1 = vv[3] * xv[0] + vv[4] * xv[1] + vv[5] * xv[2];
            const double s2 = vv[6] * xv[0] + vv[7] * xv[1] + vv[8] * xv[2];
            acc0 += live ? s0 : 0.0;
            acc1 += live ? s1 : 0.0;
            acc2 += live ? s2 : 0.0;
            const double t0 = vv[0] * C.x0 + vv[3] * C.x1 + vv[6] * C.x2;
            const double t1 = vv[1] * C.x0 + vv[4] * C.x1 + vv[7] * C.x2;
            const double t2 = vv[2] * C.x0 + vv[5] * C.x1 + vv[8] * C.x2;
            if (probe & 1) {
                if (!live) yd[lane] = t0 + t1 + t2;  // (timing probe: no transposed adds)
            } else if (DET) {
                unsigned long long *yi = reinterpret_cast<unsigned long long *>(yl);
                atomicAdd(&yi[rt], fx_of(t0, S));
                atomicAdd(&yi[RS + rt], fx_of(t1, S));
                atomicAdd(&yi[2 * RS + rt], fx_of(t2, S));
            } else {
                atomicAdd(&yl[rt], t0);
                atomicAdd(&yl[RS + rt], t1);
                atomicAdd(&yl[2 * RS + rt], t2);
            }
            if (kc + 64 < C.mu) {
                kc += 64;
                return true;
            }
            // the row is done: its direct sum (fixed-order DPP), one writer
            if (!(probe & 2)) wsum3_dpp(acc0, acc1, acc2);  // (timing probe 2: no row sums)
            if (lane < 3) yd[lane * TR + C.own] = lane == 0 ? acc0 : lane == 1 ? acc1 : acc2;
            acc0 = acc1 = acc2 = 0.0;
            const int nx = next_slot(xc + 1);
            if (nx >= NS) return false;
            xc = nx;
            kc = 0;
            slot_row(xc, C);
            return true;
        };
        while (step(v0, r0, v1, r1) && step(v1, r1, v0, r0)) {
        }
    }
    // the last (re-read) loads land before their registers are reused
    sym_wait9<0>(v0);
    sym_wait9<0>(v1);
    __syncthreads();
    KLE_PROBE_TS(ts2)
    // 4. the tile's partial sums: region nodes inside the lattice
    // (probe 64: every tile into 8 slabs; probe >> 12 = R > 0: into a ring of R tile slots)
    // aligned slots (WN > RN: every slot and component run starts on a 128-B
    // line): the whole run is written, zeros off the lattice, so every line
    // leaves L2 written whole by one workgroup -- no partially written lines
    // for the memory side to merge
    const int WN = g.WN;
    const bool whole = WN != RN;
    double *dst = ws + ((probe & 64) ? (t & 7) : (probe >> 12) ? t % max(1, probe >> 12) : t) * 3 * (int64_t)WN;
    const unsigned long long *yi = reinterpret_cast<const unsigned long long *>(yl);
    for (int k = (probe & 8) ? WN : threadIdx.x; k < WN; k += NT) {
        const int kc = min(k, RN - 1);
        const int rz = kc / (g.RX * g.RY), rem = kc - rz * g.RX * g.RY, ry = rem / g.RX, rx = rem - ry * g.RX;
        const int gx = ox + rx, gy = oy + ry, gz = tz + rz;
        const bool lat = k < RN && gx >= 0 && gx < g.Lx && gy >= 0 && gy < g.Ly && gz < g.Lz + g.hp;
        if (!lat && !whole) continue;
        const bool own = rx >= g.PX && rx < g.PX + SYM_TX && ry >= g.PY && ry < g.PY + TY && rz < TZ;
        const int sl = (rx - g.PX) + SYM_TX * ((ry - g.PY) + TY * rz);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            double v = DET ? fx_to_d(yi[b * RS + kc]) * invS : yl[b * RS + kc];
            if (own) v += yd[b * TR + sl];
            if (!lat) v = 0.0;
            if (probe & 32)
                __builtin_nontemporal_store(v, dst + b * WN + k);
            else
                pst(dst + b * WN + k, v, stpol);
        }
    }
    KLE_PROBE_TS_END(t, ts0, ts1, ts2)
}

// W_t of the DET symmetric SpMV, once per build: for each region node j of
// tile t the sum, over the tile's rows i with j in i's stored (upper) blocks
// and j != i, of max_b sum_a |B_ij[a][b]| (so |sum_i B_ij^T x_i|_inf <= that
// sum * max_i |x_i|_inf); tile_e[t] = e with 2^e > max_j of it (frexp).
// Fixed summation order: the scale, and so y, is the same in every run.
__global__ __launch_bounds__(256) void k_sym_bound(SymGeo g, const int *__restrict__ rowbox,
                                                   const int64_t *__restrict__ svptr,
                                                   const double *__restrict__ sval, int *__restrict__ tile_e)
{
    constexpr int TRM = 128;  // rows of a tile
    const int TR = SYM_TX * g.TY * g.TZ;
    __shared__ int sb[TRM], sd[TRM];
    __shared__ int64_t so[TRM];
    __shared__ double wred[256];
    const int64_t t = blockIdx.x;
    const int tix = (int)(t % g.ntx);
    const int64_t q = t / g.ntx;
    const int tiy = (int)(q % g.nty), tz = (int)(q / g.nty) * g.TZ;
    const int x0 = tix * SYM_TX, y0 = tiy * g.TY, ox = x0 - g.PX, oy = y0 - g.PY;
    const int64_t Lxy = (int64_t)g.Lx * g.Ly;
    for (int r = threadIdx.x; r < TR; r += 256) {
        const int xi = x0 + (r & 7), yi = y0 + (r >> 3) % g.TY, zi = tz + r / (SYM_TX * g.TY);
        sd[r] = 0;
        if (xi < g.Lx && yi < g.Ly && zi < g.Lz) {
            const int64_t i = xi + (int64_t)g.Lx * yi + Lxy * zi;
            sb[r] = rowbox[2 * i];
            sd[r] = rowbox[2 * i + 1];
            so[r] = svptr[i];
        }
    }
    __syncthreads();
    const int RN = g.RX * g.RY * g.RZ;
    double wm = 0.0;
    for (int k = threadIdx.x; k < RN; k += 256) {
        const int rz = k / (g.RX * g.RY), rem = k - rz * g.RX * g.RY, ry = rem / g.RX, rx = rem - ry * g.RX;
        const int gx = ox + rx, gy = oy + ry, gz = tz + rz;
        if (gx < 0 || gx >= g.Lx || gy < 0 || gy >= g.Ly || gz >= g.Lz + g.hp) continue;
        double s = 0.0;
        for (int r = 0; r < TR; ++r) {
            const int d = sd[r];
            if (!d) continue;
            const int64_t base = sb[r];
            const int bze = (int)(base / Lxy), by = (int)((base - bze * Lxy) / g.Lx);
            const int bx = (int)(base - bze * Lxy - (int64_t)by * g.Lx), bz = bze - g.zo;
            const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
            if (gx < bx || gx >= bx + bnx || gy < by || gy >= by + bny || gz < bz || gz >= bz + bnz) continue;
            const int xi = x0 + (r & 7), yi = y0 + (r >> 3) % g.TY, zi = tz + r / (SYM_TX * g.TY);
            const int k0 = (xi - bx) + bnx * ((yi - by) + bny * (zi - bz));
            const int kj = (gx - bx) + bnx * ((gy - by) + bny * (gz - bz));
            if (kj <= k0) continue;
            const int mu = bnx * bny * bnz - k0, kk = kj - k0;
            const double *v = sval + so[r];
            double bmax = 0.0;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                double cs = 0.0;
#pragma unroll
                for (int a = 0; a < 3; ++a) cs += fabs(v[vofs(1, 9, a * 3 + b, kk, mu, mu)]);
                bmax = fmax(bmax, cs);
            }
            s += bmax;
        }
        wm = fmax(wm, s);
    }
    wred[threadIdx.x] = wm;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) wred[threadIdx.x] = fmax(wred[threadIdx.x], wred[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int e = -1000;  // no transposed adds in this tile
        if (wred[0] > 0.0) (void)frexp(wred[0], &e);
        tile_e[t] = e;
    }
}

// y_j = sum of the partials of the tiles whose regions contain row j, in
// ascending (z, y, x) tile order, for the lattice rows [j0, j1) -- owned rows
// and (N > 1) the upper ghost rows, whose sums go to gsend (the reverse halo's
// send buffer, ghost row j at gsend[3 (j - n)]).  The first nrecv entries of y
// add the lower neighbour's sums for them (grecv, its upper ghost rows) last.
// With xdot (one launch over all rows, one rank): also the workgroup's
// partial of (y, x) in dpart[blockIdx.x] -- the CG's (A u, u), summed in a
// fixed order (wave sums, then the 4 waves in order), so the single-reduction
// CG needs no separate dot launch.
template <int TXW, int TY, int TZ>
__global__ __launch_bounds__(256) void k_nb_sym_gather(SymGeo g, const double *__restrict__ ws, double *__restrict__ y,
                                                       double *__restrict__ gsend, const double *__restrict__ grecv,
                                                       int64_t nrecv, int64_t j0, int64_t j1,
                                                       const int *__restrict__ istate, const double *__restrict__ xdot,
                                                       double *__restrict__ dpart)
{
    __shared__ double dred[4];
    // (the reason word: loaded first, tested before the first store -- its
    // round trip overlaps the partials' loads)
    const int stop = istate ? __builtin_amdgcn_readfirstlane(istate[I_REASON]) : 0;
    const int64_t Lxy = (int64_t)g.Lx * g.Ly, n = Lxy * g.Lz;
    const int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= j1 && !xdot) return;
    double dsum = 0.0;
    if (j < j1) {
    const int jz = (int)(j / Lxy), jy = (int)((j - jz * Lxy) / g.Lx), jx = (int)(j - jz * Lxy - (int64_t)jy * g.Lx);
    const int RN = g.RX * g.RY * g.RZ;
    // tiles whose [t*T - P, t*T - P + R) contains the coordinate
    const int x_lo = max(0, (jx + g.PX - g.RX + TXW) / TXW), x_hi = min(g.ntx - 1, (jx + g.PX) / TXW);
    const int y_lo = max(0, (jy + g.PY - g.RY + TY) / TY), y_hi = min(g.nty - 1, (jy + g.PY) / TY);
    const int z_lo = max(0, (jz - g.RZ + TZ) / TZ), z_hi = min(g.ntz - 1, jz / TZ);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int tzi = z_lo; tzi <= z_hi; ++tzi)
        for (int ty = y_lo; ty <= y_hi; ++ty)
            for (int tx = x_lo; tx <= x_hi; ++tx) {
                const int64_t t = ((int64_t)tzi * g.nty + ty) * g.ntx + tx;
                const int r = (jx - (tx * TXW - g.PX)) + g.RX * ((jy - (ty * TY - g.PY)) + g.RY * (jz - tzi * TZ));
                const double *p = ws + t * 3 * (int64_t)g.WN + r;
                s0 += p[0];
                s1 += p[g.WN];
                s2 += p[2 * g.WN];
            }
    if (stop) return;  // (uniform: the whole workgroup)
    if (j >= n) {
        double *o = gsend + 3 * (j - n);
        o[0] = s0;
        o[1] = s1;
        o[2] = s2;
        return;
    }
    if (3 * j < nrecv) {
        s0 += grecv[3 * j];
        s1 += grecv[3 * j + 1];
        s2 += grecv[3 * j + 2];
    }
    y[3 * j] = s0;
    y[3 * j + 1] = s1;
    y[3 * j + 2] = s2;
    if (xdot) dsum = s0 * xdot[3 * j] + s1 * xdot[3 * j + 1] + s2 * xdot[3 * j + 2];
    }
    if (!xdot || stop) return;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dsum += __shfl_xor(dsum, o, 64);
    if ((threadIdx.x & 63) == 0) dred[threadIdx.x >> 6] = dsum;
    __syncthreads();
    if (threadIdx.x == 0) dpart[blockIdx.x] = ((dred[0] + dred[1]) + dred[2]) + dred[3];
}

// The value array: big_alloc.  0 on success; d_sval is then set (sval_raw
// cleared).
int sval_alloc(kle_mat *A, size_t bytes)
{
    A->sval_raw = nullptr;
    void *p = nullptr;
    const int r = big_alloc(&p, bytes);
    A->d_sval = static_cast<double *>(p);
    return r < 0 ? KLE_ERR_MEM : 0;
}

// A copy of a matrix struct (Mat.duplicate) shares none of A's symmetric
// storage: forget the pointers (without freeing them).
void sym_forget(kle_mat *A)
{
    A->d_sval = nullptr;
    A->sval_raw = nullptr;
    A->sval_cap = 0;
    A->d_svptr = nullptr;
    A->d_sws = nullptr;
    A->d_stile_e = nullptr;
    A->d_sgsend = A->d_sgrecv = nullptr;
    A->d_srow = nullptr;
    A->d_sbp = nullptr;
    A->d_slid = nullptr;
    A->d_sdptr = A->d_sdict = A->d_sgptr = A->d_sgidx = A->d_sglist = nullptr;
    A->gather_rps = 0;
    A->d_sgmask = nullptr;
    A->d_ssingle = nullptr;
    A->d_swptr = nullptr;
    A->sym_wn = 0;
    A->sws_bytes = 0;
    A->sblocks = A->snvals = A->sws_entries = 0;
    A->sym_P = 0;
    A->sym_graph = 0;
    brick_forget(A);
}

void sym_drop(kle_mat *A)
{
    brick_drop(A);
    for (void *q : {A->sval_raw ? A->sval_raw : (void *)A->d_sval, (void *)A->d_svptr, (void *)A->d_sws, (void *)A->d_stile_e,
                    (void *)A->d_sgsend, (void *)A->d_sgrecv, (void *)A->d_srow, (void *)A->d_sbp,
                    (void *)A->d_slid, (void *)A->d_sdptr, (void *)A->d_sdict, (void *)A->d_sgptr,
                    (void *)A->d_sgidx, (void *)A->d_sgmask, (void *)A->d_ssingle, (void *)A->d_sglist,
                    (void *)A->d_swptr})
        if (q) (void)hipFree(q);
    sym_forget(A);
}

// ---------------------------------------------------------------------------
// Symmetric storage of an unstructured (graph-numbered) 3x3 matrix, one rank.
// The columns are streamed (bcol ascending per row; node ids in Hilbert order,
// kle_umesh.cpp), so the upper triangle j >= i of row i is the tail of its
// column list from the diagonal block on.  Rows go in groups of G
// consecutive rows, one wave per row.  A group's dictionary is the sorted set
// of its stored blocks' columns; every one is >= the group's first row, so
// positions 0 .. G-1 are the group's own rows.  The dictionary serves both
// uses of a block: x_j is read from LDS at the block's 2-byte position and
// B^T x_i is added to the partial sum at that same position.  The workgroup
// writes one partial per dictionary entry (its rows' direct sums included) and
// k_nb_gsym_gather sums, per row, the partials of the dictionary entries that
// name it, in ascending group order.  HBM per SpMV: the stored values once
// (half of the full storage), 2 B per stored block, the dictionaries, and
// the partials written and read once (~25 entries per row at p = 4).  The
// transposed adds are exact fixed-point sums as in the box kernel (scale per
// group from k_gsym_bound), so y is bitwise reproducible.
constexpr int GSYM_UCAP = 2600;  // dictionary entries per group (LDS: 48 B each)
constexpr int GSYM_CU_WAVES = 32;
constexpr size_t LDS_PER_CU_G = 163840;  // the first launch's LDS budget: this many waves per CU
constexpr int GSYM_FILL = 2;  // x-fill entries per thread and batch (3 x 196 entries per group on average)

// kle_mat.hip xcd_block: runs of ch consecutive groups per XCD

// Copy each row's upper tail (from the diagonal block k0 on) into the
// symmetric layout and measure max |B_ij - B_ji^T| per row over all its
// off-diagonal blocks; a block whose partner (j, i) is not in the pattern must
// be zero (it is then dropped from the product with nothing lost).
__global__ __launch_bounds__(256) void k_gsym_check(int64_t nrows, int64_t glo, const int *__restrict__ rowptr,
                                                    const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr,
                                                    const int *__restrict__ bcol, const double *__restrict__ val,
                                                    const int *__restrict__ sk0, const int64_t *__restrict__ svptr,
                                                    double *__restrict__ sval, double *__restrict__ rowdiff,
                                                    double *__restrict__ rowmax)
{
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= nrows) return;
    const int r0 = rowptr[i], mp = rowptr[i + 1] - r0, m = rowcnt ? rowcnt[i] : mp, k0 = sk0[i], mu = m - k0;
    const double *v = val + vptr[i];
    double *sv = sval + svptr[i];
    double dmax = 0.0, vmax = 0.0;
    for (int kk = lane; kk < mu; kk += 64)
#pragma unroll
        for (int t = 0; t < 9; ++t) sv[vofs(1, 9, t, kk, mu, mu)] = v[vofs(1, 9, t, k0 + kk, m, mp)];
    for (int k = lane; k < m; k += 64) {
        double b[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            b[t] = v[vofs(1, 9, t, k, m, mp)];
            vmax = fmax(vmax, fabs(b[t]));
        }
        const int64_t j = bcol[r0 + k] - glo;  // (owned rows: 0 .. nrows-1)
        if (j == i || j < 0 || j >= nrows) continue;  // (blocks into ghosts: sym_probe checks them)
        const int s0 = rowptr[j], mpj = rowptr[j + 1] - s0, mj = rowcnt ? rowcnt[j] : mpj;
        int lo = 0, hi = mj - 1, kj = -1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            const int64_t cm = bcol[s0 + mid] - glo;
            if (cm == i) {
                kj = mid;
                break;
            }
            if (cm < i) lo = mid + 1;
            else hi = mid - 1;
        }
        if (kj < 0) {
#pragma unroll
            for (int t = 0; t < 9; ++t)
                if (b[t] != 0.0) dmax = INFINITY;  // (i, j) without (j, i)
            continue;
        }
        const double *vj = val + vptr[j];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) dmax = fmax(dmax, fabs(b[a * 3 + c] - vj[vofs(1, 9, c * 3 + a, kj, mj, mpj)]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        dmax = fmax(dmax, __shfl_xor(dmax, o, 64));
        vmax = fmax(vmax, __shfl_xor(vmax, o, 64));
    }
    if (lane == 0) {
        rowdiff[i] = dmax;
        rowmax[i] = vmax;
    }
}

// Per group: gexp[g] = e with 2^e > the largest, over its dictionary entries
// e, of the sum over the group's rows of max_b sum_a |B[a][b]| of the block
// whose transposed part adds to e (k_sym_bound's bound; fixed order).
__global__ __launch_bounds__(256) void k_gsym_bound(int64_t nrows, int G, const int *__restrict__ dptr,
                                                    const int *__restrict__ smu, const int64_t *__restrict__ sbp,
                                                    const uint16_t *__restrict__ slid,
                                                    const int64_t *__restrict__ svptr,
                                                    const double *__restrict__ sval, int *__restrict__ gexp)
{
    __shared__ double wred[256];
    const int64_t g = blockIdx.x;
    const int d0 = dptr[g], U = dptr[g + 1] - d0;
    const int nr = (int)min<int64_t>(G, nrows - g * G);
    double wm = 0.0;
    for (int e = threadIdx.x; e < U; e += 256) {
        double s = 0.0;
        for (int r = 0; r < nr; ++r) {
            if (e == r) continue;  // (the row's own diagonal block)
            const int64_t i = g * G + r;
            const int mu = smu[i];
            const uint16_t *l = slid + sbp[i];
            int lo = 0, hi = mu - 1, kk = -1;
            while (lo <= hi) {
                const int mid = (lo + hi) >> 1, p = l[mid];
                if (p == e) {
                    kk = mid;
                    break;
                }
                if (p < e) lo = mid + 1;
                else hi = mid - 1;
            }
            if (kk < 0) continue;
            const double *v = sval + svptr[i];
            double bmax = 0.0;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                double cs = 0.0;
#pragma unroll
                for (int a = 0; a < 3; ++a) cs += fabs(v[vofs(1, 9, a * 3 + b, kk, mu, mu)]);
                bmax = fmax(bmax, cs);
            }
            s += bmax;
        }
        wm = fmax(wm, s);
    }
    wred[threadIdx.x] = wm;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) wred[threadIdx.x] = fmax(wred[threadIdx.x], wred[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int e = -1000;  // no transposed adds in this group
        if (wred[0] > 0.0) (void)frexp(wred[0], &e);
        gexp[g] = e;
    }
}

// y = A x, pass 1: one workgroup of WV waves per group of G rows, wave w
// takes rows w, w + WV, ... (G / WV rows, one after the other).  The launch
// runs the groups of glist[] (groups whose dictionaries fit its US slots).
// LDS: x of the dictionary [U][3] | transposed partials [3][US + 64] (DET:
// int64; 64 dummy slots per component take the adds of masked lanes) |
// direct row sums [G][3].
template <bool DET, int G, int WV>
__global__ __launch_bounds__(64 * WV) void k_nb_spmv_gsym(
    int64_t nrows, int64_t nlist, const int *__restrict__ glist, int US, const int64_t *__restrict__ svptr,
    const int *__restrict__ smu, const int64_t *__restrict__ sbp, const uint16_t *__restrict__ slid,
    const int *__restrict__ dptr, const int *__restrict__ dict, const int *__restrict__ wptr,
    const double *__restrict__ sval, const double *__restrict__ x, double *__restrict__ ws,
    const int *__restrict__ gexp,
    const int *__restrict__ istate, int xcd_chunk, int stpol KLE_PROBE_PARAM)
{
    KLE_PROBE_CONST
    extern __shared__ double lds[];
    // (the reason word: loaded first, tested after the x fill -- nothing is
    // written to memory before that)
    const int stop = istate ? istate[I_REASON] : 0;
    constexpr int NT = 64 * WV, RW = G / WV;
    const int64_t blk = gsym_block(xcd_chunk);
    if (blk >= nlist) return;  // whole workgroup
    KLE_PROBE_TS(ts0)
    const int64_t g = glist[blk];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int d0 = dptr[g], U = dptr[g + 1] - d0, RS = US + 64;
    const int nr = (int)min<int64_t>(G, nrows - g * G);
    double *xs = lds, *yl = lds + 3 * US, *yd = yl + 3 * RS;
    // x of the dictionary in batches of GSYM_FILL entries per thread: the id
    // loads in flight, then the x loads
    for (int f0 = (probe & 4) ? 3 * U : 0; f0 < 3 * U; f0 += GSYM_FILL * NT) {  // (probe 4: no x fill)
        int id[GSYM_FILL];
#pragma unroll
        for (int f = 0; f < GSYM_FILL; ++f) {
            const int t = min(threadIdx.x + f0 + f * NT, 3 * U - 1);
            id[f] = dict[d0 + t / 3];
        }
        double xv[GSYM_FILL];
#pragma unroll
        for (int f = 0; f < GSYM_FILL; ++f) {
            const int t = min(threadIdx.x + f0 + f * NT, 3 * U - 1);
            xv[f] = x[(int64_t)id[f] * 3 + (t - 3 * (t / 3))];
        }
#pragma unroll
        for (int f = 0; f < GSYM_FILL; ++f) {
            const int t = threadIdx.x + f0 + f * NT;
            if (t < 3 * U) xs[t] = xv[f];
        }
    }
    for (int t = threadIdx.x; t < 3 * RS; t += NT) yl[t] = 0.0;  // (0.0 is int64 0)
    if (threadIdx.x < 3 * G) yd[threadIdx.x] = 0.0;
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(stop) != 0) return;
    KLE_PROBE_TS(ts1)
    double S = 1.0, invS = 1.0;
    if (DET) {
        // max |x_i| over the group's rows: dictionary positions 0 .. nr-1
        double m = 0.0;
        int bad = 0;
        for (int r = lane; r < 3 * nr; r += 64) {
            const double a = fabs(xs[r]);
            bad |= !(a <= 1.7976931348623157e308);
            m = fmax(m, a);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
        if (__ballot(bad)) {
            S = 0.0;  // non-finite x: NaN partials, as a floating-point sum would give
            invS = __builtin_nan("");
        } else if (m > 0.0) {
            int em;
            (void)frexp(m, &em);
            const int E = min(max(gexp[g] + em, -960), 1020);
            S = ldexp(1.0, 61 - E);
            invS = ldexp(1.0, E - 61);
        }
    }
    unsigned long long *yi = reinterpret_cast<unsigned long long *>(yl);
    // B x_j into the row's sum, B^T x_i into position l (lanes past the row's
    // end and the diagonal block add into their dummy slot)
    auto sum_item = [&](const double *vv, int l, int k, int mu, double xi0, double xi1, double xi2, double &acc0,
                        double &acc1, double &acc2) {
        const bool on = k < mu;
        const double x0 = xs[3 * l], x1 = xs[3 * l + 1], x2 = xs[3 * l + 2];
        const double s0 = vv[0] * x0 + vv[1] * x1 + vv[2] * x2;
        const double s1 = vv[3] * x0 + vv[4] * x1 + vv[5] * x2;
        const double s2 = vv[6] * x0 + vv[7] * x1 + vv[8] * x2;
        acc0 += on ? s0 : 0.0;
        acc1 += on ? s1 : 0.0;
        acc2 += on ? s2 : 0.0;
        const double t0 = vv[0] * xi0 + vv[3] * xi1 + vv[6] * xi2;
        const double t1 = vv[1] * xi0 + vv[4] * xi1 + vv[7] * xi2;
        const double t2 = vv[2] * xi0 + vv[5] * xi1 + vv[8] * xi2;
        const int rt = on && k > 0 ? l : US + lane;
        if (probe & 1) {
            if (!on) yd[lane] = t0 + t1 + t2;  // (probe 1: no transposed adds)
        } else if (DET) {
            atomicAdd(&yi[rt], fx_of(t0, S));
            atomicAdd(&yi[RS + rt], fx_of(t1, S));
            atomicAdd(&yi[2 * RS + rt], fx_of(t2, S));
        } else {
            atomicAdd(&yl[rt], t0);
            atomicAdd(&yl[RS + rt], t1);
            atomicAdd(&yl[2 * RS + rt], t2);
        }
    };
    for (int rr = 0; rr < RW; ++rr) {
        const int pos = w + WV * rr;  // the row's position in the group (and its dictionary)
        if (pos >= nr) break;
        const int64_t i = g * G + pos;
        const int mu = smu[i], q16 = mu & ~15;
        const double *v = sval + svptr[i];
        const uint16_t *lr = slid + sbp[i];
        const double xi0 = xs[3 * pos], xi1 = xs[3 * pos + 1], xi2 = xs[3 * pos + 2];
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
        for (int kb = (probe & 128) ? mu : 0; kb < mu; kb += 64) {  // (probe 128: no item loop)
            // the values of one 64-block pass (lanes past the row's end re-read
            // its last block; their products are masked) and the blocks' positions
            const int k = kb + lane, kk = min(k, mu - 1);
            const bool ch = kk < q16;
            const int o0 = ch ? (kk >> 4) * 144 + (kk & 15) : q16 * 9 + (kk - q16);
            const int st = ch ? 16 : mu - q16;
            double vv[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) vv[t] = __builtin_nontemporal_load(v + o0 + t * st);
            const int l = __builtin_nontemporal_load(lr + kk);
            sum_item(vv, l, k, mu, xi0, xi1, xi2, acc0, acc1, acc2);
        }
        wsum3_dpp(acc0, acc1, acc2);  // fixed order, one writer per row
        if (lane < 3) yd[3 * pos + lane] = lane == 0 ? acc0 : lane == 1 ? acc1 : acc2;
    }
    __syncthreads();
    KLE_PROBE_TS(ts2)
    // one partial per dictionary entry, [entry][3] (coalesced), from the
    // group's slot start wptr[g]; aligned slots (spmv_sym_align: 128-B slot
    // starts) are written to the end of their last line, zeros past the
    // entries, so every line leaves L2 written whole by one workgroup
    // (probe 64: into 8 slabs; probe >> 12 = R > 0: into a ring of R group slots)
    const int64_t w0 = wptr[g];
    const int nw = (int)(wptr[g + 1] - w0);
    double *dst = ws + ((probe & 64) ? (g & 7) * 3 * 2048 : (probe >> 12) ? (g % max(1, probe >> 12)) * 3 * 2048 : w0);
    for (int t = (probe & 8) ? nw : threadIdx.x; t < nw; t += NT) {  // (probe 8: no partial stores)
        const int tc = min(t, 3 * U - 1);
        const int e = tc / 3, c = tc - 3 * e;
        double s = DET ? fx_to_d(yi[c * RS + e]) * invS : yl[c * RS + e];
        if (e < G) s += yd[tc];
        if (t >= 3 * U) s = 0.0;
        if (probe & 32)
            __builtin_nontemporal_store(s, dst + t);  // (probe 32: nontemporal partial stores)
        else
            pst(dst + t, s, stpol);
    }
    KLE_PROBE_TS_END(g, ts0, ts1, ts2)
}

// y_j = the partials of the dictionary entries naming row j, ascending group
// order.  A wave takes a slice of 64 consecutive rows.  Each group's
// dictionary is sorted, so its entries that name rows of the slice are one
// contiguous run of its partials; a run is stored as (first entry, 64-bit
// mask of the slice rows it names), the runs of a slice in ascending group
// order.  Lane j adds the run's entry popcount(mask below j) when its bit is
// set: the wave's loads of a run are one contiguous stretch of partials
// (instead of one scattered 24-B read per row and entry), and each row still
// sums its entries in ascending group order.  With xdot: the workgroup's
// partial of (y, x) in dpart[blockIdx.x] (k_nb_sym_gather's fixed order).
// N > 1: the rows past the owned ones (nrows .. ntot-1) are the upper ghost
// nodes, whose sums go to gsend (the reverse halo's send buffer).
// WPS waves per slice (a workgroup: 4 slices, 256 WPS threads): wave q of a
// slice sums the q-th WPS-th of its runs, and the slice's first wave adds
// the WPS parts in order through LDS -- small parts have many short runs per
// slice (a 1/8 slab about 21), whose loads one wave would chain.  The loads
// that do not depend on the runs (runptr, the row's direct sum in y, xdot, a
// one-block row's block and x) go out first.
template <int WPS>
__global__ __launch_bounds__(256 * WPS) __attribute__((amdgpu_num_sgpr(64))) void k_nb_gsym_gather(int64_t nrows, int64_t ntot, const int *__restrict__ runptr,
                                                        const int *__restrict__ rstart,
                                                        const unsigned long long *__restrict__ rmask,
                                                        const double *__restrict__ ws, double *__restrict__ y,
                                                        double *__restrict__ gsend, const int *__restrict__ istate,
                                                        const double *__restrict__ xdot, double *__restrict__ dpart,
                                                        int preload, int64_t sl0, int64_t sl1,
                                                        const unsigned long long *__restrict__ single,
                                                        const double *__restrict__ sval,
                                                        const int64_t *__restrict__ svptr,
                                                        const double *__restrict__ xs)
{
    __shared__ double dred[4];
    __shared__ double pred[WPS > 1 ? 4 * (WPS - 1) * 3 * 64 : 1];
    const int stop = istate ? __builtin_amdgcn_readfirstlane(istate[I_REASON]) : 0;  // (tested before the first store)
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ws4 = wv / WPS, part = wv - ws4 * WPS;  // (slice of the workgroup, part of its runs)
    const int64_t sl = sl0 + (int64_t)blockIdx.x * 4 + ws4;
    const int64_t j = sl * 64 + lane;
    const bool on = sl < sl1 && sl * 64 < ntot;  // (the slices [sl0, sl1) of this launch)
    const bool lead = part == 0;
    double dsum = 0.0;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    bool one = false;
    double d0 = 0.0, d1 = 0.0, d2 = 0.0, e0 = 0.0, e1 = 0.0, e2 = 0.0;
    if (on) {
        int rb = runptr[sl];
        const int re = runptr[sl + 1];
        // (the first wave: the row's own terms, independent of the runs)
        if (lead && j < nrows) {
            one = single && sl < (nrows + 63) / 64 && ((single[sl] >> lane) & 1ull);
            if (one) {
                // (box bricks: a row of one stored block is no item of its
                // brick; its direct sum B_ii x_i here, the expression the
                // brick kernel evaluates -- the same bits)
                const double *v = sval + svptr[j];
                const double x0 = xs[3 * j], x1 = xs[3 * j + 1], x2 = xs[3 * j + 2];
                d0 = v[0] * x0 + v[1] * x1 + v[2] * x2;
                d1 = v[3] * x0 + v[4] * x1 + v[5] * x2;
                d2 = v[6] * x0 + v[7] * x1 + v[8] * x2;
            } else if (preload) {  // (the rows' direct sums are in y)
                d0 = y[3 * j];
                d1 = y[3 * j + 1];
                d2 = y[3 * j + 2];
            }
            if (xdot) {
                e0 = xdot[3 * j];
                e1 = xdot[3 * j + 1];
                e2 = xdot[3 * j + 2];
            }
        }
        int r1 = re;
        if constexpr (WPS > 1) {
            const int cnt = re - rb;
            r1 = rb + (cnt * (part + 1)) / WPS;
            rb += (cnt * part) / WPS;
        }
        const unsigned long long below = (1ull << lane) - 1ull;
        // (loads unconditional -- absent lanes re-read the run's first entry --
        // so the unrolled runs' loads are all in flight before the adds)
#pragma unroll 8
        for (int r = rb; r < r1; ++r) {
            const unsigned long long m = rmask[r];
            const bool in = (m >> lane) & 1ull;
            const double *p = ws + (int64_t)rstart[r] + (in ? 3 * __popcll(m & below) : 0);
            const double a0 = p[0], a1 = p[1], a2 = p[2];
            s0 += in ? a0 : 0.0;
            s1 += in ? a1 : 0.0;
            s2 += in ? a2 : 0.0;
        }
    }
    if constexpr (WPS > 1) {
        // the parts in order: the first wave's own, then parts 1 .. WPS-1
        if (!lead) {
            double *q = pred + ((ws4 * (WPS - 1) + part - 1) * 3) * 64 + lane;
            q[0] = s0;
            q[64] = s1;
            q[128] = s2;
        }
        __syncthreads();
        if (lead) {
#pragma unroll
            for (int pp = 1; pp < WPS; ++pp) {
                const double *q = pred + ((ws4 * (WPS - 1) + pp - 1) * 3) * 64 + lane;
                s0 += q[0];
                s1 += q[64];
                s2 += q[128];
            }
        }
    }
    if (stop) return;  // (uniform: the whole workgroup)
    if (on && lead) {
        if (j < nrows) {
            s0 += d0;
            s1 += d1;
            s2 += d2;
            y[3 * j] = s0;
            y[3 * j + 1] = s1;
            y[3 * j + 2] = s2;
            if (xdot) dsum = s0 * e0 + s1 * e1 + s2 * e2;
        } else if (j < ntot) {
            double *o = gsend + 3 * (j - nrows);
            o[0] = s0;
            o[1] = s1;
            o[2] = s2;
        }
    }
    if (!xdot) return;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dsum += __shfl_xor(dsum, o, 64);
    if (lane == 0 && lead) dred[ws4] = dsum;
    __syncthreads();
    if (threadIdx.x == 0) dpart[blockIdx.x] = ((dred[0] + dred[1]) + dred[2]) + dred[3];
}

// y[0 .. n) += r: the reverse halo's sums for a slab's lowest nodes
__global__ void k_axpy_first(int64_t n, const double *__restrict__ r, double *__restrict__ y,
                             const int *__restrict__ istate)
{
    if (istate && istate[I_REASON] != 0) return;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) y[t] += r[t];
}

// y[idx[q]] += the reverse halo's sums rbuf[q] (3 entries per node), one
// launch per lower peer in ascending rank order (fixed order per row)
__global__ void k_gsym_unpack(int64_t cnt, const int32_t *__restrict__ idx, const double *__restrict__ rbuf,
                              double *__restrict__ y, const int *__restrict__ istate)
{
    if (istate && istate[I_REASON] != 0) return;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 3 * cnt) return;
    const int64_t q = t / 3;
    y[3 * (int64_t)idx[q] + (t - 3 * q)] += rbuf[t];
}

static size_t gsym_lds(int US, int G) { return (size_t)(3 * US + 3 * (US + 64) + 3 * G) * sizeof(double); }

static int any_rank(kle_ctx *c, int64_t flag, bool &any);
static int sym_probe(kle_mat *A, double vmax_all, bool &bad);

// Build the graph symmetric storage: one rank, or a graph partition (the ext
// columns [lower ranks' ghosts | owned | higher ranks' ghosts], node ids in
// rank order, so an owned row's upper triangle holds owned columns from its
// own on and every upper ghost, never a lower ghost).  Refuses a matrix that
// is not symmetric to 1e-12 of its largest entry, whose pattern holds a
// nonzero block without its partner, or whose group dictionaries exceed the
// LDS.  Collective at N > 1: every rank takes the same decision (any_rank),
// and one hashed product through both storages checks the blocks between
// ranks (sym_probe).
// Graph bricks: contiguous row ranges (Hilbert order: spatially compact) of
// about equal cost -- a row costs its 64-block passes, each as if full (the
// box bricks' measured cost model, kle_brick_plan.cpp row_cost) -- one per CU,
// or k per CU (up to 8) until every range's dictionary (its rows, then the
// upper-triangle columns past them) fits GB_UCAP LDS entries.  false: none
// fits (the 64-row groups are used).
static bool gbrick_ranges(int64_t n, int64_t glo, int64_t ntot, const std::vector<int> &rp,
                          const std::vector<int> &cnt, const std::vector<int> &bcol, const std::vector<int> &k0,
                          const std::vector<int> &smu, int ncu, std::vector<int64_t> &gst)
{
    if (n <= 0) return false;
    std::vector<double> P(n + 1, 0.0);
    // (a row of one stored block costs nothing when the gather forms it)
    for (int64_t i = 0; i < n; ++i)
        P[i + 1] = P[i] + (g_tune.spmv_brick_singles && smu[i] == 1 ? 0.0 : 4608.0 * ((smu[i] + 63) / 64));
    std::vector<int> mark(std::max<int64_t>(ntot, 1), -1);
    int stamp = 0;
    // k bricks per CU (whole rounds of ncu bricks: a partial last round would
    // leave CUs idle for one brick's time); the largest dictionary of k
    auto umax_of = [&](int k, std::vector<int64_t> &st) {
        const int NB = k * ncu;
        st.assign(1, 0);
        for (int q = 1; q < NB; ++q) {
            const double t = P[n] * q / NB;
            const int64_t r = std::lower_bound(P.begin(), P.end(), t) - P.begin();
            if (r > st.back() && r < n) st.push_back(r);
        }
        st.push_back(n);
        const int nb = (int)st.size() - 1;
        int umax = 0;
        for (int q = 0; q < nb && umax <= GB_UCAP; ++q) {
            const int64_t r0 = st[q], r1 = st[q + 1];
            int u = (int)(r1 - r0);
            ++stamp;
            for (int64_t i = r0; i < r1; ++i)
                for (int kk = rp[i] + k0[i]; kk < rp[i] + cnt[i]; ++kk) {
                    const int64_t col = bcol[kk] - glo;
                    if (col >= r1 && mark[col] != stamp) {
                        mark[col] = stamp;
                        ++u;
                    }
                }
            umax = std::max(umax, u);
        }
        return umax;
    };
    // first guess from the 1M-DoF p = 4 mesh (486-row ranges: 3,230 entries);
    // then the fewest whole rounds that fit, at most 64 per CU
    int k = (int)std::max<int64_t>(1, (n + 450LL * ncu - 1) / (450LL * ncu));
    std::vector<int64_t> st;
    if (umax_of(k, st) <= GB_UCAP) {
        gst = st;
        while (k > 1 && umax_of(k - 1, st) <= GB_UCAP) {
            gst = st;
            --k;
        }
        return true;
    }
    for (++k; k <= 64; ++k)
        if (umax_of(k, st) <= GB_UCAP) {
            gst = st;
            return true;
        }
    gst.clear();
    return false;
}

static int gsym_build(kle_mat *A)
{
    kle_ctx *c = A->ctx;
    const int64_t n = A->nrows, glo = A->ghost_lo / 3, nhi = A->ghost_hi / 3;
    const bool dist = c->nranks > 1;
    const bool slab = dist && !A->plan && (A->lo_rank >= 0 || A->hi_rank >= 0);
    const bool graph = dist && A->plan && !A->plan->peers.empty();
    std::string why;
    if (!(A->kind == 0 && A->R == 3 && A->C == 3 && A->vlayout == 1 && A->d_bcol && !A->d_rowbox &&
          A->m_local == A->n_local && n > 0 && A->ghost_lo % 3 == 0 && A->ghost_hi % 3 == 0))
        why = "symmetric storage of an unstructured matrix needs a 3x3 node-block matrix with owned rows";
    else if (slab && (A->send_lo % 3 || A->send_hi % 3))
        why = "symmetric storage: slab halo of partial nodes";
    const int G = g_tune.spmv_gsym_rows;
    const int WV = g_tune.spmv_gsym_waves ? g_tune.spmv_gsym_waves : G >= 64 ? 16 : 8;
    if (why.empty() && !((WV == 8 && G <= 64) || (WV == 16 && G >= 32)))  // (the kernels instantiated in gsym_spmv)
        why = "symmetric storage: " + std::to_string(G) + "-row groups on " + std::to_string(WV) + " waves";
    int64_t ng = (n + G - 1) / G;
    const int64_t ntot = n + nhi, ns = (ntot + 63) / 64;
    std::vector<int> rp, cnt, bcol, k0, smu, usz, dptr(ng + 1, 0), wptr(ng + 1, 0), glist(ng), dict, runptr(ns + 1, 0),
        rstart;
    // one rank: graph bricks (kle_gbrick.hip) -- the groups become one
    // contiguous row range per CU (gst), the rest of the machinery unchanged
    bool gb = g_tune.spmv_gsym_brick && g_tune.spmv_sym_det;
    bool gb_on = false;
    std::vector<int64_t> gst;
    auto gr0 = [&](int64_t g) { return gb_on ? gst[g] : g * G; };
    auto gr1 = [&](int64_t g) { return gb_on ? gst[g + 1] : std::min<int64_t>(n, (g + 1) * G); };
    std::vector<int64_t> svp, sbp;
    std::vector<uint16_t> slid;
    std::vector<unsigned long long> rmask;
    int64_t tot = 0, blocks = 0, E = 0, n1 = 0, n2 = 0, NR = 0, ninner[2] = {0, 0};
    int US = 0, US1 = 0;
    auto analyse = [&]() -> std::string {
        rp.resize(n + 1);
        cnt.resize(n);
        bcol.resize(std::max<int64_t>(A->nblocks, 1));
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(rp.data(), A->d_rowptr, sizeof(int) * (n + 1), hipMemcpyDeviceToHost) != hipSuccess ||
            (A->d_rowcnt && hipMemcpy(cnt.data(), A->d_rowcnt, sizeof(int) * n, hipMemcpyDeviceToHost) != hipSuccess) ||
            hipMemcpy(bcol.data(), A->d_bcol, sizeof(int) * bcol.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return "symmetric storage: pattern copy failed";
        if (!A->d_rowcnt)
            for (int64_t i = 0; i < n; ++i) cnt[i] = rp[i + 1] - rp[i];
        // per row: the diagonal block's position (columns ascending), stored count
        k0.resize(n);
        smu.resize(n);
        svp.resize(n + 1);
        sbp.resize(n + 1);
        for (int64_t i = 0; i < n; ++i) {
            const int *b = bcol.data() + rp[i], *e = b + cnt[i];
            if (!std::is_sorted(b, e)) return "symmetric storage: row " + std::to_string(i) + "'s columns are not ascending";
            const int *d = std::lower_bound(b, e, (int)(glo + i));
            if (d == e || *d != glo + i) return "symmetric storage: row " + std::to_string(i) + " has no diagonal block";
            if (b[cnt[i] - 1] >= glo + ntot) return "symmetric storage: column beyond the ghost range";
            k0[i] = (int)(d - b);
            smu[i] = cnt[i] - k0[i];
            svp[i] = tot;
            sbp[i] = blocks;
            tot += ((int64_t)smu[i] * 9 + 15) & ~int64_t(15);
            blocks += smu[i];
        }
        svp[n] = tot;
        sbp[n] = blocks;
        gb_on = gb && gbrick_ranges(n, glo, ntot, rp, cnt, bcol, k0, smu, std::max(1, c->num_cus), gst);
        ng = gb_on ? (int64_t)gst.size() - 1 : (n + G - 1) / G;
        dptr.assign(ng + 1, 0);
        wptr.assign(ng + 1, 0);
        glist.assign(ng, 0);
        US = US1 = 0;
        n1 = n2 = 0;
        ninner[0] = ninner[1] = 0;
        const int ucap = gb_on ? GB_UCAP : GSYM_UCAP;
        // group dictionaries (threads over groups; ext column ids)
        usz.assign(ng, 0);
        std::vector<std::vector<int>> dl(ng);
        slid.assign(std::max<int64_t>(blocks, 1), 0);
        const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::atomic<bool> big{false};
        auto work = [&](int t) {
            for (int64_t g = t; g < ng; g += nt) {
                const int64_t r0 = gr0(g), r1 = gr1(g);
                std::vector<int> &L = dl[g];
                for (int64_t r = r0; r < r1; ++r)
                    L.insert(L.end(), bcol.begin() + rp[r] + k0[r], bcol.begin() + rp[r] + cnt[r]);
                std::sort(L.begin(), L.end());
                L.erase(std::unique(L.begin(), L.end()), L.end());
                if ((int64_t)L.size() > ucap) {
                    big = true;
                    continue;
                }
                for (int64_t r = r0; r < r1; ++r)
                    for (int k = k0[r]; k < cnt[r]; ++k)
                        slid[sbp[r] + k - k0[r]] =
                            (uint16_t)(std::lower_bound(L.begin(), L.end(), bcol[rp[r] + k]) - L.begin());
                usz[g] = (int)L.size();
            }
        };
        {
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
            for (auto &x : th) x.join();
        }
        if (big) return "symmetric storage: a row group's columns exceed " + std::to_string(ucap) + " LDS slots";
        for (int64_t g = 0; g < ng; ++g) {
            if ((int64_t)dptr[g] + usz[g] > INT_MAX / 3) return "symmetric storage: dictionaries too large";
            dptr[g + 1] = dptr[g] + usz[g];
            US = std::max(US, usz[g]);
            for (int64_t e = 0; e < usz[g] && e < gr1(g) - gr0(g); ++e)
                if (dl[g][e] != glo + gr0(g) + e)  // (cannot happen: the rows lead)
                    return "symmetric storage: group " + std::to_string(g) + " does not lead with its rows";
        }
        E = dptr[ng];
        // the partials' slots (doubles): packed, or each group's from a 128-B line
        for (int64_t g = 0; g < ng; ++g) {
            const int64_t w = g_tune.spmv_sym_align ? ((3 * (int64_t)usz[g] + 15) & ~int64_t(15)) : 3 * (int64_t)usz[g];
            if ((int64_t)wptr[g] + w > INT_MAX) return "symmetric storage: partial slots too large";
            wptr[g + 1] = wptr[g] + (int)w;
        }
        // the launches: groups whose dictionaries fit US4 slots (4 workgroups
        // per CU), then the rest (US = the largest)
        const int lds1 = (int)(LDS_PER_CU_G * WV / GSYM_CU_WAVES);  // 4 workgroups of 8 waves or 2 of 16 per CU
        int US4 = (int)((lds1 / sizeof(double) - 3 * 64 - 3 * G) / 6);
        if (g_tune.spmv_gsym_split > 0) US4 = std::min(US4, g_tune.spmv_gsym_split);
        // inside each launch, the groups that read no ghost column first
        // (N > 1: they run while the halo is in flight)
        auto tier1 = [&](int64_t g) { return US <= US4 || usz[g] <= US4; };
        auto inner = [&](int64_t g) { return dl[g].back() < glo + n; };
        for (int pass = 0; pass < 4; ++pass) {
            const int64_t k0 = n1 + n2;
            for (int64_t g = 0; g < ng; ++g)
                if (tier1(g) == (pass < 2) && inner(g) == (pass % 2 == 0)) glist[n1 + n2++] = (int)g;
            if (pass == 0) ninner[0] = n2;
            if (pass == 1) {
                n1 = n2;
                n2 = 0;
            }
            if (pass == 2) ninner[1] = n2;
            (void)k0;
        }
        for (int64_t g = 0; g < ng; ++g)
            if (tier1(g)) US1 = std::max(US1, usz[g]);
        // gather runs: per 64-node slice of [owned | upper ghosts], the groups
        // naming its nodes in ascending order, each as (first entry, mask)
        dict.assign(std::max<int64_t>(E, 1), 0);
        std::vector<std::vector<std::pair<int, unsigned long long>>> sruns(ns);
        for (int64_t g = 0; g < ng; ++g)
            for (int e = 0; e < usz[g];) {
                const int sl = (int)((dl[g][e] - glo) >> 6), e0 = e;
                unsigned long long m = 0;
                for (; e < usz[g] && ((dl[g][e] - glo) >> 6) == sl; ++e) {
                    dict[dptr[g] + e] = dl[g][e];
                    m |= 1ull << ((dl[g][e] - glo) & 63);
                }
                sruns[sl].push_back({wptr[g] + 3 * e0, m});  // (the run's first partial, in doubles)
            }
        for (int64_t sl = 0; sl < ns; ++sl) {
            if ((int64_t)runptr[sl] + (int64_t)sruns[sl].size() > INT_MAX) return "symmetric storage: gather runs too many";
            runptr[sl + 1] = runptr[sl] + (int)sruns[sl].size();
        }
        NR = runptr[ns];
        rstart.assign(std::max<int64_t>(NR, 1), 0);
        rmask.assign(std::max<int64_t>(NR, 1), 0);
        for (int64_t sl = 0; sl < ns; ++sl)
            for (size_t k = 0; k < sruns[sl].size(); ++k) {
                rstart[runptr[sl] + k] = sruns[sl][k].first;
                rmask[runptr[sl] + k] = sruns[sl][k].second;
            }
        return "";
    };
    if (why.empty()) why = analyse();
    bool any = false;
    if (dist && why.empty() && gb) {
        // every rank runs the same product schedule: bricks everywhere or
        // groups everywhere
        KLE_TRY(any_rank(c, !gb_on, any));
        if (any && gb_on) {
            gb = false;
            why = analyse();
        }
    }
    KLE_TRY(any_rank(c, !why.empty(), any));
    if (any) return fail(KLE_ERR_SUP, "%s", why.empty() ? "symmetric storage refused on another rank" : why.c_str());
    // device arrays; the value copy and the symmetry check
    const int64_t nsend = graph ? (int64_t)A->plan->send_idx.size() * 3 : slab ? A->send_lo : 0;
    int *dk0 = nullptr;
    double *rowdiff = nullptr, *rowmax = nullptr;
    const bool nomem =
        hipMalloc(&A->d_svptr, sizeof(int64_t) * (n + 1)) != hipSuccess ||
        sval_alloc(A, sizeof(double) * std::max<int64_t>(tot, 1)) != 0 ||
        hipMalloc(&A->d_srow, sizeof(int) * n) != hipSuccess || hipMalloc(&A->d_sbp, sizeof(int64_t) * (n + 1)) != hipSuccess ||
        hipMalloc(&A->d_slid, sizeof(uint16_t) * slid.size()) != hipSuccess ||
        hipMalloc(&A->d_sdptr, sizeof(int) * (ng + 1)) != hipSuccess ||
        hipMalloc(&A->d_sdict, sizeof(int) * dict.size()) != hipSuccess ||
        hipMalloc(&A->d_sglist, sizeof(int) * ng) != hipSuccess ||
        hipMalloc(&A->d_sgptr, sizeof(int) * (ns + 1)) != hipSuccess ||
        hipMalloc(&A->d_sgidx, sizeof(int) * rstart.size()) != hipSuccess ||
        hipMalloc(&A->d_sgmask, sizeof(unsigned long long) * rmask.size()) != hipSuccess ||
        (A->sws_bytes = sizeof(double) * std::max<int64_t>(wptr[ng], 1),
         hipMalloc(&A->d_sws, A->sws_bytes) != hipSuccess) ||
        hipMalloc(&A->d_swptr, sizeof(int) * (ng + 1)) != hipSuccess ||
        hipMalloc(&A->d_stile_e, sizeof(int) * ng) != hipSuccess || hipMalloc(&dk0, sizeof(int) * n) != hipSuccess ||
        (nhi && hipMalloc(&A->d_sgsend, sizeof(double) * 3 * nhi) != hipSuccess) ||
        (nsend && hipMalloc(&A->d_sgrecv, sizeof(double) * nsend) != hipSuccess) ||
        (graph && !A->plan->d_send_idx && !A->plan->send_idx.empty() &&
         hipMalloc(&A->plan->d_send_idx, sizeof(int32_t) * A->plan->send_idx.size()) != hipSuccess) ||
        hipMalloc(&rowdiff, sizeof(double) * n) != hipSuccess || hipMalloc(&rowmax, sizeof(double) * n) != hipSuccess;
    (void)hipGetLastError();
    auto done = [&](int rc) {  // the temporaries go; A's storage too on failure
        for (void *q : {(void *)dk0, (void *)rowdiff, (void *)rowmax})
            if (q) (void)hipFree(q);
        dk0 = nullptr;
        rowdiff = rowmax = nullptr;
        if (rc) sym_drop(A);
        return rc;
    };
    {
        const int rc = any_rank(c, nomem, any);
        if (rc) return done(rc);
    }
    if (any) return done(fail(KLE_ERR_MEM, "out of device memory for symmetric storage"));
    A->sym_graph = 1;
    KLE_TRY(h2d(A->d_svptr, svp.data(), sizeof(int64_t) * (n + 1)));
    KLE_TRY(h2d(A->d_srow, smu.data(), sizeof(int) * n));
    KLE_TRY(h2d(A->d_sbp, sbp.data(), sizeof(int64_t) * (n + 1)));
    KLE_TRY(h2d(A->d_slid, slid.data(), sizeof(uint16_t) * slid.size()));
    KLE_TRY(h2d(A->d_sdptr, dptr.data(), sizeof(int) * (ng + 1)));
    KLE_TRY(h2d(A->d_sdict, dict.data(), sizeof(int) * dict.size()));
    KLE_TRY(h2d(A->d_swptr, wptr.data(), sizeof(int) * (ng + 1)));
    KLE_TRY(h2d(A->d_sglist, glist.data(), sizeof(int) * ng));
    A->gather_rps = (int)((runptr[ns] + ns - 1) / std::max<int64_t>(ns, 1));
    KLE_TRY(h2d(A->d_sgptr, runptr.data(), sizeof(int) * (ns + 1)));
    KLE_TRY(h2d(A->d_sgidx, rstart.data(), sizeof(int) * rstart.size()));
    KLE_TRY(h2d(A->d_sgmask, rmask.data(), sizeof(unsigned long long) * rmask.size()));
    KLE_TRY(h2d(dk0, k0.data(), sizeof(int) * n));
    if (graph && !A->plan->send_idx.empty())
        KLE_TRY(h2d(A->plan->d_send_idx, A->plan->send_idx.data(), sizeof(int32_t) * A->plan->send_idx.size()));
    hipLaunchKernelGGL(k_gsym_check, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, c->stream, n, glo, A->d_rowptr,
                       A->d_rowcnt, A->d_vptr, A->d_bcol, A->d_val, dk0, A->d_svptr, A->d_sval, rowdiff, rowmax);
    KLE_HIP(hipGetLastError());
    std::vector<double> hd(n), hm(n);
    KLE_HIP(hipStreamSynchronize(c->stream));
    KLE_HIP(hipMemcpy(hd.data(), rowdiff, sizeof(double) * n, hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(hm.data(), rowmax, sizeof(double) * n, hipMemcpyDeviceToHost));
    double dmax = 0.0, vmax = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        dmax = std::isnan(hd[i]) ? INFINITY : std::max(dmax, hd[i]);
        vmax = std::max(vmax, hm[i]);
    }
    // the largest entry over all ranks (the tolerances' scale): one-hot sums
    double vmax_all = vmax;
    if (dist) {
        std::vector<int64_t> vb;
        const int rc = allgather_i64(c, (int64_t)std::ilogb(std::max(vmax, 1e-300)), vb);
        if (rc) return done(rc);
        for (int64_t e : vb) vmax_all = std::max(vmax_all, std::ldexp(1.0, (int)e));
    }
    {
        const int rc = any_rank(c, !(dmax <= 1e-12 * vmax_all), any);
        if (rc) return done(rc);
    }
    if (any)
        return done(fail(KLE_ERR_SUP, "matrix is not symmetric (max |A_ij - A_ji| = %g, max |A_ij| = %g)", dmax, vmax));
    if (gb_on) {
        // the bricks' descriptors and per-row (value offset / 16, position
        // offset, stored blocks), then their bounds
        std::vector<GBrickDesc> hb(ng);
        std::vector<int> rowd(4 * (size_t)std::max<int64_t>(n, 1), 0);
        std::vector<unsigned long long> ssm((n + 63) / 64 + 1, 0ull);  // (one-block rows per 64-row slice)
        for (int64_t q = 0; q < ng; ++q) {
            GBrickDesc &B = hb[q];
            const int64_t r0 = gst[q], r1 = gst[q + 1];
            B.r0 = (int)r0;
            B.nr = (int)(r1 - r0);
            B.U = usz[q];
            B.eb = 0;
            B.d0 = dptr[q];
            B.vbase = svp[r0];
            B.sbase = sbp[r0];
            B.wsoff = wptr[q];
            // slots of the brick's rows (value offset / 16, position offset,
            // blocks, the row's dictionary entry); the rows of one stored
            // block go to the gather instead (spmv_brick_singles; box bricks
            // alike), so nr counts the others
            int64_t k = r0;
            for (int64_t i = r0; i < r1; ++i) {
                if (g_tune.spmv_brick_singles && smu[i] == 1) {
                    ssm[i >> 6] |= 1ull << (i & 63);
                    continue;
                }
                rowd[4 * k] = (int)((svp[i] - svp[r0]) / 16);
                rowd[4 * k + 1] = (int)(sbp[i] - sbp[r0]);
                rowd[4 * k + 2] = smu[i];
                rowd[4 * k + 3] = (int)(i - r0);
                ++k;
            }
            B.nr = (int)(k - r0);
        }
        if (hipMalloc(&A->d_bdesc, sizeof(GBrickDesc) * ng) != hipSuccess ||
            hipMalloc(&A->d_browd, sizeof(int) * rowd.size()) != hipSuccess) {
            (void)hipGetLastError();
            return done(fail(KLE_ERR_MEM, "out of device memory for the graph bricks"));
        }
        KLE_TRY(h2d(A->d_bdesc, hb.data(), sizeof(GBrickDesc) * ng));
        KLE_TRY(h2d(A->d_browd, rowd.data(), sizeof(int) * rowd.size()));
        if (g_tune.spmv_brick_singles) {
            if (hipMalloc(&A->d_ssingle, sizeof(unsigned long long) * ssm.size()) != hipSuccess) {
                (void)hipGetLastError();
                A->d_ssingle = nullptr;
                return done(fail(KLE_ERR_MEM, "out of device memory for the graph bricks' one-block rows"));
            }
            KLE_TRY(h2d(A->d_ssingle, ssm.data(), sizeof(unsigned long long) * ssm.size()));
        }
        A->nbricks = (int)ng;
        A->brick_lds_u = US;
        A->brick_lds = (int)brick_lds(US);
        A->sym_gbrick = 1;
        KLE_TRY(gbrick_bound(A, vmax_all));
    } else {
        hipLaunchKernelGGL(k_gsym_bound, dim3((unsigned)ng), dim3(256), 0, c->stream, n, G, A->d_sdptr, A->d_srow,
                           A->d_sbp, A->d_slid, A->d_svptr, A->d_sval, A->d_stile_e);
        KLE_HIP(hipGetLastError());
        KLE_HIP(hipStreamSynchronize(c->stream));
    }
    A->sym_reg[0] = US1;
    A->sym_reg[1] = US;
    A->sym_reg[2] = (int)n1;
    A->sym_reg[3] = G;
    A->sym_reg[4] = WV;
    A->gsym_inner[0] = ninner[0];
    A->gsym_inner[1] = ninner[1];
    A->sblocks = blocks;
    A->snvals = tot;
    A->sws_entries = E;
    if (dist) {
        bool bad = false;
        const int rc = sym_probe(A, vmax_all, bad);
        if (rc) return done(rc);
        if (bad) return done(fail(KLE_ERR_SUP, "matrix is not symmetric across ranks (product probe)"));
    }
    if (const char *e = getenv("KLE_TIMING"))
        if (atoi(e))
            fprintf(stderr, "[kle gsym r%d] rows %lld (+%lld upper ghosts), stored blocks %lld (of %lld), %s %lld, "
                            "dictionary entries %lld (%.2f per row, largest group %d; %lld groups within %d slots), "
                            "gather runs %lld (%.1f per 64 rows)\n",
                    c->rank, (long long)n, (long long)nhi, (long long)blocks, (long long)A->nblocks_real,
                    gb_on ? "bricks" : "groups", (long long)ng, (long long)E, (double)E / n, US, (long long)n1, US1,
                    (long long)NR, (double)NR / ns);
    return done(0);
}

// The run-mask gather over the rows [r0, r1) of [owned | upper ghosts]
// (r0 a multiple of 64; rows past the owned ones go to d_sgsend): per row
// the runs' sums in stored order, plus y first when preload (the rows'
// direct sums).  One workgroup per 4 slices of 64 rows; with xdot, its
// (y, x) partial in dpart[workgroup].
// the gather's waves per 64-row slice: by the runs per slice (a 1/8 slab of
// config 2: about 21 -> 2 waves; config 2: 1), or spmv_gather_wps
static int gather_wps(const kle_mat *A)
{
    return g_tune.spmv_gather_wps ? g_tune.spmv_gather_wps : A->gather_rps >= 8 ? 2 : 1;
}

int gsym_gather(kle_mat *A, double *y, int64_t r0, int64_t r1, const int *istate, const double *xdot, double *dpart,
                int preload, hipStream_t st, const double *xs, int wps_force)
{
    if (r1 <= r0) return 0;
    const int64_t s0 = r0 / 64, s1 = (r1 + 63) / 64, ntot = A->nrows + A->ghost_hi / 3;
    const int wps = wps_force ? wps_force : gather_wps(A);
    auto go = [&](auto kern, int wp) {
        hipLaunchKernelGGL(kern, dim3((unsigned)((s1 - s0 + 3) / 4)), dim3(256 * wp), 0, st, A->nrows, ntot,
                           A->d_sgptr, A->d_sgidx, A->d_sgmask, A->d_sws, y, A->d_sgsend, istate, xdot, dpart,
                           preload, s0, s1, xs ? A->d_ssingle : nullptr, A->d_sval, A->d_svptr, xs);
    };
    if (wps == 4) go(k_nb_gsym_gather<4>, 4);
    else if (wps == 2) go(k_nb_gsym_gather<2>, 2);
    else go(k_nb_gsym_gather<1>, 1);
    KLE_HIP(hipGetLastError());
    return 0;
}

static int gsym_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart)
{
    kle_ctx *c = A->ctx;
    hipStream_t st = c->stream;
    if (A->sym_gbrick && c->nranks == 1) {
        KLE_TRY(gbrick_launch(A, x, y, istate));
        return gsym_gather(A, y->d, 0, A->nrows, istate, dpart ? x->d : nullptr, dpart, 1, st,
                           A->d_ssingle ? x->d : nullptr);
    }
    const int G = A->sym_reg[3], WV = A->sym_reg[4];
    const int64_t n = A->nrows, ng = (n + G - 1) / G, n1 = A->sym_reg[2], nhi = A->ghost_hi / 3;
    const bool dist = c->nranks > 1;
    const bool det = g_tune.spmv_sym_det != 0;
    // N > 1 with overlap: the groups that read no ghost column, then (comm
    // stream) the halo, then the rest; all RCCL calls on the comm stream
    const bool ovl = dist && A->halo_overlap != 0;
    hipStream_t cs = ovl ? c->comm_stream : st;
    auto launch = [&](auto kern, int slot, int64_t l0, int64_t nl, int US) {
        if (nl <= 0) return;
        const size_t lds = gsym_lds(US, G);
        (void)slot;
        dyn_lds(A->ctx, reinterpret_cast<const void *>(kern), lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)nl), dim3(64 * WV), lds, st, n, nl, A->d_sglist + l0, US, A->d_svptr,
                           A->d_srow, A->d_sbp, A->d_slid, A->d_sdptr, A->d_sdict, A->d_swptr, A->d_sval, x->base, A->d_sws,
                           A->d_stile_e, istate, g_tune.spmv_xcd_chunk, g_tune.spmv_gsym_stpol KLE_PROBE_ARG);
    };
    // part 0: the inner groups of both launches, part 1: the others (one
    // rank or no overlap: both parts back to back)
    const int64_t i1 = A->gsym_inner[0], i2 = A->gsym_inner[1];
    auto launch2 = [&](auto kern, int slot, int part) {
        if (part == 0) {
            launch(kern, slot, 0, i1, A->sym_reg[0]);
            launch(kern, slot + 1, n1, i2, A->sym_reg[1]);
        } else {
            launch(kern, slot, i1, n1 - i1, A->sym_reg[0]);
            launch(kern, slot + 1, n1 + i2, ng - n1 - i2, A->sym_reg[1]);
        }
    };
    auto tiles = [&](int part) -> int {
#define GSYM_CASE(GG, WW, SLOT)                                            \
    if (G == GG && WV == WW) {                                             \
        if (det) launch2(k_nb_spmv_gsym<true, GG, WW>, SLOT, part);        \
        else launch2(k_nb_spmv_gsym<false, GG, WW>, SLOT + 2, part);       \
    } else
        GSYM_CASE(8, 8, 0) GSYM_CASE(16, 8, 4) GSYM_CASE(32, 8, 8) GSYM_CASE(32, 16, 12) GSYM_CASE(64, 8, 16)
        GSYM_CASE(64, 16, 20) GSYM_CASE(128, 16, 24) {
#undef GSYM_CASE
            return fail(KLE_ERR_SUP, "symmetric SpMV: %d rows per group on %d waves", G, WV);
        }
        return 0;
    };
    if (A->sym_gbrick) {
        // graph bricks at N > 1: every brick's dictionary may hold ghost
        // columns, so the forward halo first (comm stream with overlap, as
        // the group path's RCCL calls), then the bricks
        if (ovl) {
            KLE_HIP(hipEventRecord(c->ev_x_ready, st));
            KLE_HIP(hipStreamWaitEvent(cs, c->ev_x_ready, 0));
        }
        KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank, x->send_lo,
                              x->send_hi, cs, x->plan.get()));
        if (ovl) {
            KLE_HIP(hipEventRecord(c->ev_halo_done, cs));
            KLE_HIP(hipStreamWaitEvent(st, c->ev_halo_done, 0));
        }
        KLE_TRY(gbrick_launch(A, x, y, istate));
    } else if (!dist) {
        KLE_TRY(tiles(0));
        KLE_TRY(tiles(1));
    } else if (ovl) {
        KLE_HIP(hipEventRecord(c->ev_x_ready, st));
        KLE_HIP(hipStreamWaitEvent(cs, c->ev_x_ready, 0));
        KLE_TRY(tiles(0));
        KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank, x->send_lo,
                              x->send_hi, cs, x->plan.get()));
        KLE_HIP(hipEventRecord(c->ev_halo_done, cs));
        KLE_HIP(hipStreamWaitEvent(st, c->ev_halo_done, 0));
        KLE_TRY(tiles(1));
    } else {
        KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank, x->send_lo,
                              x->send_hi, st, x->plan.get()));
        KLE_TRY(tiles(0));
        KLE_TRY(tiles(1));
    }
    const int64_t ntot = n + (dist ? nhi : 0);
    KLE_TRY(gsym_gather(A, y->d, 0, ntot, istate, dpart && !dist ? x->d : nullptr, dpart, A->sym_gbrick, st,
                        A->sym_gbrick && A->d_ssingle ? x->d : nullptr));
    KLE_HIP(hipGetLastError());
    if (!dist) return 0;
    // the upper ghost nodes' sums back to their owners, added in ascending
    // rank order of the senders (MPISBAIJ's reverse scatter)
    if (ovl) {
        KLE_HIP(hipEventRecord(c->ev_x_ready, st));
        KLE_HIP(hipStreamWaitEvent(cs, c->ev_x_ready, 0));
    }
    if (A->plan && !A->plan->peers.empty()) {
        const HaloPlan &P = *A->plan;
        KLE_TRY(halo_reverse_plan(c, P, A->ghost_lo / 3 + n, 3, A->d_sgsend, A->d_sgrecv, cs));
        if (ovl) {
            KLE_HIP(hipEventRecord(c->ev_halo_done, cs));
            KLE_HIP(hipStreamWaitEvent(st, c->ev_halo_done, 0));
        }
        for (size_t k = 0; k < P.peers.size() && P.peers[k] < c->rank; ++k)
            if (P.send_cnt[k])
                hipLaunchKernelGGL(k_gsym_unpack, dim3((unsigned)((3 * P.send_cnt[k] + 255) / 256)), dim3(256), 0, st,
                                   P.send_cnt[k], P.d_send_idx + P.send_off[k], A->d_sgrecv + 3 * P.send_off[k], y->d,
                                   istate);
    } else {
        const int64_t nrecv = A->lo_rank >= 0 ? A->send_lo : 0;
        KLE_TRY(halo_reverse(c, A->d_sgsend, A->ghost_hi, A->hi_rank, A->d_sgrecv, nrecv, A->lo_rank, cs));
        if (ovl) {
            KLE_HIP(hipEventRecord(c->ev_halo_done, cs));
            KLE_HIP(hipStreamWaitEvent(st, c->ev_halo_done, 0));
        }
        if (nrecv)
            hipLaunchKernelGGL(k_axpy_first, dim3((unsigned)((nrecv + 255) / 256)), dim3(256), 0, st, nrecv,
                               A->d_sgrecv, y->d, istate);
    }
    KLE_HIP(hipGetLastError());
    return 0;
}

static SymGeo sym_geo(const kle_mat *A)
{
    SymGeo g;
    const int P = A->sym_P;
    g.TX = SYM_TX;
    g.TZ = A->sym_TZ;
    g.TY = A->sym_TY;
    g.Lx = (int)A->row_lat[0];
    g.Ly = (int)A->row_lat[1];
    g.Lz = (int)A->row_lat[2];
    const int64_t plane3 = 3 * A->row_lat[0] * A->row_lat[1];
    g.zo = (int)(A->ghost_lo / plane3);
    g.hp = (int)(A->ghost_hi / plane3);
    g.P = P;
    g.PX = A->sym_reg[0];
    g.RX = A->sym_reg[1];
    g.PY = A->sym_reg[2];
    g.RY = A->sym_reg[3];
    g.RZ = A->sym_reg[4];
    g.WN = A->sym_wn > 0 ? A->sym_wn : g.RX * g.RY * g.RZ;
    g.ntx = (g.Lx + g.TX - 1) / g.TX;
    g.nty = (g.Ly + g.TY - 1) / g.TY;
    g.ntz = (g.Lz + g.TZ - 1) / g.TZ;
    return g;
}

// LDS of the x-in-LDS kernel: x and y of the region, the tile's direct row sums
struct SymRegion {
    int PX, RX, PY, RY, RZ;
};

static SymRegion sym_region(const kle_mat *A)
{
    return {A->sym_reg[0], A->sym_reg[1], A->sym_reg[2], A->sym_reg[3], A->sym_reg[4]};
}

static size_t sym_xl_lds(const SymRegion &r)
{
    const size_t RN = (size_t)r.RX * r.RY * r.RZ;
    return (6 * RN + 3 * 64 + 3 * 128) * sizeof(double);
}
constexpr size_t LDS_PER_CU = 163840;

// Waves per workgroup of the x-in-LDS kernel: 8 while two workgroups fit a
// CU's LDS (P <= 4), else 16 (one workgroup of 16 waves per CU);
// kle_set_tuning("spmv_sym_waves") overrides.
// The x fill is one pass of SYM_FILL loads per thread: 16 waves where 8 would
// need more (P >= 5).
static bool sym_fill_fits(const SymRegion &r, int wv)
{
    const int NL = r.RY * r.RZ, fstep = 64 * wv / (3 * r.RX);
    return NL <= SYM_FILL * fstep;
}


// every rank's flag -> whether any rank raised it (one collective; one rank:
// no communication)
static int any_rank(kle_ctx *c, int64_t flag, bool &any)
{
    any = flag != 0;
    if (c->nranks == 1) return 0;
    std::vector<int64_t> all;
    KLE_TRY(allgather_i64(c, flag, all));
    any = false;
    for (int64_t v : all) any |= v != 0;
    return 0;
}

// x_i = uniform[-1, 1) of a splitmix64 hash of the global entry index
__global__ void k_sym_probe_x(int64_t n, int64_t lo, double *__restrict__ x)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint64_t z = 0x5EED5EEDull + (uint64_t)(lo + k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    x[k] = (double)(z >> 11) * 0x1p-52 - 1.0;
}

// N > 1: the stored triangle also feeds other ranks' rows (a block (i, j)
// with j an upper ghost stands in for the neighbour's (j, i)), which
// k_sym_build cannot compare locally.  One product with a hashed x through
// both storages checks it: max |A_full x - A_sym x| <= 1e-12 max |A_ij|, the
// single-rank criterion (a block asymmetric by d changes y by ~d |x_i|).
static int sym_probe(kle_mat *A, double vmax_all, bool &bad)
{
    kle_ctx *c = A->ctx;
    bad = false;
    kle_vec *x = nullptr, *y1 = nullptr, *y2 = nullptr;
    int rc = vec_alloc(c, A->n_local, A->n_global, A->col_lo, A->ghost_lo, A->ghost_hi, &x);
    if (!rc) rc = vec_alloc(c, A->m_local, A->m_global, A->row_lo, 0, 0, &y1);
    if (!rc) rc = vec_alloc(c, A->m_local, A->m_global, A->row_lo, 0, 0, &y2);
    if (!rc) {
        x->bs = A->C;
        x->lo_rank = A->lo_rank;
        x->hi_rank = A->hi_rank;
        x->send_lo = A->send_lo;
        x->send_hi = A->send_hi;
        x->plan = A->plan;
        hipLaunchKernelGGL(k_sym_probe_x, dim3((unsigned)((A->n_local + 255) / 256)), dim3(256), 0, c->stream,
                           A->n_local, A->col_lo, x->d);
        rc = hipGetLastError() == hipSuccess ? 0 : fail(KLE_ERR_DEVICE, "probe launch failed");
    }
    double *sv = A->d_sval;
    if (!rc) {
        A->d_sval = nullptr;  // (the full storage)
        rc = spmv(A, x, y1, nullptr);
        A->d_sval = sv;
    }
    if (!rc) rc = sym_spmv(A, x, y2, nullptr);
    double dmax = 0.0;
    if (!rc) {
        std::vector<double> h1(A->m_local), h2(A->m_local);
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(h1.data(), y1->d, sizeof(double) * A->m_local, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(h2.data(), y2->d, sizeof(double) * A->m_local, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(KLE_ERR_DEVICE, "probe copy failed");
        for (int64_t k = 0; k < A->m_local && !rc; ++k) {
            const double d = std::fabs(h1[k] - h2[k]);
            dmax = std::isnan(d) ? INFINITY : std::max(dmax, d);
        }
    }
    for (kle_vec *v : {x, y1, y2})
        if (v) {
            (void)hipFree(v->base);
            delete v;
        }
    if (rc) return rc;
    // (a flag per rank: an asymmetry anywhere refuses the storage everywhere)
    return any_rank(c, !(dmax <= 1e-12 * vmax_all), bad);
}

// Build the symmetric (upper-triangle) storage of a structured 3x3 matrix
// from its full storage (one rank, or z slabs with lower / upper ghost
// planes).  Refuses a matrix whose blocks are not symmetric to 1e-12 of its
// largest entry or whose pattern is not symmetric.  At N > 1 collective: every
// rank decides the same way (any_rank), so no rank runs the symmetric SpMV
// and its reverse halo while a neighbour runs the full storage.
static int sym_build_impl(kle_mat *A);

// Every error return of the builders, wherever it happens (a refused check,
// a device error between the allocations and the last check), leaves A
// without symmetric storage: no SpMV can run over a half-built copy.
int sym_build(kle_mat *A)
{
    const int rc = sym_build_impl(A);
    if (rc) sym_drop(A);
    return rc;
}

static int sym_build_impl(kle_mat *A)
{
    kle_ctx *c = A->ctx;
    sym_drop(A);
    if (A->kind == 0 && !A->d_rowbox && A->d_bcol) return gsym_build(A);  // unstructured rows
    const int64_t Lx = A->row_lat[0], Ly = A->row_lat[1], Lz = A->row_lat[2], n = A->nrows, Lxy = Lx * Ly;
    std::string why;
    if (!(A->kind == 0 && A->R == 3 && A->C == 3 && A->vlayout == 1 && A->d_rowbox && !A->plan &&
          A->m_local == A->n_local))
        why = "symmetric storage needs a 3x3 node-block matrix with box-lattice rows (one rank or z slabs)";
    else if (Lx * Ly * Lz != n || A->box_lx != Lx || A->box_lxy != Lxy || Lx > INT_MAX / 2 ||
             A->ghost_lo % (3 * Lxy) || A->ghost_hi % (3 * Lxy) || A->send_lo % (3 * Lxy))
        why = "symmetric storage: the rows are not one box lattice with whole ghost planes";
    const int64_t zo = why.empty() ? A->ghost_lo / (3 * Lxy) : 0, hp = why.empty() ? A->ghost_hi / (3 * Lxy) : 0;
    std::vector<int> rb, rp, cnt;
    std::vector<int64_t> sv;
    std::vector<int> srow;  // per row: x-bx, y-by, z-bz, bnx, bny, bnz (4 bits each)
    int P = 0;
    // reach of the rows' upper triangles relative to their tile's origin, per
    // tile shape (0: 8 x 4 x 4, 1: 8 x 8 x 2): x / y low, x / y / z high
    // tile shapes (rows TX x TY x TZ): 8 x 4 x 4, 8 x 8 x 2, and 8 x 2 x 4 (64 rows)
    constexpr int NSH = 3;
    const int shape_ty[NSH] = {4, 8, 2}, shape_tz[NSH] = {4, 2, 4};
    int64_t rlo[NSH][2] = {{0, 0}, {0, 0}, {0, 0}},
            rhi[NSH][3] = {{SYM_TX - 1, 3, 3}, {SYM_TX - 1, 7, 1}, {SYM_TX - 1, 1, 3}};
    int64_t tot = 0, blocks = 0, all = 0, up_ghost = 0, lo_ghost = 0;
    if (why.empty()) {
        rb.resize(2 * n);
        rp.resize(n + 1);
        cnt.resize(n);
        sv.resize(n + 1);
        srow.resize(n);
        KLE_HIP(hipStreamSynchronize(c->stream));
        KLE_HIP(hipMemcpy(rb.data(), A->d_rowbox, sizeof(int) * 2 * n, hipMemcpyDeviceToHost));
        KLE_HIP(hipMemcpy(rp.data(), A->d_rowptr, sizeof(int) * (n + 1), hipMemcpyDeviceToHost));
        if (A->d_rowcnt) KLE_HIP(hipMemcpy(cnt.data(), A->d_rowcnt, sizeof(int) * n, hipMemcpyDeviceToHost));
        else
            for (int64_t i = 0; i < n; ++i) cnt[i] = rp[i + 1] - rp[i];
        for (int64_t i = 0; i < n && why.empty(); ++i) {
            // (x, y, z): the row in column (ext) coordinates
            const int64_t z = i / Lxy + zo, y = (i % Lxy) / Lx, x = i % Lx;
            const int64_t base = rb[2 * i];
            const int d = rb[2 * i + 1];
            const int64_t bz = base / Lxy, by = (base - bz * Lxy) / Lx, bx = base - bz * Lxy - by * Lx;
            const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
            if (x < bx || x >= bx + bnx || y < by || y >= by + bny || z < bz || z >= bz + bnz ||
                cnt[i] != bnx * bny * bnz || bz + bnz > zo + Lz + hp) {
                why = "symmetric storage: row " + std::to_string(i) + "'s box does not hold its diagonal";
                break;
            }
            P = std::max<int>(P, (int)std::max({x - bx, bx + bnx - 1 - x, y - by, by + bny - 1 - y, bz + bnz - 1 - z}));
            if (bnx > 15 || bny > 15 || bnz > 15) {
                why = "symmetric storage: row boxes wider than 15 nodes";
                break;
            }
            srow[i] = (int)((x - bx) | (y - by) << 4 | (z - bz) << 8) | bnx << 12 | bny << 16 | bnz << 20;
            {
                // the upper triangle's extent: the planes above take the
                // whole box, the row's own plane the lines from its own on
                const int64_t uz1 = bz + bnz - 1, uy1 = by + bny - 1, ux1 = bx + bnx - 1;
                const int64_t uy0 = uz1 > z ? by : y, ux0 = uz1 > z || uy1 > y ? bx : x;
                for (int s = 0; s < NSH; ++s) {
                    const int64_t x0 = x / SYM_TX * SYM_TX, y0 = y / shape_ty[s] * shape_ty[s];
                    const int64_t z0 = (z - zo) / shape_tz[s] * shape_tz[s] + zo;
                    rlo[s][0] = std::min(rlo[s][0], ux0 - x0);
                    rlo[s][1] = std::min(rlo[s][1], uy0 - y0);
                    rhi[s][0] = std::max(rhi[s][0], ux1 - x0);
                    rhi[s][1] = std::max(rhi[s][1], uy1 - y0);
                    rhi[s][2] = std::max(rhi[s][2], uz1 - z0);
                }
            }
            const int k0 = (int)((x - bx) + bnx * ((y - by) + (int64_t)bny * (z - bz)));
            const int64_t mu = cnt[i] - k0;
            sv[i] = tot;
            tot += (mu * 9 + 15) & ~int64_t(15);
            blocks += mu;
            all += cnt[i];
            up_ghost += (int64_t)bnx * bny * std::max<int64_t>(0, bz + bnz - std::max<int64_t>(bz, zo + Lz));
            lo_ghost += (int64_t)bnx * bny * std::max<int64_t>(0, std::min<int64_t>(bz + bnz, zo) - bz);
        }
        sv[n] = tot;
        // k_sym_build checks that every stored (i, j) between owned rows has its
        // (j, i); with that, a symmetric pattern holds 2 (upper blocks) - n
        // blocks, less the upper blocks into upper ghosts, plus the blocks into
        // lower ghosts -- a block without its partner shows up here
        if (why.empty() && 2 * blocks - n - up_ghost + lo_ghost != all)
            why = "symmetric storage: the block pattern is not symmetric (" + std::to_string(all) + " blocks, " +
                  std::to_string(blocks) + " upper)";
    }
    // one rank, no ghosts: bricks (kle_brick.hip) -- the values go in brick
    // order, and none of the tile set-up below is needed
    void *bplan = nullptr;
    struct PlanGuard {
        void *&p;
        ~PlanGuard() { brick_plan_free(p); }
    } bguard{bplan};
    // (one rank, or z slabs; every rank takes the same decision)
    if (why.empty() && g_tune.spmv_sym_brick && g_tune.spmv_sym_det && (c->nranks == 1 ? zo == 0 && hp == 0 : !A->plan)) {
        std::string bwhy;
        std::vector<int64_t> svb;
        KLE_TRY(brick_setup(A, rb, cnt, srow, P, svb, bwhy, &bplan));
        bool none = false;
        KLE_TRY(any_rank(c, !bplan, none));
        if (none && bplan) {
            brick_plan_free(bplan);
            bplan = nullptr;
            bwhy = "not on every rank";
        }
        if (bplan) {
            sv.swap(svb);
            tot = std::max<int64_t>(tot, sv[n]);
        }
        else if (const char *e = getenv("KLE_TIMING"))
            if (atoi(e)) fprintf(stderr, "[kle brick r%d] not used: %s\n", c->rank, bwhy.c_str());
    }
    SymRegion reg[NSH];
    for (int s = 0; s < NSH; ++s)
        reg[s] = {(int)-rlo[s][0], (int)(rhi[s][0] - rlo[s][0] + 1), (int)-rlo[s][1], (int)(rhi[s][1] - rlo[s][1] + 1),
                  (int)(rhi[s][2] + 1)};
    if (why.empty() && !bplan && sym_xl_lds(reg[1]) > LDS_PER_CU)
        why = "symmetric storage: row boxes reach " + std::to_string(P) + " nodes (region of " +
              std::to_string(reg[1].RX * reg[1].RY * reg[1].RZ) + " nodes does not fit the LDS)";
    // tile shape: 8 x 4 x 4 rows (default where two workgroups of 8 waves fit
    // a CU: P <= 4) or 8 x 8 x 2 -- the same 128 rows and, at P = 4, the same
    // 1536-node region, but a 4-plane tile spans a whole p = 4 element layer,
    // so every tile holds the same mix of row lengths (rows on element-
    // boundary planes carry 4 planes of upper blocks, the next ones 3, 2, 1)
    // 8 x 2 x 4 (64 rows, still a whole element layer deep): where the
    // 128-row tiles would not fill the chip -- a small part (z slab at N > 1)
    // whose few heavy tiles set the kernel's length (spmv_sym_tile64: 0 auto
    // below spmv_sym_tile64_max 128-row tiles, 1 wherever 8 x 4 x 4 fits, 2 never)
    // (P >= 5, where 8 x 4 x 4 regions do not fit two workgroups per CU, the
    // 64-row tiles still may: forced only, spmv_sym_tile64 1)
    int TZ = g_tune.spmv_sym_tz != 2 && why.empty() && 2 * sym_xl_lds(reg[0]) <= LDS_PER_CU &&
                     sym_fill_fits(reg[0], 8) ? 4 : 2;
    int TY = TZ == 4 ? 4 : 8;
    if (g_tune.spmv_sym_tile64 != 2 && why.empty() && 2 * sym_xl_lds(reg[2]) <= LDS_PER_CU &&
        sym_fill_fits(reg[2], 8)) {
        const int64_t t128 = ((Lx + SYM_TX - 1) / SYM_TX) * ((Ly + 3) / 4) * ((Lz + 3) / 4);
        if (g_tune.spmv_sym_tile64 == 1 || (TZ == 4 && t128 < g_tune.spmv_sym_tile64_max)) {
            TZ = 4;
            TY = 2;
        }
    }
    const SymRegion &rg = reg[TY == 2 ? 2 : TZ == 4 ? 0 : 1];
    bool any = false;
    KLE_TRY(any_rank(c, !why.empty(), any));
    if (any) return fail(KLE_ERR_SUP, "%s", why.empty() ? "symmetric storage refused on another rank" : why.c_str());
    if (c->nranks > 1) {
        // the slab pattern across a cut: my blocks into the upper ghosts are
        // the upper neighbour's blocks into its lower ghosts
        std::vector<int64_t> ups, los;
        KLE_TRY(allgather_i64(c, up_ghost, ups));
        KLE_TRY(allgather_i64(c, lo_ghost, los));
        bool bad = false;
        if (A->hi_rank >= 0 && ups[c->rank] != los[A->hi_rank]) bad = true;
        if (A->lo_rank >= 0 && los[c->rank] != ups[A->lo_rank]) bad = true;
        KLE_TRY(any_rank(c, bad, any));
        if (any) return fail(KLE_ERR_SUP, "symmetric storage: the block pattern is not symmetric across ranks");
    }
    double *rowdiff = nullptr, *rowmax = nullptr;
    int64_t nomem = 0;
    if (hipMalloc(&A->d_svptr, sizeof(int64_t) * (n + 1)) != hipSuccess ||
        hipMalloc(&A->d_srow, sizeof(int) * std::max<int64_t>(n, 1)) != hipSuccess ||
        sval_alloc(A, sizeof(double) * std::max<int64_t>(tot, 1)) != 0 ||
        hipMalloc(&rowdiff, sizeof(double) * n) != hipSuccess || hipMalloc(&rowmax, sizeof(double) * n) != hipSuccess)
        nomem = 1;
    double dmax = 0.0, vmax = 0.0;
    if (!nomem) {
        KLE_TRY(h2d(A->d_svptr, sv.data(), sizeof(int64_t) * (n + 1)));
        KLE_TRY(h2d(A->d_srow, srow.data(), sizeof(int) * n));
        hipLaunchKernelGGL(k_sym_build, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, c->stream, n, (int)Lx, (int)Ly,
                           (int)zo, A->d_rowptr, A->d_rowcnt, A->d_rowbox, A->d_vptr, A->d_val, A->d_svptr, A->d_sval,
                           rowdiff, rowmax);
        KLE_HIP(hipGetLastError());
        std::vector<double> hd(n), hm(n);
        KLE_HIP(hipStreamSynchronize(c->stream));
        KLE_HIP(hipMemcpy(hd.data(), rowdiff, sizeof(double) * n, hipMemcpyDeviceToHost));
        KLE_HIP(hipMemcpy(hm.data(), rowmax, sizeof(double) * n, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < n; ++i) {
            dmax = std::max(dmax, hd[i]);
            vmax = std::max(vmax, hm[i]);
            if (std::isnan(hd[i])) dmax = INFINITY;
        }
    }
    (void)hipGetLastError();
    hipFree(rowdiff);
    hipFree(rowmax);
    // the largest entry over all ranks (the tolerances' scale): one-hot sums
    double vmax_all = vmax;
    if (c->nranks > 1) {
        std::vector<int64_t> vb;
        KLE_TRY(allgather_i64(c, (int64_t)std::ilogb(std::max(vmax, 1e-300)), vb));  // exponents (exact)
        for (int64_t e : vb) vmax_all = std::max(vmax_all, std::ldexp(1.0, (int)e));
    }
    const bool asym = !nomem && !(dmax <= 1e-12 * vmax_all);
    KLE_TRY(any_rank(c, nomem ? 1 : asym ? 2 : 0, any));
    if (any) {
        sym_drop(A);
        if (nomem) return fail(KLE_ERR_MEM, "out of device memory for symmetric storage");
        if (asym)
            return fail(KLE_ERR_SUP, "matrix is not symmetric (max |A_ij - A_ji| = %g, max |A_ij| = %g)", dmax, vmax);
        return fail(KLE_ERR_SUP, "symmetric storage refused on another rank");
    }
    if (bplan) {
        A->sym_P = P;
        A->sblocks = blocks;
        A->snvals = tot;
        void *p = bplan;
        bplan = nullptr;  // (brick_finish owns it)
        int rc = brick_finish(A, p);
        bool any_fail = false;
        if (c->nranks > 1) {
            const int arc = any_rank(c, rc != 0, any_fail);
            if (!rc && arc) rc = arc;
            if (!rc && any_fail) rc = fail(KLE_ERR_MEM, "symmetric storage: bricks failed on another rank");
            if (!rc) {
                bool bad = false;
                rc = sym_probe(A, vmax_all, bad);
                if (!rc && bad) rc = fail(KLE_ERR_SUP, "matrix is not symmetric across ranks (product probe)");
            }
        }
        if (rc) sym_drop(A);
        return rc;
    }
    A->sym_P = P;
    A->sym_TZ = TZ;
    A->sym_TY = TY;
    A->sym_reg[0] = rg.PX;
    A->sym_reg[1] = rg.RX;
    A->sym_reg[2] = rg.PY;
    A->sym_reg[3] = rg.RY;
    A->sym_reg[4] = rg.RZ;
    {
        const int rn = rg.RX * rg.RY * rg.RZ;
        A->sym_wn = g_tune.spmv_sym_align ? (rn + 15) & ~15 : rn;
    }
    const SymGeo g = sym_geo(A);
    const int64_t ntiles = (int64_t)g.ntx * g.nty * g.ntz;
    auto span = [](int64_t o, int64_t r, int64_t L) { return std::max<int64_t>(0, std::min(o + r, L) - std::max<int64_t>(o, 0)); };
    // lattice entries of every tile region (written by the SpMV, read by the gather)
    int64_t ents = 0;
    for (int64_t t = 0; t < g.ntz; ++t)
        for (int ty = 0; ty < g.nty; ++ty)
            for (int tx = 0; tx < g.ntx; ++tx)
                ents += span(tx * g.TX - g.PX, g.RX, Lx) * span(ty * g.TY - g.PY, g.RY, Ly) *
                        span(t * g.TZ, g.RZ, Lz + hp);
    A->sws_bytes = sizeof(double) * ntiles * 3 * g.WN;
    nomem = hipMalloc(&A->d_sws, A->sws_bytes) != hipSuccess ||
            hipMalloc(&A->d_stile_e, sizeof(int) * ntiles) != hipSuccess ||
            (A->ghost_hi && hipMalloc(&A->d_sgsend, sizeof(double) * A->ghost_hi) != hipSuccess) ||
            (A->send_lo && hipMalloc(&A->d_sgrecv, sizeof(double) * A->send_lo) != hipSuccess);
    (void)hipGetLastError();
    KLE_TRY(any_rank(c, nomem, any));
    if (any) {
        sym_drop(A);
        return fail(KLE_ERR_MEM, "out of device memory for the symmetric SpMV workspace");
    }
    hipLaunchKernelGGL(k_sym_bound, dim3((unsigned)ntiles), dim3(256), 0, c->stream, g, A->d_rowbox, A->d_svptr,
                       A->d_sval, A->d_stile_e);
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(c->stream));
    A->sws_entries = ents;
    A->sblocks = blocks;
    A->snvals = tot;
    if (c->nranks > 1) {
        bool bad = false;
        KLE_TRY(sym_probe(A, vmax_all, bad));
        if (bad) {
            sym_drop(A);
            return fail(KLE_ERR_SUP, "matrix is not symmetric across ranks (product probe)");
        }
    }
    return 0;
}

static int sym_waves(const kle_mat *A)
{
    const int P = A->sym_P;
    const SymRegion r = sym_region(A);
    if (A->sym_TZ == 4) return 8;
    if (g_tune.spmv_sym_waves && sym_fill_fits(r, g_tune.spmv_sym_waves)) return g_tune.spmv_sym_waves;
    return 2 * sym_xl_lds(r) <= LDS_PER_CU && sym_fill_fits(r, 8) ? 8 : 16;
}

template <int WV, bool DET, int TY, int TZ>
static void launch_sym_xl(const kle_mat *A, const SymGeo &g, const kle_vec *x, int64_t t0, int64_t t1,
                          const int *istate, hipStream_t st)
{
    if (t1 <= t0) return;
    const size_t lds = sym_xl_lds(sym_region(A));
    dyn_lds(A->ctx, reinterpret_cast<const void *>(&k_nb_spmv_sym_xl<WV, DET, TY, TZ>), lds);
    hipLaunchKernelGGL((k_nb_spmv_sym_xl<WV, DET, TY, TZ>), dim3((unsigned)(t1 - t0)), dim3(64 * WV), lds, st, g,
                       A->d_srow, A->d_svptr, A->d_sval, x->base, A->d_sws, A->d_stile_e, istate,
                       (int)t0, g_tune.spmv_sym_early, g_tune.spmv_sym_stpol, g_tune.spmv_sym_xcd KLE_PROBE_ARG);
}

static void launch_sym_tiles(const kle_mat *A, const SymGeo &g, const kle_vec *x, int64_t t0, int64_t t1,
                             const int *istate, hipStream_t st)
{
    const bool det = g_tune.spmv_sym_det != 0;
    if (g.TZ == 4 && g.TY == 2) {
        if (det) launch_sym_xl<8, true, 2, 4>(A, g, x, t0, t1, istate, st);
        else launch_sym_xl<8, false, 2, 4>(A, g, x, t0, t1, istate, st);
    } else if (g.TZ == 4) {
        if (det) launch_sym_xl<8, true, 4, 4>(A, g, x, t0, t1, istate, st);
        else launch_sym_xl<8, false, 4, 4>(A, g, x, t0, t1, istate, st);
    } else if (sym_waves(A) == 16) {
        if (det) launch_sym_xl<16, true, 8, 2>(A, g, x, t0, t1, istate, st);
        else launch_sym_xl<16, false, 8, 2>(A, g, x, t0, t1, istate, st);
    } else {
        if (det) launch_sym_xl<8, true, 8, 2>(A, g, x, t0, t1, istate, st);
        else launch_sym_xl<8, false, 8, 2>(A, g, x, t0, t1, istate, st);
    }
}

static void launch_sym_gather(const kle_mat *A, const SymGeo &g, kle_vec *y, int64_t j0, int64_t j1, int64_t nrecv,
                              const int *istate, hipStream_t st, const double *xdot = nullptr,
                              double *dpart = nullptr)
{
    if (j1 <= j0) return;
    const dim3 grid((unsigned)((j1 - j0 + 255) / 256));
    if (g.TZ == 4 && g.TY == 2)
        hipLaunchKernelGGL((k_nb_sym_gather<SYM_TX, 2, 4>), grid, dim3(256), 0, st, g, A->d_sws, y->d, A->d_sgsend,
                           A->d_sgrecv, nrecv, j0, j1, istate, xdot, dpart);
    else if (g.TZ == 4)
        hipLaunchKernelGGL((k_nb_sym_gather<SYM_TX, 4, 4>), grid, dim3(256), 0, st, g, A->d_sws, y->d, A->d_sgsend,
                           A->d_sgrecv, nrecv, j0, j1, istate, xdot, dpart);
    else
        hipLaunchKernelGGL((k_nb_sym_gather<SYM_TX, 8, 2>), grid, dim3(256), 0, st, g, A->d_sws, y->d, A->d_sgsend,
                           A->d_sgrecv, nrecv, j0, j1, istate, xdot, dpart);
}

int sym_dot_parts(const kle_mat *A)
{
    if (A->sym_brick) return A->ctx->nranks > 1 ? 0 : (int)((A->nrows + 255) / 256);
    const bool dist = A->ctx->nranks > 1 && (A->sym_graph || A->lo_rank >= 0 || A->hi_rank >= 0);
    return dist ? 0 : (int)((A->nrows + 255) / 256);
}

// y = A x over the symmetric storage.  N > 1 (z slabs), per SpMV:
//   main: tiles whose regions stay below the upper ghost planes, while the
//         comm stream exchanges the forward halo (x ghosts);
//   main: the remaining tiles, then the upper ghost rows' sums -> d_sgsend;
//   comm: the reverse halo (d_sgsend up, the lower neighbour's sums for my
//         lowest rows -> d_sgrecv), while main gathers the rows it does not
//         touch; main: the lowest rows, + d_sgrecv last (fixed order: y stays
//         bitwise reproducible with spmv_sym_det).
// All RCCL calls stay on the comm stream, in the same order on every rank.
int sym_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart)
{
    kle_ctx *c = A->ctx;
    hipStream_t st = c->stream;
    if (A->sym_graph) return gsym_spmv(A, x, y, istate, dpart);
    if (A->sym_brick) return brick_spmv(A, x, y, istate, dpart);
    const SymGeo g = sym_geo(A);
    const int64_t ntiles = (int64_t)g.ntx * g.nty * g.ntz, n = A->nrows, Lxy = (int64_t)g.Lx * g.Ly;
    const bool dist = c->nranks > 1 && (A->lo_rank >= 0 || A->hi_rank >= 0);
    if (!dist) {
        launch_sym_tiles(A, g, x, 0, ntiles, istate, st);
        launch_sym_gather(A, g, y, 0, n, 0, istate, st, dpart ? x->d : nullptr, dpart);
        KLE_HIP(hipGetLastError());
        return 0;
    }
    // tiles [0, nin): regions below the owned top (no upper ghost x).  With
    // overlap they run in two parts: [0, nA) beside the forward halo, then
    // the top tiles (the only ones whose regions hold upper ghost rows) and
    // the ghost rows' sums, then [nA, nin) beside the reverse halo -- so the
    // reverse halo's latency hides behind tile work too, not only behind the
    // gather (spmv_sym_ovl_b: the percentage of the interior tiles kept for
    // the second part).  Tile partials do not depend on the launch order,
    // and the gather sums them in a fixed order: y is bitwise the plain one.
    const int64_t ntz_in = g.Lz >= g.RZ ? (g.Lz - g.RZ) / g.TZ + 1 : 0;
    const int64_t nin = std::min(ntiles, ntz_in * g.nty * g.ntx);
    const int64_t nrecv = A->lo_rank >= 0 ? A->send_lo : 0, jr = nrecv / 3;
    const bool ovl = A->halo_overlap != 0;
    const int64_t nA = ovl && A->hi_rank >= 0 ? nin - nin * g_tune.spmv_sym_ovl_b / 100 : nin;
    if (ovl) {
        KLE_HIP(hipEventRecord(c->ev_x_ready, st));
        KLE_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_x_ready, 0));
        launch_sym_tiles(A, g, x, 0, nA, istate, st);
        KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank, x->send_lo,
                              x->send_hi, c->comm_stream, nullptr));
        KLE_HIP(hipEventRecord(c->ev_halo_done, c->comm_stream));
        KLE_HIP(hipStreamWaitEvent(st, c->ev_halo_done, 0));
        launch_sym_tiles(A, g, x, nin, ntiles, istate, st);
    } else {
        KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank, x->send_lo,
                              x->send_hi, st, nullptr));
        launch_sym_tiles(A, g, x, 0, ntiles, istate, st);
    }
    launch_sym_gather(A, g, y, n, n + (int64_t)g.hp * Lxy, 0, istate, st);  // upper ghost rows -> d_sgsend
    KLE_HIP(hipGetLastError());
    if (ovl) {
        KLE_HIP(hipEventRecord(c->ev_x_ready, st));
        KLE_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_x_ready, 0));
        KLE_TRY(halo_reverse(c, A->d_sgsend, A->ghost_hi, A->hi_rank, A->d_sgrecv, nrecv, A->lo_rank, c->comm_stream));
        KLE_HIP(hipEventRecord(c->ev_halo_done, c->comm_stream));
        launch_sym_tiles(A, g, x, nA, nin, istate, st);
        launch_sym_gather(A, g, y, jr, n, 0, istate, st);
        KLE_HIP(hipStreamWaitEvent(st, c->ev_halo_done, 0));
        launch_sym_gather(A, g, y, 0, jr, nrecv, istate, st);
    } else {
        KLE_TRY(halo_reverse(c, A->d_sgsend, A->ghost_hi, A->hi_rank, A->d_sgrecv, nrecv, A->lo_rank, st));
        launch_sym_gather(A, g, y, 0, n, nrecv, istate, st);
    }
    KLE_HIP(hipGetLastError());
    return 0;
}

std::string sym_kernel_name(const kle_mat *A)
{
    if (A->sym_brick)
        return std::string("k_nb_spmv_sym_brick<") + std::to_string(BRICK_WV) + ",true,false>+k_nb_gsym_gather<" +
               std::to_string(gather_wps(A)) + ">";
    if (A->sym_gbrick) return "k_nb_spmv_gsym_brick<16,1>+k_nb_gsym_gather<" + std::to_string(gather_wps(A)) + ">";
    if (A->sym_graph)
        return std::string("k_nb_spmv_gsym<") + (g_tune.spmv_sym_det ? "true," : "false,") +
               std::to_string(A->sym_reg[3]) + "," + std::to_string(A->sym_reg[4]) + ">+k_nb_gsym_gather<" +
               std::to_string(gather_wps(A)) + ">";
    return std::string("k_nb_spmv_sym_xl<") + std::to_string(sym_waves(A)) + "," +
           (g_tune.spmv_sym_det ? "true" : "false") + "," + std::to_string(A->sym_TY) + "," +
           std::to_string(A->sym_TZ) + ">+k_nb_sym_gather<8," + std::to_string(A->sym_TY) + "," +
           std::to_string(A->sym_TZ) + ">";
}

// symmetric storage: the stored (upper) blocks, per row its value offset and
// box, x and y once, the tile partials written and read
// A split box-brick product (brick_spmv split: the CG update gathers it):
// the bricks alone move the values, the row descriptors, x and y's direct
// sums once, and write their region sums once -- the sums' read is the
// update's
double brick_split_bytes(const kle_mat *A)
{
    return (double)A->sblocks * 72.0 + A->nrows * (8.0 + 48.0) + (double)A->sws_entries * 24.0;
}

double sym_spmv_bytes(const kle_mat *A)
{
    // graph: values + 2-B dictionary positions per stored block; per row its
    // value offset, slid offset, count, x and y; per dictionary entry its node
    // id and the partial written and read (the gather runs, 12 B per ~8
    // entries, are not counted)
    // bricks: values, 8 B of row descriptor per row, x and y once, each
    // brick's region sums written once and read once
    if (A->sym_brick) return (double)A->sblocks * 72.0 + A->nrows * (8.0 + 48.0) + (double)A->sws_entries * 48.0;
    // graph bricks: values + positions, 16 B of row descriptor per row, x
    // and y once, per dictionary entry its node id and its sums written and
    // read once
    if (A->sym_gbrick)
        return (double)A->sblocks * 74.0 + A->nrows * (16.0 + 48.0) + (double)A->sws_entries * (4.0 + 48.0);
    if (A->sym_graph)
        return (double)A->sblocks * 74.0 + A->nrows * (8.0 + 8.0 + 4.0 + 48.0) + (double)A->sws_entries * (4.0 + 48.0);
    return (double)A->sblocks * 72.0 + A->nrows * 16.0 + (double)A->nrows * 48.0 + (double)A->sws_entries * 48.0;
}

}  // namespace kle

#ifdef KLE_PROBE_BUILD
// probe build only: the occupancy API's resident workgroups per CU for the
// default symmetric tile kernels at a given dynamic LDS (which: 0 box
// k_nb_spmv_sym_xl<8,true,4,4>, 1 graph k_nb_spmv_gsym<true,64,16>)
extern "C" int kle_probe_occupancy(int which, int lds_bytes, int *blocks)
{
    using namespace kle;
    KLE_ARG(blocks && lds_bytes >= 0, "bad arg");
    const void *f = which == 0 ? reinterpret_cast<const void *>(&k_nb_spmv_sym_xl<8, true, 4, 4>)
                               : reinterpret_cast<const void *>(&k_nb_spmv_gsym<true, 64, 16>);
    KLE_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
    KLE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, f, which == 0 ? 512 : 1024, (size_t)lds_bytes));
    return 0;
}
#endif

#ifdef KLE_PROBE_BUILD
// probe build only: move the box symmetric storage's values (what 1, copied)
// or tile-partial workspace (what 2) to a fresh allocation, `shift` bytes into
// it -- does the SpMV's speed depend on where these arrays land?  The old
// arrays are not freed (probe runs only).
extern "C" int kle_probe_realloc(kle_mat *A, int what, long long shift)
{
    using namespace kle;
    // (what 3: the full storage's values, d_val -- does the full-storage SpMV care?)
    KLE_ARG(A && (what == 3 || (A->d_sval && !A->sym_graph)) && what >= 1 && what <= 3 && shift >= 0 &&
                shift % 8 == 0, "bad arg");
    size_t bytes = sizeof(double) * (size_t)std::max<int64_t>(A->nvals, 1);
    if (what != 3) {
        const SymGeo g = sym_geo(A);
        bytes = what == 1 ? sizeof(double) * (size_t)std::max<int64_t>(A->snvals, 1)
                          : sizeof(double) * (size_t)g.ntx * g.nty * g.ntz * 3 * g.WN;
    }
    char *raw = nullptr;
    KLE_HIP(hipMalloc(&raw, bytes + (size_t)shift));
    double *np = reinterpret_cast<double *>(raw + shift);
    double **pp = what == 1 ? &A->d_sval : what == 2 ? &A->d_sws : &A->d_val;
    KLE_HIP(hipMemcpy(np, *pp, bytes, hipMemcpyDeviceToDevice));
    *pp = np;
    fprintf(stderr, "[kle probe] moved %s to %p (raw %p, %zu bytes)\n",
            what == 1 ? "values" : what == 2 ? "workspace" : "full-storage values", (void *)np, (void *)raw, bytes);
    return 0;
}
#endif
