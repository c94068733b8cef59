// kle_sym.hip -- symmetric (SBAIJ-style, upper-triangle) node-block storage of
// the KLE K and its SpMV kernels for gfx950 (kle_mat_set_symmetric =
// MatSetOption(MAT_SPD); K is SPD: MatFS.buildFS, mat_fs.py:150-192).
#include <algorithm>
#include <climits>
#include <cmath>
#include <string>
#include <vector>

#include "kle_internal.hpp"

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
constexpr int SYM_TX = 8, SYM_TY = 8, SYM_TZ = 2;
constexpr int SYM_FILL = 12;  // x-fill loads per thread of k_nb_spmv_sym_xl (one pass over the region)
struct SymGeo {
    int Lx, Ly, Lz, P, TX, TZ, RX, RY, RZ, ntx, nty, ntz;
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
__global__ __launch_bounds__(256) void k_sym_build(int64_t nrows, int Lx, int Ly, const int *__restrict__ rowptr,
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
        int cx, cy, cz, cnx, cny, cnz;
        sym_box(rowbox, j, Lx, Lxy, cx, cy, cz, cnx, cny, cnz);
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

// Wave sum through DPP row moves (VALU only; __shfl_xor is a ds_bpermute per
// 32-bit half, i.e. 12 LDS instructions per double): quad swaps, half-row
// and row mirrors, then row_bcast15 / row_bcast31 carry the row sums into
// lane 63, which every lane reads back.
template <int ctrl, int row_mask>
__device__ __forceinline__ double dpp_step(double v)
{
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const int l2 = __builtin_amdgcn_update_dpp(0, lo, ctrl, row_mask, 0xF, false);
    const int h2 = __builtin_amdgcn_update_dpp(0, hi, ctrl, row_mask, 0xF, false);
    return v + __hiloint2double(h2, l2);
}

__device__ __forceinline__ double wsum_dpp(double v)
{
    v = dpp_step<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = dpp_step<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = dpp_step<0x141, 0xF>(v);  // row_half_mirror
    v = dpp_step<0x140, 0xF>(v);  // row_mirror
    v = dpp_step<0x142, 0xA>(v);  // row_bcast15 into rows 1, 3
    v = dpp_step<0x143, 0xC>(v);  // row_bcast31 into rows 2, 3
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
    return __hiloint2double(hi, lo);
}

// Same tile pass with the wave's (row, 64-block pass) items flattened into one
// software-pipelined loop: the values and x entries of the next item are in
// flight while the current one is multiplied and accumulated (a wave's rows
// average 1.4 passes of 64 blocks, so one item at a time leaves it waiting
// on HBM latency at every row).
struct SymRow {
    int64_t i;
    const double *v;
    double x0, x1, x2;
    int bx, by, bz, bnx, bnxy, k0, mu, rx0, ry0, rz0, own;
    float ibnx, ibnxy;  // 1/bnx, 1/bnxy: quotients of block positions by float multiply + one fix-up
};

// q = n / d for 0 <= n < 2^20, d >= 1 (block position in its row box)
__device__ __forceinline__ int sym_div(int n, int d, float inv)
{
    int q = (int)((float)n * inv);
    q += (q + 1) * d <= n;
    q -= q * d > n;
    return q;
}

__device__ __forceinline__ double uni_d(double v)
{
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}


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
__device__ __forceinline__ unsigned long long fx_of(double c, double S)
{
    const double v = __builtin_rint(c * S);           // |v| <= 2^61: an integer
    const double hi = __builtin_floor(v * 0x1p-32);  // exact
    const double lo = __builtin_fma(hi, -0x1p32, v);  // exact, in [0, 2^32)
    return ((unsigned long long)(unsigned)(int)hi << 32) + (unsigned long long)(unsigned)lo;
}

__device__ __forceinline__ double fx_to_d(unsigned long long u)
{
    return (double)(int)((long long)u >> 32) * 0x1p32 + (double)(unsigned)(u & 0xffffffffull);
}

// Value loads of one item of k_nb_spmv_sym_xl, issued in inline asm so the
// compiler's wait bookkeeping cannot drain them: it saw the next item's loads
// as hazards on registers of the current one and put s_waitcnt vmcnt(0) in
// front of them at every second item.  The wait for an item (vmcnt(9): the
// next item's 9 loads stay in flight) names its 9 registers as read-write
// operands, so nothing reads them before the data has landed.
__device__ __forceinline__ void sym_ld9(double *v, const double *base, const unsigned *o)
{
    asm volatile(
        "s_nop 4\n\t"
        "global_load_dwordx2 %0, %9, %18 nt\n\t"
        "global_load_dwordx2 %1, %10, %18 nt\n\t"
        "global_load_dwordx2 %2, %11, %18 nt\n\t"
        "global_load_dwordx2 %3, %12, %18 nt\n\t"
        "global_load_dwordx2 %4, %13, %18 nt\n\t"
        "global_load_dwordx2 %5, %14, %18 nt\n\t"
        "global_load_dwordx2 %6, %15, %18 nt\n\t"
        "global_load_dwordx2 %7, %16, %18 nt\n\t"
        "global_load_dwordx2 %8, %17, %18 nt"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
          "=&v"(v[8])
        : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "v"(o[5]), "v"(o[6]), "v"(o[7]), "v"(o[8]),
          "s"(base)
        : "memory");
}

template <int N>
__device__ __forceinline__ void sym_wait9(double *v)
{
    asm volatile("s_waitcnt vmcnt(%9)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8])
                 : "i"(N));
}

// Single loads the compiler does not count (inline asm): uniform base + 32-bit
// byte offset.  The caller waits with sym_waitn and names the registers.
__device__ __forceinline__ void asm_ld_f64(double &v, const void *base, unsigned off)
{
    asm volatile("global_load_dwordx2 %0, %1, %2" : "=v"(v) : "v"(off), "s"(base) : "memory");
}
__device__ __forceinline__ void asm_ld_i32(int &v, const void *base, unsigned off)
{
    asm volatile("global_load_dword %0, %1, %2" : "=v"(v) : "v"(off), "s"(base) : "memory");
}
template <int N>
__device__ __forceinline__ void sym_waitn()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
template <class T>
__device__ __forceinline__ void asm_touch(T &v)  // after a wait: v's register holds the data now
{
    asm volatile("" : "+v"(v));
}

template <int WV, bool DET, int AHEAD>
__global__ __launch_bounds__(64 * WV, 4) void k_nb_spmv_sym_xl(SymGeo g, const int *__restrict__ rowbox,
                                                             const int64_t *__restrict__ svptr,
                                                             const double *__restrict__ sval,
                                                             const double *__restrict__ x, double *__restrict__ ws,
                                                             const int *__restrict__ tile_e,
                                                             const int *__restrict__ istate, int probe)
{
    // LDS: x [3][RN] | y [3][RN + 64] (DET: int64; 64 dummy slots per
    // component take the adds of masked lanes) | direct row sums [3][TR]
    extern __shared__ double lds[];
    if (istate && istate[I_REASON] != 0) return;
    constexpr int TZ = SYM_TZ, TR = SYM_TX * SYM_TY * TZ, NT = 64 * WV;
    constexpr int NQ = SYM_TX * SYM_TY / WV;  // row slots per wave and plane
    constexpr int NS = NQ * TZ;               // row slots per wave
    const int RN = g.RX * g.RY * g.RZ, RS = RN + 64;
    double *xl = lds, *yl = lds + 3 * RN, *yd = lds + 3 * RN + 3 * RS;
    const int64_t t = blockIdx.x;
    const int tix = (int)(t % g.ntx);
    const int64_t q = t / g.ntx;
    const int tiy = (int)(q % g.nty), tz = (int)(q / g.nty) * TZ;
    const int x0 = tix * SYM_TX, y0 = tiy * SYM_TY, ox = x0 - g.P, oy = y0 - g.P;
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
    // 1. the wave's row descriptors (box, value offset): lane s holds slot s
    int pb, pd, psl, psh;
    {
        const bool ok = lane < NS && slot_ok(lane);
        const int64_t i =
            ok ? x0 + slot_x(lane) + (int64_t)g.Lx * (y0 + slot_y(lane)) + Lxy * (tz + lane / NQ) : 0;
        pb = rowbox[2 * i];
        pd = rowbox[2 * i + 1];
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
        const bool ok = fx_ok && l < NL && oy + ry >= 0 && oy + ry < g.Ly && tz + rz < g.Lz;
        const int64_t node = ok ? (int64_t)(ox + frx) + (int64_t)g.Lx * (oy + ry) + Lxy * (tz + rz) : 0;
        const double v = x[3 * node + fcc];
        fv[f] = ok ? v : 0.0;
    }
    for (int k = threadIdx.x; k < 3 * RS; k += NT) yl[k] = 0.0;
    for (int k = threadIdx.x; k < 3 * TR; k += NT) yd[k] = 0.0;
    auto slot_row = [&](int s, SymRow &R) {
        const int xg = x0 + slot_x(s), yy = y0 + slot_y(s), zz = tz + s / NQ;
        R.i = xg + (int64_t)g.Lx * yy + Lxy * zz;
        const int64_t base = __builtin_amdgcn_readlane(pb, s);
        const int d = __builtin_amdgcn_readlane(pd, s);
        R.bz = (int)(base / Lxy);
        const int64_t rem = base - (int64_t)R.bz * Lxy;
        R.by = (int)(rem / g.Lx);
        R.bx = (int)(rem - (int64_t)R.by * g.Lx);
        R.bnx = d & 255;
        const int bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
        R.bnxy = R.bnx * bny;
        R.ibnx = 1.0f / (float)R.bnx;
        R.ibnxy = 1.0f / (float)R.bnxy;
        R.k0 = (xg - R.bx) + R.bnx * ((yy - R.by) + bny * (zz - R.bz));
        R.mu = R.bnxy * bnz - R.k0;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(psl, s);
        const int64_t hi = __builtin_amdgcn_readlane(psh, s);
        R.v = sval + ((hi << 32) | lo);
        R.rx0 = R.bx - ox;
        R.ry0 = R.by - oy;
        R.rz0 = R.bz - tz;
        R.own = (xg - x0) + SYM_TX * ((yy - y0) + SYM_TY * (zz - tz));  // row slot in the tile
        const int ir = (xg - ox) + g.RX * ((yy - oy) + g.RY * (zz - tz));  // its region index
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
        const int64_t o0 = ch ? (int64_t)((kk >> 4) * 144 + (kk & 15)) : (int64_t)q16 * 9 + (kk - q16);
        const int st = ch ? 16 : R.mu - q16;
        unsigned o[9];
#pragma unroll
        for (int s = 0; s < 9; ++s) o[s] = (unsigned)(o0 + s * st) * 8u;
        sym_ld9(vv, R.v, o);
        const int k = R.k0 + kk;
        const int kz = sym_div(k, R.bnxy, R.ibnxy), rem = k - kz * R.bnxy;
        const int ky = sym_div(rem, R.bnx, R.ibnx), kx = rem - ky * R.bnx;
        rr = (R.rx0 + kx) + g.RX * ((R.ry0 + ky) + g.RY * (R.rz0 + kz));
    };
    auto load_x = [&](int rr, double *xv) {
        xv[0] = xl[rr];
        xv[1] = xl[RN + rr];
        xv[2] = xl[2 * RN + rr];
    };
    // 3. items = (row, pass of 64 blocks).  The issue cursor (row I, slot xi,
    // pass ki) runs AHEAD items in front of the compute cursor (row C, slot
    // xc, pass kc); past the wave's last item it stays there, re-reading it
    // (cache hits), so every step issues exactly 9 loads and the wait for the
    // item being summed is a fixed vmcnt(9 AHEAD).  A wave without rows in
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
#pragma unroll
    for (int f = 0; f < SYM_FILL; ++f) {
        const int l = fl0 + f * fstep;  // (unused slots store into a dummy y slot: no branch)
        xl[fl0 < fstep && l < NL ? fcc * RN + frx + g.RX * l : 4 * RN + lane] = fv[f];
    }
    double v0[9], v1[9], v2[9];
    int r0, r1 = 0, r2 = 0;
    load_v(I, ki, v0, r0);  // in flight across the barrier
    if (AHEAD == 2) {
        issue_next();
        load_v(I, ki, v1, r1);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // LDS stores done (lgkmcnt 0); the value loads stay in flight
    __builtin_amdgcn_s_barrier();
    double S = 1.0, invS = 1.0;
    if (DET) {
        // max |x_i| over the tile's rows (every wave computes it; max is exact)
        double m = 0.0;
        int bad = 0;
        for (int r = lane; r < TR; r += 64) {
            const int k = (g.P + (r & 7)) + g.RX * ((g.P + ((r >> 3) & 7)) + g.RY * (r >> 6));
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
    if (any) {
        int xc = next_slot(0), kc = 0;
        slot_row(xc, C);  // (x_i from LDS, now that the fill has landed)
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
        // one item: issue the item AHEAD in front into vn, wait for vv (the
        // AHEAD items issued after it stay in flight), sum it
        auto step = [&](double *vv, const int rr, double *vn, int &rn) {
            issue_next();
            load_v(I, ki, vn, rn);
            double xv[3];
            if (probe & 4)
                xv[0] = xv[1] = xv[2] = C.x0;
            else
                load_x(rr, xv);  // LDS latency overlaps the wait
            sym_wait9<9 * AHEAD>(vv);
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
            acc0 = wsum_dpp(acc0);
            acc1 = wsum_dpp(acc1);
            acc2 = wsum_dpp(acc2);
            if (lane < 3) yd[lane * TR + C.own] = lane == 0 ? acc0 : lane == 1 ? acc1 : acc2;
            acc0 = acc1 = acc2 = 0.0;
            const int nx = next_slot(xc + 1);
            if (nx >= NS) return false;
            xc = nx;
            kc = 0;
            slot_row(xc, C);
            return true;
        };
        if (AHEAD == 1) {
            while (step(v0, r0, v1, r1) && step(v1, r1, v0, r0)) {
            }
        } else {
            while (step(v0, r0, v2, r2) && step(v1, r1, v0, r0) && step(v2, r2, v1, r1)) {
            }
        }
    }
    // the last (re-read) loads land before their registers are reused
    sym_wait9<0>(v0);
    sym_wait9<0>(v1);
    if (AHEAD == 2) sym_wait9<0>(v2);
    __syncthreads();
    // 4. the tile's partial sums: region nodes inside the lattice
    double *dst = ws + ((probe & 64) ? (t & 7) : t) * 3 * (int64_t)RN;  // (probe 64: every tile into 8 slabs)
    const unsigned long long *yi = reinterpret_cast<const unsigned long long *>(yl);
    for (int k = (probe & 8) ? RN : threadIdx.x; k < RN; k += NT) {
        const int rz = k / (g.RX * g.RY), rem = k - rz * g.RX * g.RY, ry = rem / g.RX, rx = rem - ry * g.RX;
        const int gx = ox + rx, gy = oy + ry, gz = tz + rz;
        if (gx < 0 || gx >= g.Lx || gy < 0 || gy >= g.Ly || gz >= g.Lz) continue;
        const bool own = rx >= g.P && rx < g.P + SYM_TX && ry >= g.P && ry < g.P + SYM_TY && rz < TZ;
        const int sl = (rx - g.P) + SYM_TX * ((ry - g.P) + SYM_TY * rz);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            double v = DET ? fx_to_d(yi[b * RS + k]) * invS : yl[b * RS + k];
            if (own) v += yd[b * TR + sl];
            if (probe & 32)
                __builtin_nontemporal_store(v, dst + b * RN + k);
            else
                dst[b * RN + k] = v;
        }
    }
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
    constexpr int TR = SYM_TX * SYM_TY * SYM_TZ;
    __shared__ int sb[TR], sd[TR];
    __shared__ int64_t so[TR];
    __shared__ double wred[256];
    const int64_t t = blockIdx.x;
    const int tix = (int)(t % g.ntx);
    const int64_t q = t / g.ntx;
    const int tiy = (int)(q % g.nty), tz = (int)(q / g.nty) * SYM_TZ;
    const int x0 = tix * SYM_TX, y0 = tiy * SYM_TY, ox = x0 - g.P, oy = y0 - g.P;
    const int64_t Lxy = (int64_t)g.Lx * g.Ly;
    for (int r = threadIdx.x; r < TR; r += 256) {
        const int xi = x0 + (r & 7), yi = y0 + ((r >> 3) & 7), zi = tz + (r >> 6);
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
        if (gx < 0 || gx >= g.Lx || gy < 0 || gy >= g.Ly || gz >= g.Lz) continue;
        double s = 0.0;
        for (int r = 0; r < TR; ++r) {
            const int d = sd[r];
            if (!d) continue;
            const int64_t base = sb[r];
            const int bz = (int)(base / Lxy), by = (int)((base - bz * Lxy) / g.Lx);
            const int bx = (int)(base - bz * Lxy - (int64_t)by * g.Lx);
            const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
            if (gx < bx || gx >= bx + bnx || gy < by || gy >= by + bny || gz < bz || gz >= bz + bnz) continue;
            const int xi = x0 + (r & 7), yi = y0 + ((r >> 3) & 7), zi = tz + (r >> 6);
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
// ascending (z, y, x) tile order.
template <int TXW, int TZ>
__global__ __launch_bounds__(256) void k_nb_sym_gather(SymGeo g, const double *__restrict__ ws, double *__restrict__ y,
                                                       const int *__restrict__ istate)
{
    if (istate && istate[I_REASON] != 0) return;
    const int64_t Lxy = (int64_t)g.Lx * g.Ly, n = Lxy * g.Lz;
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int jz = (int)(j / Lxy), jy = (int)((j - jz * Lxy) / g.Lx), jx = (int)(j - jz * Lxy - (int64_t)jy * g.Lx);
    const int RN = g.RX * g.RY * g.RZ;
    // tiles whose [t*T - P, t*T - P + R) contains the coordinate
    const int x_lo = max(0, (jx + g.P - g.RX + TXW) / TXW), x_hi = min(g.ntx - 1, (jx + g.P) / TXW);
    const int y_lo = max(0, (jy + g.P - g.RY + SYM_TY) / SYM_TY), y_hi = min(g.nty - 1, (jy + g.P) / SYM_TY);
    const int z_lo = max(0, (jz - g.RZ + TZ) / TZ), z_hi = min(g.ntz - 1, jz / TZ);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int tzi = z_lo; tzi <= z_hi; ++tzi)
        for (int ty = y_lo; ty <= y_hi; ++ty)
            for (int tx = x_lo; tx <= x_hi; ++tx) {
                const int64_t t = ((int64_t)tzi * g.nty + ty) * g.ntx + tx;
                const int r = (jx - (tx * TXW - g.P)) + g.RX * ((jy - (ty * SYM_TY - g.P)) + g.RY * (jz - tzi * TZ));
                const double *p = ws + t * 3 * (int64_t)RN + r;
                s0 += p[0];
                s1 += p[RN];
                s2 += p[2 * RN];
            }
    y[3 * j] = s0;
    y[3 * j + 1] = s1;
    y[3 * j + 2] = s2;
}

// ---------------------------------------------------------------------------
// Column-walk symmetric SpMV (round 3; default while P <= 4).
//
// The tile kernel above writes every tile's whole region partial (16 x 16 x 6
// nodes at P = 4, 12 partials per node) and its workgroup then ends -- and a
// wave's s_endpgm waits for its stores to be acknowledged.  Under the full
// read stream those acknowledgements take tens of microseconds (timing probe:
// the partial stores cost 45-100 us of a 0.50-0.54 ms SpMV; the same stores
// into an L2-resident slab cost 11 us).  Here a workgroup walks a column
// (tix, tiy) of tiles upward in z: consecutive tiles' regions share P of
// their TZ + P planes, so x and the partial sums live in LDS rings indexed by
// plane mod RZ, and a tile transition only moves the TZ planes that leave
// (final for this column: rows above add nothing to them) and the TZ planes
// that enter.  One helper wave per workgroup does all of that traffic -- it
// loads the entering x planes a tile ahead and stores the leaving partials --
// so the 8 compute waves never wait for a store, and a node collects at most
// 2 x 2 column partials (+ one or two at run boundaries) instead of 12:
// 33 MB of partials each way per SpMV at config 2 instead of 90 MB.
//
// Work: the column-major tile sequence is cut into one chunk per resident
// workgroup (2 per CU), balanced by stored blocks; a chunk is one or more
// runs (consecutive tiles of one column).  A run starts cold (whole x
// window, zeroed y ring) and, where it stops below the column's top, writes
// the P planes above its last tile to overlap slabs the gather adds.  DET:
// one fixed-point scale per run, 2^(61-E) with 2^E > W_run max|x| over the
// run's region (W_run: k_sym_bound_cw), transposed and direct sums alike.
struct SymRun {
    int c, kz0, kz1, ovl;  // column, its tiles [kz0, kz1), first overlap slab (-1: none)
};
constexpr int CW_WV = 7;                  // compute waves per workgroup (+ the helper: 8 waves, 2 per SIMD x 2 per CU)
constexpr int CW_NT = 64 * (CW_WV + 1);

__device__ __forceinline__ int cw_ring(int v, int s0, int RZ)
{
    const int r = v + s0;
    return r >= RZ ? r - RZ : r;
}

template <int P, bool DET>
__global__ __launch_bounds__(CW_NT, 4) void k_nb_spmv_sym_cw(SymGeo g, const int *__restrict__ rowbox,
                                                            const int64_t *__restrict__ svptr,
                                                            const double *__restrict__ sval,
                                                            const double *__restrict__ x, double *__restrict__ wsA,
                                                            double *__restrict__ wsB, const SymRun *__restrict__ runs,
                                                            const int *__restrict__ chunk_run,
                                                            const int *__restrict__ run_e,
                                                            const int *__restrict__ istate, int probe)
{
    // LDS: x ring [3][RZ][RY][RX] | y ring [3][RZ * RY * RX + 64 dummy] (DET: int64)
    extern __shared__ double lds[];
    __shared__ double red[CW_WV + 1];
    if (istate && istate[I_REASON] != 0) return;
    constexpr int TZ = SYM_TZ, TR = SYM_TX * SYM_TY * TZ, NS = (TR + CW_WV - 1) / CW_WV;
    constexpr int RX = SYM_TX + 2 * P, RY = SYM_TY + 2 * P, RZ = TZ + P, RXY = RX * RY, RN = RXY * RZ, RS = RN + 64;
    constexpr int L3 = 3 * RX;
    double *xl = lds, *yl = lds + 3 * RN;
    unsigned long long *yi = reinterpret_cast<unsigned long long *>(yl);
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool helper = w == CW_WV;
    const int64_t Lxy = (int64_t)g.Lx * g.Ly;
    const int r0 = chunk_run[blockIdx.x], r1 = chunk_run[blockIdx.x + 1];
    // workgroup barrier over LDS only: __syncthreads() would also wait for every
    // global access in flight (vmcnt(0)) -- the storer's stores and the compute
    // waves' prefetched loads are exactly what must stay in flight across it
    auto lds_barrier = []() {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
    };
    for (int r = r0; r < r1; ++r) {
        const SymRun R = runs[r];
        const int tix = R.c % g.ntx, tiy = R.c / g.ntx;
        const int x0 = tix * SYM_TX, y0 = tiy * SYM_TY, ox = x0 - P, oy = y0 - P;
        const int nx = min(SYM_TX, g.Lx - x0);
        const int zr0 = R.kz0 * TZ, zr1 = min(R.kz1 * TZ, g.Lz), zhi = min(zr1 + P, g.Lz);
        // global x of region node (rx, ry) in plane z (0 outside the lattice)
        auto xin = [&](int rx, int ry, int z) {
            return ox + rx >= 0 && ox + rx < g.Lx && oy + ry >= 0 && oy + ry < g.Ly && z < g.Lz;
        };
        auto xaddr = [&](int rx, int ry, int z, int cc) {
            return 3 * ((int64_t)(ox + rx) + (int64_t)g.Lx * (oy + ry) + Lxy * z) + cc;
        };
        // (an opaque copy of the thread id: values derived from it for the
        // cold start are recomputed per run instead of being hoisted out of the
        // run loop and spilled)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        auto olane = [&]() {  // an opaque lane id: derived values are recomputed where used
            int l = lane;
            asm volatile("" : "+v"(l));
            return l;
        };
        // ---- cold start: zero the y ring, x window [zr0, zr0 + RZ), DET scale
        for (int k = tid; k < 3 * RS; k += CW_NT) yl[k] = 0.0;
        constexpr int CT = CW_WV * 64;  // the compute waves' threads (the storer loads nothing)
        if (tid < (CT / L3) * L3) {
            const int f = tid % L3, rx = f / 3, cc = f - 3 * rx;
            for (int l = tid / L3; l < RZ * RY; l += CT / L3) {
                const int pz = l / RY, ry = l - pz * RY, z = zr0 + pz;
                const bool ok = xin(rx, ry, z);
                const double v = x[ok ? xaddr(rx, ry, z, cc) : 0];
                xl[cc * RN + (z % RZ) * RXY + ry * RX + rx] = ok ? v : 0.0;
            }
        }
        double S = 1.0, invS = 1.0;
        if (DET) {
            double m = 0.0;
            int bad = 0;
            if (tid < (CT / L3) * L3) {
                const int f = tid % L3, rx = f / 3, cc = f - 3 * rx;
                for (int l = tid / L3; l < (zhi - zr0) * RY; l += CT / L3) {
                    const int pz = l / RY, ry = l - pz * RY, z = zr0 + pz;
                    const bool ok = xin(rx, ry, z);
                    const double a = fabs(x[ok ? xaddr(rx, ry, z, cc) : 0]);
                    bad |= ok && !(a <= 1.7976931348623157e308);
                    m = ok ? fmax(m, a) : m;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
            bad = __ballot(bad) != 0;
            if (lane == 0) red[w] = bad ? -1.0 : m;
            __syncthreads();
            m = 0.0;
            bad = 0;
            for (int k = 0; k <= CW_WV; ++k) {
                bad |= red[k] < 0.0;
                m = fmax(m, red[k]);
            }
            if (bad) {
                S = 0.0;  // non-finite x: the partials come out NaN, as a floating-point sum would
                invS = __builtin_nan("");
            } else if (m > 0.0) {
                int em;
                (void)frexp(m, &em);
                const int E = min(max(run_e[r] + em, -960), 1020);
                S = ldexp(1.0, 61 - E);
                invS = ldexp(1.0, E - 61);
            }
        }
        // ---- helper wave: entering x planes a tile ahead (registers), leaving partials out
        // The TZ planes a tile adds to its predecessor's window are loaded by
        // the compute waves at the start of the previous tile (in flight during
        // it) and written into the ring after T1: compute wave w takes the
        // planes' lattice lines w, w + 7, ... (lane l < 3 RX: position l of the line).
        constexpr int NLN = TZ * RY, XE = (NLN + CW_WV - 1) / CW_WV;
        double xe[XE];
        // (the out-of-lattice mask is applied when storing: a select right
        // after a load would wait for it)
        auto xe_ok = [&](int ln0, int rx, int q, int kz, int &ry, int &z) {
            const int ln = w + CW_WV * q, pz = ln / RY;
            ry = ln - pz * RY;
            z = kz * TZ + RZ - TZ + pz;
            return ln0 < L3 && ox + rx >= 0 && ox + rx < g.Lx && ln < NLN && oy + ry >= 0 && oy + ry < g.Ly &&
                   z < g.Lz;
        };
        // (asm loads: a load the compiler counts makes it wait for everything
        // in flight before the next barrier; waited with sym_waitn in xe_store)
        auto xe_load = [&](int kz) {
            const int ln0 = olane(), rx = ln0 / 3, cc = ln0 - 3 * rx;
#pragma unroll
            for (int q = 0; q < XE; ++q) {
                int ry, z;
                const bool ok = xe_ok(ln0, rx, q, kz, ry, z);
                asm_ld_f64(xe[q], x, (uint32_t)(ok ? xaddr(rx, ry, z, cc) : 0) * 8u);
            }
        };
        auto xe_store = [&](int kz) {  // after sym_waitn for the loads
#pragma unroll
            for (int q = 0; q < XE; ++q) asm_touch(xe[q]);
            const int ln0 = olane(), rx = ln0 / 3, cc = ln0 - 3 * rx;
            if (ln0 < L3) {
#pragma unroll
                for (int q = 0; q < XE; ++q) {
                    int ry, z;
                    const bool ok = xe_ok(ln0, rx, q, kz, ry, z);
                    if (w + CW_WV * q < NLN) xl[cc * RN + (z % RZ) * RXY + ry * RX + rx] = ok ? xe[q] : 0.0;
                }
            }
        };
        // the partials of plane z to global memory (every node of the region
        // plane, unconditional stores: exact wait counts), its ring slot zeroed
        auto y_out = [&](int z, double *dst) {
            const int sl = z % RZ;
#pragma unroll 1
            for (int k = lane; k < RXY; k += 64) {
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    const int e = b * RS + sl * RXY + k;
                    const double v = DET ? fx_to_d(yi[e]) * invS : yl[e];
                    yl[e] = 0.0;
                    if (!(probe & 256)) dst[b * RXY + k] = v;  // (timing probe 256: no partial stores)
                }
            }
        };
        // ---- compute waves: slot s of wave w is the tile's row w + 7 s (row r:
        // plane r / 64, line (r / 8) % 8, x offset r % 8).  Per tile, lane s
        // decodes slot s's row once (box, value offset, region offsets, ring
        // index) into a few VGPRs; a row starts with readlanes, and the valid
        // slots are a ballot mask (next slot = s_ff1).  zk: the tile's first
        // plane, s0: its ring slot.
        int zk = zr0, s0 = zr0 % RZ;
        int nb = 0, nd = 0, nsl = 0, nsh = 0;  // raw descriptors of a tile (rowbox base, dims, value offset)
        auto desc_load = [&](int kz) {  // asm loads (see xe_load), waited before desc_decode
            const int ln0 = olane(), r = w + CW_WV * ln0, z1 = kz * TZ;
            const bool ok = ln0 < NS && r < TR && y0 + ((r >> 3) & 7) < g.Ly && x0 + (r & 7) < g.Lx &&
                            z1 + (r >> 6) < g.Lz;
            const uint32_t i = ok ? (x0 + (r & 7)) + g.Lx * (y0 + ((r >> 3) & 7)) + (uint32_t)Lxy * (z1 + (r >> 6)) : 0;
            asm_ld_i32(nb, rowbox, i * 8u);
            asm_ld_i32(nd, rowbox, i * 8u + 4u);
            asm_ld_i32(nsl, svptr, i * 8u);
            asm_ld_i32(nsh, svptr, i * 8u + 4u);
        };
        auto desc_wait = [&]() {
            asm_touch(nb);
            asm_touch(nd);
            asm_touch(nsl);
            asm_touch(nsh);
        };
        uint64_t smask = 0;                 // valid slots of the tile
        int qlo = 0, qhi = 0, qa = 0, qb = 0, qc = 0;  // decoded slot records (lane s: slot s)
        float qix = 1.0f, qixy = 1.0f;
        auto desc_decode = [&]() {  // after nb.. have landed; zk, s0 of the tile
            const int ln0 = olane(), r = w + CW_WV * ln0;
            const int xg = x0 + (r & 7), yy = y0 + ((r >> 3) & 7), zz = zk + (r >> 6);
            const bool ok = ln0 < NS && r < TR && yy < g.Ly && xg < g.Lx && zz < g.Lz;
            smask = __ballot(ok);
            const int64_t base = nb;
            const int bz = (int)(base / Lxy), by = (int)((base - bz * Lxy) / g.Lx);
            const int bx = (int)(base - bz * Lxy - (int64_t)by * g.Lx);
            const int bnx = nd & 255, bny = (nd >> 8) & 255, bnz = (nd >> 16) & 255;
            const int k0 = (xg - bx) + bnx * ((yy - by) + bny * (zz - bz));
            const int mu = bnx * bny * bnz - k0;
            qlo = nsl;
            qhi = nsh;
            qa = ok ? (k0 | (mu << 16)) : (0 | (1 << 16));
            qb = bnx | ((bnx * bny) << 8) | ((bx - ox + 32) << 20);  // rx0 in [-P, RX)
            qc = (by - oy + 32) | ((bz - zk + 32) << 8) |
                 (((xg - ox) + RX * ((yy - oy) + RY * cw_ring(zz - zk, s0, RZ))) << 16);  // ry0, rz0, own
            qix = 1.0f / (float)bnx;
            qixy = 1.0f / (float)(bnx * bny);
        };
        auto next_slot = [&](int s) {  // first valid slot >= s, or NS
            const uint64_t m = s < 64 ? smask >> s : 0;
            return m ? s + (int)__builtin_ctzll(m) : NS;
        };
        auto slot_row = [&](int s, SymRow &Rw) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(qlo, s);
            const int64_t hi = __builtin_amdgcn_readlane(qhi, s);
            const int a = __builtin_amdgcn_readlane(qa, s), b = __builtin_amdgcn_readlane(qb, s);
            const int c = __builtin_amdgcn_readlane(qc, s);
            Rw.v = sval + ((hi << 32) | lo);
            Rw.k0 = a & 0xFFFF;
            Rw.mu = a >> 16;
            Rw.bnx = b & 255;
            Rw.bnxy = (b >> 8) & 0xFFF;
            Rw.rx0 = ((b >> 20) & 255) - 32;
            Rw.ry0 = (c & 255) - 32;
            Rw.rz0 = ((c >> 8) & 255) - 32;
            Rw.own = (c >> 16) & 0xFFFF;
            Rw.ibnx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, qix), s));
            Rw.ibnxy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, qixy), s));
            Rw.x0 = uni_d(xl[Rw.own]);
            Rw.x1 = uni_d(xl[RN + Rw.own]);
            Rw.x2 = uni_d(xl[2 * RN + Rw.own]);
        };
        auto load_v = [&](const SymRow &Rw, int kb, double *vv, int &rr) {
            const int kk = min(kb + lane, Rw.mu - 1);
            const int q16 = Rw.mu & ~15;
            const bool ch = kk < q16;
            const int64_t o0 = ch ? (int64_t)((kk >> 4) * 144 + (kk & 15)) : (int64_t)q16 * 9 + (kk - q16);
            const int st = ch ? 16 : Rw.mu - q16;
            unsigned o[9];
#pragma unroll
            for (int s = 0; s < 9; ++s) o[s] = (unsigned)(o0 + s * st) * 8u;
            sym_ld9(vv, Rw.v, o);
            const int k = Rw.k0 + kk;
            const int kzz = sym_div(k, Rw.bnxy, Rw.ibnxy), rem = k - kzz * Rw.bnxy;
            const int ky = sym_div(rem, Rw.bnx, Rw.ibnx), kx = rem - ky * Rw.bnx;
            rr = (Rw.rx0 + kx) + RX * ((Rw.ry0 + ky) + RY * cw_ring(Rw.rz0 + kzz, s0, RZ));
        };
        // the issue cursor (row I, slot xi, pass ki) runs one item ahead of the
        // compute cursor; the first item of a tile is issued before the
        // transition into it (its rows' x lie in the previous tile's window)
        int xi = NS, ki = 0;
        bool any = false, idone = true;
        SymRow I, C;
        double v0[9], v1[9];
        int ra = 0, rb = 0;
        auto tile_begin = [&]() {  // zk, s0 and the decoded slots of the tile
            xi = next_slot(0);
            ki = 0;
            any = xi < NS;
            idone = !any;
            if (any) {
                slot_row(xi, I);
            } else {  // no rows of this wave in the tile: a dummy item
                I.v = sval;
                I.mu = 1;
                I.k0 = 0;
                I.bnx = I.bnxy = 1;
                I.ibnx = I.ibnxy = 1.0f;
                I.rx0 = I.ry0 = I.rz0 = 0;
                I.own = 0;
            }
            load_v(I, ki, v0, ra);
        };
        auto issue_next = [&]() {
            if (idone) return;
            if (ki + 64 < I.mu) {
                ki += 64;
                return;
            }
            const int nx2 = next_slot(xi + 1);
            if (nx2 >= NS) {
                idone = true;
                return;
            }
            xi = nx2;
            ki = 0;
            slot_row(xi, I);
        };
        // Helper and compute waves run separate loops with the same barrier
        // sequence (cold start, then T1 / T2 per tile): the helper's entering-x
        // registers are then not live across the compute waves' item loop.
        if (helper) {
            // the storer: it issues no loads, so no wait of its own ever covers
            // its stores; they drain in the background
            __syncthreads();  // cold start done
            for (int kz = R.kz0; kz < R.kz1; ++kz) {
                const bool last = kz + 1 >= R.kz1;
                lds_barrier();  // T1: the tile's adds are done
                // the leaving planes z1 .. z1 + TZ - 1 are final for this column;
                // at the run's end also the P planes above (overlap slabs)
                const int z1 = kz * TZ, zo = last ? zhi : min(z1 + TZ, g.Lz);
                for (int z = z1; z < zo; ++z)
                    y_out(z, z < zr1 ? wsA + ((int64_t)R.c * g.Lz + z) * 3 * RXY
                                     : wsB + (int64_t)(R.ovl + z - zr1) * 3 * RXY);
                lds_barrier();  // T2: the window of tile kz + 1 is in LDS
            }
            continue;
        }
        desc_load(R.kz0);
        sym_waitn<0>();
        desc_wait();
        __syncthreads();  // cold start done: x window and zeroed y ring in LDS
        desc_decode();
        tile_begin();
        for (int kz = R.kz0; kz < R.kz1; ++kz) {
            const bool last = kz + 1 >= R.kz1;
            if (!last) desc_load(kz + 1);  // (in flight during the tile)
            if (any && !(probe & 1024)) {  // (timing probe 1024: no items)
                int xc = xi, kc = 0;
                C = I;
                C.x0 = uni_d(xl[C.own]);  // (issued before the window was complete)
                C.x1 = uni_d(xl[RN + C.own]);
                C.x2 = uni_d(xl[2 * RN + C.own]);
                double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
                auto step = [&](double *vv, const int rr, double *vn, int &rn) {
                    issue_next();
                    load_v(I, ki, vn, rn);
                    const double xv0 = xl[rr], xv1 = xl[RN + rr], xv2 = xl[2 * RN + rr];
                    sym_wait9<9>(vv);
                    const int kk = kc + lane;
                    const bool live = kk < C.mu;
                    const int rt = live && kk > 0 ? rr : RN + lane;
                    const double s0v = vv[0] * xv0 + vv[1] * xv1 + vv[2] * xv2;
                    const double s1v = vv[3] * xv0 + vv[4] * xv1 + vv[5] * xv2;
                    const double s2v = vv[6] * xv0 + vv[7] * xv1 + vv[8] * xv2;
                    acc0 += live ? s0v : 0.0;
                    acc1 += live ? s1v : 0.0;
                    acc2 += live ? s2v : 0.0;
                    const double t0 = vv[0] * C.x0 + vv[3] * C.x1 + vv[6] * C.x2;
                    const double t1 = vv[1] * C.x0 + vv[4] * C.x1 + vv[7] * C.x2;
                    const double t2 = vv[2] * C.x0 + vv[5] * C.x1 + vv[8] * C.x2;
                    if (DET) {
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
                    // the row is done: its direct sum (fixed-order DPP) into its own node
                    acc0 = wsum_dpp(acc0);
                    acc1 = wsum_dpp(acc1);
                    acc2 = wsum_dpp(acc2);
                    if (lane < 3) {
                        const double s = lane == 0 ? acc0 : lane == 1 ? acc1 : acc2;
                        if (DET) atomicAdd(&yi[lane * RS + C.own], fx_of(s, S));
                        else atomicAdd(&yl[lane * RS + C.own], s);
                    }
                    acc0 = acc1 = acc2 = 0.0;
                    const int nx2 = next_slot(xc + 1);
                    if (nx2 >= NS) return false;
                    xc = nx2;
                    kc = 0;
                    slot_row(xc, C);
                    return true;
                };
                while (step(v0, ra, v1, rb) && step(v1, rb, v0, ra)) {
                }
            }
            sym_wait9<0>(v0);  // (the last, re-read item: L2 hits; the descriptors too)
            sym_wait9<0>(v1);
            if (!last) {
                // tile kz + 1's new x planes, issued once this wave's items are
                // done (holding them over the whole tile costs spills), and its
                // first item, both in flight across the transition
                desc_wait();
                xe_load(kz + 1);
                zk += TZ;
                s0 = zk % RZ;
                desc_decode();
                tile_begin();
            }
            lds_barrier();  // T1: the tile's adds are done
            if (!last) {
                sym_waitn<9>();  // the x planes (the next item's 9 loads stay in flight)
                xe_store(kz + 1);  // into the slots of planes kz * TZ .. + TZ - 1 (outside tile kz + 1's window)
            }
            lds_barrier();  // T2: the window of tile kz + 1 is in LDS
        }
    }
}

// W_run of the DET column walk: for each node j of the run's region, the
// sum over the run's rows i with j in i's stored blocks (j != i) of
// max_b sum_a |B_ij[a][b]|, plus, when j is a row of the run, the sum over its
// stored blocks of max_a sum_b |B_jk[a][b]| -- a bound on |partial_j| per
// unit max|x| over the region; run_e[r] = e with 2^e > max_j.  Fixed order.
__global__ __launch_bounds__(256) void k_sym_bound_cw(SymGeo g, const int *__restrict__ rowbox,
                                                      const int64_t *__restrict__ svptr,
                                                      const double *__restrict__ sval,
                                                      const SymRun *__restrict__ runs, int *__restrict__ run_e)
{
    __shared__ double wred[256];
    const SymRun R = runs[blockIdx.x];
    const int TZ = SYM_TZ, P = g.P;
    const int tix = R.c % g.ntx, tiy = R.c / g.ntx;
    const int x0 = tix * SYM_TX, y0 = tiy * SYM_TY, ox = x0 - P, oy = y0 - P;
    const int zr0 = R.kz0 * TZ, zr1 = min(R.kz1 * TZ, g.Lz), zhi = min(zr1 + P, g.Lz);
    const int64_t Lxy = (int64_t)g.Lx * g.Ly;
    const int RXY = g.RX * g.RY;
    auto blk = [&](const double *v, int kk, int mu, bool tr) {
        double bm = 0.0;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            double cs = 0.0;
#pragma unroll
            for (int a = 0; a < 3; ++a) cs += fabs(v[vofs(1, 9, tr ? a * 3 + b : b * 3 + a, kk, mu, mu)]);
            bm = fmax(bm, cs);
        }
        return bm;
    };
    double wm = 0.0;
    for (int k = threadIdx.x; k < RXY * (zhi - zr0); k += 256) {
        const int pz = k / RXY, rem = k - pz * RXY, ry = rem / g.RX, rx = rem - ry * g.RX;
        const int gx = ox + rx, gy = oy + ry, gz = zr0 + pz;
        if (gx < 0 || gx >= g.Lx || gy < 0 || gy >= g.Ly) continue;
        double s = 0.0;
        for (int zi = max(zr0, gz - P); zi <= min(zr1 - 1, gz); ++zi)
            for (int yi = y0; yi < min(y0 + SYM_TY, g.Ly); ++yi)
                for (int xi = x0; xi < min(x0 + SYM_TX, g.Lx); ++xi) {
                    const int64_t i = xi + (int64_t)g.Lx * yi + Lxy * zi;
                    const int64_t base = rowbox[2 * i];
                    const int d = rowbox[2 * i + 1];
                    const int bz = (int)(base / Lxy), by = (int)((base - bz * Lxy) / g.Lx);
                    const int bx = (int)(base - bz * Lxy - (int64_t)by * g.Lx);
                    const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
                    if (gx < bx || gx >= bx + bnx || gy < by || gy >= by + bny || gz < bz || gz >= bz + bnz) continue;
                    const int k0 = (xi - bx) + bnx * ((yi - by) + bny * (zi - bz));
                    const int kj = (gx - bx) + bnx * ((gy - by) + bny * (gz - bz));
                    if (kj <= k0) continue;
                    const int mu = bnx * bny * bnz - k0;
                    s += blk(sval + svptr[i], kj - k0, mu, true);
                }
        if (gx >= x0 && gx < x0 + SYM_TX && gy >= y0 && gy < y0 + SYM_TY && gz < zr1) {  // j is a row of the run
            const int64_t j = gx + (int64_t)g.Lx * gy + Lxy * gz;
            const int d = rowbox[2 * j + 1];
            const int64_t base = rowbox[2 * j];
            const int bz = (int)(base / Lxy), by = (int)((base - bz * Lxy) / g.Lx);
            const int bx = (int)(base - bz * Lxy - (int64_t)by * g.Lx);
            const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
            const int k0 = (gx - bx) + bnx * ((gy - by) + bny * (gz - bz)), mu = bnx * bny * bnz - k0;
            const double *v = sval + svptr[j];
            for (int kk = 0; kk < mu; ++kk) s += blk(v, kk, mu, false);
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
        int e = -1000;
        if (wred[0] > 0.0) (void)frexp(wred[0], &e);
        run_e[blockIdx.x] = e;
    }
}

// y_j = the column partials of j's plane (2 x 2 columns whose regions hold
// it, ascending (y, x)), each followed by its overlap slabs, in that fixed order.
__global__ __launch_bounds__(256) void k_nb_sym_gather_cw(SymGeo g, const double *__restrict__ wsA,
                                                          const double *__restrict__ wsB, const int *__restrict__ ovl,
                                                          double *__restrict__ y, const int *__restrict__ istate)
{
    if (istate && istate[I_REASON] != 0) return;
    const int64_t Lxy = (int64_t)g.Lx * g.Ly, n = Lxy * g.Lz;
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int jz = (int)(j / Lxy), jy = (int)((j - jz * Lxy) / g.Lx), jx = (int)(j - jz * Lxy - (int64_t)jy * g.Lx);
    const int RXY = g.RX * g.RY;
    const int x_lo = max(0, (jx + g.P - g.RX + SYM_TX) / SYM_TX), x_hi = min(g.ntx - 1, (jx + g.P) / SYM_TX);
    const int y_lo = max(0, (jy + g.P - g.RY + SYM_TY) / SYM_TY), y_hi = min(g.nty - 1, (jy + g.P) / SYM_TY);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int ty = y_lo; ty <= y_hi; ++ty)
        for (int tx = x_lo; tx <= x_hi; ++tx) {
            const int c = ty * g.ntx + tx;
            const int q = (jy - (ty * SYM_TY - g.P)) * g.RX + (jx - (tx * SYM_TX - g.P));
            const double *p = wsA + ((int64_t)c * g.Lz + jz) * 3 * RXY + q;
            s0 += p[0];
            s1 += p[RXY];
            s2 += p[2 * RXY];
#pragma unroll
            for (int o = 0; o < 2; ++o) {
                const int k = ovl[((int64_t)c * g.Lz + jz) * 2 + o];
                if (k < 0) continue;
                const double *pb = wsB + (int64_t)k * 3 * RXY + q;
                s0 += pb[0];
                s1 += pb[RXY];
                s2 += pb[2 * RXY];
            }
        }
    y[3 * j] = s0;
    y[3 * j + 1] = s1;
    y[3 * j + 2] = s2;
}

// A copy of a matrix struct (Mat.duplicate) shares none of A's symmetric
// storage: forget the pointers (without freeing them).
void sym_forget(kle_mat *A)
{
    A->d_sval = nullptr;
    A->d_svptr = nullptr;
    A->d_sws = nullptr;
    A->d_stile_e = nullptr;
    A->d_cw_runs = nullptr;
    A->d_cw_chunk = A->d_cw_rune = A->d_cw_ovl = nullptr;
    A->d_cw_wsA = A->d_cw_wsB = nullptr;
    A->cw_nchunk = 0;
    A->cw_entries = 0;
    A->sblocks = A->snvals = A->sws_entries = 0;
    A->sym_P = 0;
}

void sym_drop(kle_mat *A)
{
    if (A->d_sval) (void)hipFree(A->d_sval);
    if (A->d_svptr) (void)hipFree(A->d_svptr);
    if (A->d_sws) (void)hipFree(A->d_sws);
    if (A->d_stile_e) (void)hipFree(A->d_stile_e);
    for (void *q : {A->d_cw_runs, (void *)A->d_cw_chunk, (void *)A->d_cw_rune, (void *)A->d_cw_ovl,
                    (void *)A->d_cw_wsA, (void *)A->d_cw_wsB})
        if (q) (void)hipFree(q);
    A->d_cw_runs = nullptr;
    A->d_cw_chunk = A->d_cw_rune = A->d_cw_ovl = nullptr;
    A->d_cw_wsA = A->d_cw_wsB = nullptr;
    A->cw_nchunk = 0;
    A->cw_entries = 0;
    A->d_sval = nullptr;
    A->d_svptr = nullptr;
    A->d_sws = nullptr;
    A->d_stile_e = nullptr;
    A->sblocks = A->snvals = A->sws_entries = 0;
    A->sym_P = 0;
}

static SymGeo sym_geo(const kle_mat *A)
{
    SymGeo g;
    const int P = A->sym_P;
    g.TX = SYM_TX;
    g.TZ = SYM_TZ;
    g.Lx = (int)A->row_lat[0];
    g.Ly = (int)A->row_lat[1];
    g.Lz = (int)A->row_lat[2];
    g.P = P;
    g.RX = g.TX + 2 * P;
    g.RY = SYM_TY + 2 * P;
    g.RZ = g.TZ + P;
    g.ntx = (g.Lx + g.TX - 1) / g.TX;
    g.nty = (g.Ly + SYM_TY - 1) / SYM_TY;
    g.ntz = (g.Lz + g.TZ - 1) / g.TZ;
    return g;
}

// LDS of the x-in-LDS kernel: x and y of the region, the tile's direct row sums
static size_t sym_xl_lds(int P)
{
    const size_t RN = (size_t)(SYM_TX + 2 * P) * (SYM_TY + 2 * P) * (SYM_TZ + P);
    return (6 * RN + 3 * 64 + 3 * SYM_TX * SYM_TY * SYM_TZ) * sizeof(double);
}
constexpr size_t LDS_PER_CU = 163840;

// LDS of the column-walk kernel: x and y rings (y with 64 dummy slots per component)
static size_t sym_cw_lds(int P)
{
    const size_t RN = (size_t)(SYM_TX + 2 * P) * (SYM_TY + 2 * P) * (SYM_TZ + P);
    return (6 * RN + 3 * 64) * sizeof(double);
}

// Column-walk work plan: the tiles in column-major order (column c =
// tiy * ntx + tix, tile kz fastest) cut into one chunk per resident
// workgroup with equal stored blocks (+ 16 per row for the per-row fixed
// cost), each chunk split into runs at column changes; a run ending below its
// column's top writes the P planes above it to overlap slabs, which the
// gather finds through ovl[(c * Lz + z) * 2 + {0, 1}].
static int cw_build(kle_mat *A, const std::vector<int> &mu_row)
{
    const SymGeo g = sym_geo(A);
    const int P = g.P, TZ = SYM_TZ;
    const int ncol = g.ntx * g.nty, ntz = g.ntz;
    const int64_t ntiles = (int64_t)ncol * ntz, Lx = g.Lx, Lxy = (int64_t)g.Lx * g.Ly;
    std::vector<double> wt(ntiles, 0.0);
    for (int c = 0; c < ncol; ++c) {
        const int x0 = (c % g.ntx) * SYM_TX, y0 = (c / g.ntx) * SYM_TY;
        for (int kz = 0; kz < ntz; ++kz) {
            double s = 0.0;
            for (int z = kz * TZ; z < std::min(kz * TZ + TZ, g.Lz); ++z)
                for (int y = y0; y < std::min(y0 + SYM_TY, g.Ly); ++y)
                    for (int x = x0; x < std::min(x0 + SYM_TX, g.Lx); ++x) s += mu_row[x + Lx * y + Lxy * z] + 16;
            wt[(int64_t)c * ntz + kz] = s + g_tune.spmv_sym_cw_tile;  // + a tile's fixed cost (transition)
        }
    }
    const int per_cu = 2 * sym_cw_lds(P) <= LDS_PER_CU ? 2 : 1;
    int64_t nch = std::min<int64_t>((int64_t)A->ctx->num_cus * per_cu, ntiles);
    double tot = 0.0;
    for (double v : wt) tot += v;
    // cut points: chunk k starts at the first tile whose prefix weight reaches k * tot / nch
    std::vector<int64_t> cut{0};
    double pre = 0.0;
    for (int64_t t = 0, k = 1; t < ntiles && k < nch; ++t) {
        pre += wt[t];
        if (pre >= (double)k * tot / nch && t + 1 < ntiles) {
            cut.push_back(t + 1);
            while (k < nch && pre >= (double)k * tot / nch) ++k;
        }
    }
    cut.push_back(ntiles);
    nch = (int64_t)cut.size() - 1;
    std::vector<SymRun> runs;
    std::vector<int> chunk_run{0};
    for (int64_t k = 0; k < nch; ++k) {
        for (int64_t t = cut[k]; t < cut[k + 1];) {
            const int c = (int)(t / ntz), kz0 = (int)(t % ntz);
            const int64_t tend = std::min<int64_t>(cut[k + 1], (int64_t)(c + 1) * ntz);
            runs.push_back({c, kz0, (int)(tend - (int64_t)c * ntz), -1});
            t = tend;
        }
        chunk_run.push_back((int)runs.size());
    }
    // overlap slabs
    std::vector<int> ovl((size_t)ncol * g.Lz * 2, -1);
    int nslab = 0;
    for (auto &R : runs) {
        const int zr1 = std::min(R.kz1 * TZ, g.Lz), zhi = std::min(zr1 + P, g.Lz);
        if (zhi <= zr1) continue;
        R.ovl = nslab;
        for (int z = zr1; z < zhi; ++z) {
            int *o = &ovl[((size_t)R.c * g.Lz + z) * 2];
            if (o[0] < 0) o[0] = nslab + z - zr1;
            else if (o[1] < 0) o[1] = nslab + z - zr1;
            else return fail(KLE_ERR_SUP, "symmetric storage: column-walk runs too short for P = %d", P);
        }
        nslab += zhi - zr1;
    }
    // lattice entries of the column partials (+ overlap slabs): written and read once per SpMV
    auto span = [](int64_t o, int64_t r, int64_t L) { return std::max<int64_t>(0, std::min(o + r, L) - std::max<int64_t>(o, 0)); };
    int64_t ents = 0;
    for (int c = 0; c < ncol; ++c) {
        const int64_t a = span((c % g.ntx) * SYM_TX - P, g.RX, g.Lx) * span((c / g.ntx) * SYM_TY - P, g.RY, g.Ly);
        int64_t planes = g.Lz;
        for (int z = 0; z < g.Lz; ++z) planes += (ovl[((size_t)c * g.Lz + z) * 2] >= 0) + (ovl[((size_t)c * g.Lz + z) * 2 + 1] >= 0);
        ents += a * planes;
    }
    const int64_t RXY = (int64_t)g.RX * g.RY;
    kle_ctx *cx = A->ctx;
    if (hipMalloc(&A->d_cw_runs, sizeof(SymRun) * runs.size()) != hipSuccess ||
        hipMalloc(&A->d_cw_chunk, sizeof(int) * chunk_run.size()) != hipSuccess ||
        hipMalloc(&A->d_cw_rune, sizeof(int) * runs.size()) != hipSuccess ||
        hipMalloc(&A->d_cw_ovl, sizeof(int) * ovl.size()) != hipSuccess ||
        hipMalloc(&A->d_cw_wsA, sizeof(double) * (size_t)ncol * g.Lz * 3 * RXY) != hipSuccess ||
        hipMalloc(&A->d_cw_wsB, sizeof(double) * (size_t)std::max(nslab, 1) * 3 * RXY) != hipSuccess) {
        (void)hipGetLastError();
        sym_drop(A);
        return fail(KLE_ERR_MEM, "out of device memory for the column-walk SpMV workspace");
    }
    KLE_HIP(hipMemcpy(A->d_cw_runs, runs.data(), sizeof(SymRun) * runs.size(), hipMemcpyHostToDevice));
    KLE_HIP(hipMemcpy(A->d_cw_chunk, chunk_run.data(), sizeof(int) * chunk_run.size(), hipMemcpyHostToDevice));
    KLE_HIP(hipMemcpy(A->d_cw_ovl, ovl.data(), sizeof(int) * ovl.size(), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_sym_bound_cw, dim3((unsigned)runs.size()), dim3(256), 0, cx->stream, g, A->d_rowbox,
                       A->d_svptr, A->d_sval, (const SymRun *)A->d_cw_runs, A->d_cw_rune);
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(cx->stream));
    A->cw_nchunk = (int)nch;
    A->cw_entries = ents;
    return 0;
}

// Build the symmetric (upper-triangle) storage of a single-rank structured
// 3x3 matrix from its full storage; refuses a matrix whose blocks are not
// symmetric to 1e-12 of its largest entry or whose pattern is not symmetric.
int sym_build(kle_mat *A)
{
    kle_ctx *c = A->ctx;
    sym_drop(A);
    if (!(A->kind == 0 && A->R == 3 && A->C == 3 && A->vlayout == 1 && A->d_rowbox && c->nranks == 1 &&
          A->ghost_lo == 0 && A->ghost_hi == 0 && A->m_local == A->n_local))
        return fail(KLE_ERR_SUP, "symmetric storage needs a single-rank 3x3 node-block matrix with box-lattice rows");
    const int64_t Lx = A->row_lat[0], Ly = A->row_lat[1], Lz = A->row_lat[2], n = A->nrows;
    if (Lx * Ly * Lz != n || A->box_lx != Lx || A->box_lxy != Lx * Ly || Lx > INT_MAX / 2)
        return fail(KLE_ERR_SUP, "symmetric storage: the rows are not one box lattice");
    std::vector<int> rb(2 * n), rp(n + 1), cnt(n);
    KLE_HIP(hipStreamSynchronize(c->stream));
    KLE_HIP(hipMemcpy(rb.data(), A->d_rowbox, sizeof(int) * 2 * n, hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(rp.data(), A->d_rowptr, sizeof(int) * (n + 1), hipMemcpyDeviceToHost));
    if (A->d_rowcnt) KLE_HIP(hipMemcpy(cnt.data(), A->d_rowcnt, sizeof(int) * n, hipMemcpyDeviceToHost));
    else
        for (int64_t i = 0; i < n; ++i) cnt[i] = rp[i + 1] - rp[i];
    std::vector<int64_t> sv(n + 1);
    std::vector<int> mu_row(n);
    int P = 0;
    int64_t tot = 0, blocks = 0, all = 0;
    const int64_t Lxy = Lx * Ly;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t z = i / Lxy, y = (i - z * Lxy) / Lx, x = i - z * Lxy - y * Lx;
        const int64_t base = rb[2 * i];
        const int d = rb[2 * i + 1];
        const int64_t bz = base / Lxy, by = (base - bz * Lxy) / Lx, bx = base - bz * Lxy - by * Lx;
        const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
        if (x < bx || x >= bx + bnx || y < by || y >= by + bny || z < bz || z >= bz + bnz ||
            cnt[i] != bnx * bny * bnz)
            return fail(KLE_ERR_SUP, "symmetric storage: row %lld's box does not hold its diagonal", (long long)i);
        P = std::max<int>(P, (int)std::max({x - bx, bx + bnx - 1 - x, y - by, by + bny - 1 - y, bz + bnz - 1 - z}));
        const int k0 = (int)((x - bx) + bnx * ((y - by) + (int64_t)bny * (z - bz)));
        const int64_t mu = cnt[i] - k0;
        mu_row[i] = (int)mu;
        sv[i] = tot;
        tot += (mu * 9 + 15) & ~int64_t(15);
        blocks += mu;
        all += cnt[i];
    }
    sv[n] = tot;
    // k_sym_build checks that every stored (i, j) has its (j, i); with that,
    // a symmetric pattern holds exactly 2 (upper blocks) - n blocks, so a
    // lower block without its upper partner shows up here
    if (2 * blocks - n != all)
        return fail(KLE_ERR_SUP, "symmetric storage: the block pattern is not symmetric (%lld blocks, %lld upper)",
                    (long long)all, (long long)blocks);
    if (sym_xl_lds(P) > LDS_PER_CU)
        return fail(KLE_ERR_SUP, "symmetric storage: row boxes reach %d nodes (at most 6 supported)", P);
    double *rowdiff = nullptr, *rowmax = nullptr;
    if (hipMalloc(&A->d_svptr, sizeof(int64_t) * (n + 1)) != hipSuccess ||
        hipMalloc(&A->d_sval, sizeof(double) * std::max<int64_t>(tot, 1)) != hipSuccess ||
        hipMalloc(&rowdiff, sizeof(double) * n) != hipSuccess || hipMalloc(&rowmax, sizeof(double) * n) != hipSuccess) {
        (void)hipGetLastError();
        hipFree(rowdiff);
        hipFree(rowmax);
        sym_drop(A);
        return fail(KLE_ERR_MEM, "out of device memory for symmetric storage");
    }
    KLE_HIP(hipMemcpy(A->d_svptr, sv.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_sym_build, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, c->stream, n, (int)Lx, (int)Ly,
                       A->d_rowptr, A->d_rowcnt, A->d_rowbox, A->d_vptr, A->d_val, A->d_svptr, A->d_sval, rowdiff,
                       rowmax);
    KLE_HIP(hipGetLastError());
    std::vector<double> hd(n), hm(n);
    KLE_HIP(hipStreamSynchronize(c->stream));
    KLE_HIP(hipMemcpy(hd.data(), rowdiff, sizeof(double) * n, hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(hm.data(), rowmax, sizeof(double) * n, hipMemcpyDeviceToHost));
    hipFree(rowdiff);
    hipFree(rowmax);
    double dmax = 0.0, vmax = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        dmax = std::max(dmax, hd[i]);
        vmax = std::max(vmax, hm[i]);
        if (std::isnan(hd[i])) dmax = INFINITY;
    }
    if (!(dmax <= 1e-12 * vmax)) {
        sym_drop(A);
        return fail(KLE_ERR_SUP, "matrix is not symmetric (max |A_ij - A_ji| = %g, max |A_ij| = %g)", dmax, vmax);
    }
    A->sym_P = P;
    const SymGeo g = sym_geo(A);
    const int64_t ntiles = (int64_t)g.ntx * g.nty * g.ntz;
    auto span = [](int64_t o, int64_t r, int64_t L) { return std::max<int64_t>(0, std::min(o + r, L) - std::max<int64_t>(o, 0)); };
    // lattice entries of every tile region (written by the SpMV, read by the gather)
    int64_t ents = 0;
    for (int64_t t = 0; t < g.ntz; ++t)
        for (int ty = 0; ty < g.nty; ++ty)
            for (int tx = 0; tx < g.ntx; ++tx)
                ents += span(tx * g.TX - P, g.RX, Lx) * span(ty * SYM_TY - P, g.RY, Ly) * span(t * g.TZ, g.RZ, Lz);
    if (hipMalloc(&A->d_sws, sizeof(double) * ntiles * 3 * g.RX * g.RY * g.RZ) != hipSuccess ||
        hipMalloc(&A->d_stile_e, sizeof(int) * ntiles) != hipSuccess) {
        (void)hipGetLastError();
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
    if (P >= 1 && P <= 4) KLE_TRY(cw_build(A, mu_row));
    return 0;
}

// Waves per workgroup of the x-in-LDS kernel: 8 while two workgroups fit a
// CU's LDS (P <= 4), else 16 (one workgroup of 16 waves per CU);
// kle_set_tuning("spmv_sym_waves") overrides.
// The x fill is one pass of SYM_FILL loads per thread: 16 waves where 8 would
// need more (P >= 5).
static bool sym_fill_fits(int P, int wv)
{
    const int RX = SYM_TX + 2 * P, NL = (SYM_TY + 2 * P) * (SYM_TZ + P), fstep = 64 * wv / (3 * RX);
    return NL <= SYM_FILL * fstep;
}

static int sym_waves(const kle_mat *A)
{
    const int P = A->sym_P;
    if (g_tune.spmv_sym_waves && sym_fill_fits(P, g_tune.spmv_sym_waves)) return g_tune.spmv_sym_waves;
    return 2 * sym_xl_lds(P) <= LDS_PER_CU && sym_fill_fits(P, 8) ? 8 : 16;
}

template <int WV, bool DET, int AHEAD>
static void launch_sym_xl(const kle_mat *A, const SymGeo &g, const kle_vec *x, const int *istate, hipStream_t st)
{
    const size_t lds = sym_xl_lds(A->sym_P);
    static size_t lds_set = 0;  // dynamic LDS above 64 KB must be declared per kernel
    if (lds > lds_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_nb_spmv_sym_xl<WV, DET, AHEAD>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        lds_set = lds;
    }
    const int64_t ntiles = (int64_t)g.ntx * g.nty * g.ntz;
    hipLaunchKernelGGL((k_nb_spmv_sym_xl<WV, DET, AHEAD>), dim3((unsigned)ntiles), dim3(64 * WV), lds, st, g,
                       A->d_rowbox, A->d_svptr, A->d_sval, x->base, A->d_sws, A->d_stile_e, istate,
                       g_tune.spmv_sym_probe);
}

template <int WV, bool DET>
static void launch_sym_xl2(const kle_mat *A, const SymGeo &g, const kle_vec *x, const int *istate, hipStream_t st)
{
    if (g_tune.spmv_sym_ahead == 1) launch_sym_xl<WV, DET, 1>(A, g, x, istate, st);
    else launch_sym_xl<WV, DET, 2>(A, g, x, istate, st);
}

static bool sym_use_cw(const kle_mat *A) { return g_tune.spmv_sym_kernel == 3 && A->d_cw_wsA && A->cw_nchunk > 0; }

int sym_spmv(const kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, hipStream_t st)
{
    const SymGeo g = sym_geo(A);
    const bool det = g_tune.spmv_sym_det != 0;
    if (sym_use_cw(A)) {
        const size_t lds = sym_cw_lds(A->sym_P);
        const SymRun *runs = (const SymRun *)A->d_cw_runs;
#define CW_LAUNCH(PP, DD)                                                                                        \
    do {                                                                                                         \
        static size_t attr = 0; /* dynamic LDS above 64 KB is declared per kernel (static LDS: red[]) */         \
        if (lds > attr) {                                                                                        \
            KLE_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_nb_spmv_sym_cw<PP, DD>),               \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                  \
            attr = lds;                                                                                          \
        }                                                                                                        \
        hipLaunchKernelGGL((k_nb_spmv_sym_cw<PP, DD>), dim3((unsigned)A->cw_nchunk), dim3(CW_NT), lds, st, g,    \
                           A->d_rowbox, A->d_svptr, A->d_sval, x->base, A->d_cw_wsA, A->d_cw_wsB, runs,          \
                           A->d_cw_chunk, A->d_cw_rune, istate, g_tune.spmv_sym_probe);                          \
    } while (0)
        switch (A->sym_P * 2 + det) {
        case 2: CW_LAUNCH(1, false); break;
        case 3: CW_LAUNCH(1, true); break;
        case 4: CW_LAUNCH(2, false); break;
        case 5: CW_LAUNCH(2, true); break;
        case 6: CW_LAUNCH(3, false); break;
        case 7: CW_LAUNCH(3, true); break;
        case 8: CW_LAUNCH(4, false); break;
        default: CW_LAUNCH(4, true); break;
        }
#undef CW_LAUNCH
        hipLaunchKernelGGL(k_nb_sym_gather_cw, dim3((unsigned)((A->nrows + 255) / 256)), dim3(256), 0, st, g,
                           A->d_cw_wsA, A->d_cw_wsB, A->d_cw_ovl, y->d, istate);
        KLE_HIP(hipGetLastError());
        return 0;
    }
    if (sym_waves(A) == 16) {
        if (det) launch_sym_xl2<16, true>(A, g, x, istate, st);
        else launch_sym_xl2<16, false>(A, g, x, istate, st);
    } else {
        if (det) launch_sym_xl2<8, true>(A, g, x, istate, st);
        else launch_sym_xl2<8, false>(A, g, x, istate, st);
    }
    hipLaunchKernelGGL((k_nb_sym_gather<SYM_TX, SYM_TZ>), dim3((unsigned)((A->nrows + 255) / 256)), dim3(256), 0, st,
                       g, A->d_sws, y->d, istate);
    KLE_HIP(hipGetLastError());
    return 0;
}

std::string sym_kernel_name(const kle_mat *A)
{
    if (sym_use_cw(A))
        return std::string("k_nb_spmv_sym_cw<") + (g_tune.spmv_sym_det ? "true" : "false") + ">+k_nb_sym_gather_cw";
    return std::string("k_nb_spmv_sym_xl<") + std::to_string(sym_waves(A)) + "," +
           (g_tune.spmv_sym_det ? "true" : "false") + "," + std::to_string(g_tune.spmv_sym_ahead == 1 ? 1 : 2) +
           ">+k_nb_sym_gather<8,2>";
}

// symmetric storage: the stored (upper) blocks, per row its value offset and
// box, x and y once, the tile partials written and read
double sym_spmv_bytes(const kle_mat *A)
{
    if (sym_use_cw(A))  // column walk: the column partials written and read
        return (double)A->sblocks * 72.0 + A->nrows * 16.0 + (double)A->nrows * 48.0 + (double)A->cw_entries * 48.0;
    return (double)A->sblocks * 72.0 + A->nrows * 16.0 + (double)A->nrows * 48.0 + (double)A->sws_entries * 48.0;
}

}  // namespace kle
