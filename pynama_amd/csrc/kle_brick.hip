// kle_brick.hip -- the box symmetric SpMV on bricks (round 5).
//
// Symmetric (SBAIJ-style, upper-triangle) storage of the structured KLE K
// (kle_mat_set_symmetric = MatSetOption(MAT_SPD); MatFS.buildFS,
// mat_fs.py:150-192; the product is the MatMult inside KSPSolve,
// kle_solver.py:35).  Block (i, j), j >= i, serves row i (B x_j) and row j
// (B^T x_i), so the rows a workgroup touches extend past the rows it owns and
// their sums meet those of other workgroups.  Rounds 2-4 cut the lattice into
// 128-row tiles and wrote each tile's region sums to HBM in the middle of the
// value stream (4.6 partial entries per row, 90 MB per SpMV at config 2);
// those stores made the stream's speed depend on where the value array lay
// (424-491 us at config 2).
//
// Here the owned lattice is cut into at most one element-aligned brick per
// CU (planner: kle_brick_plan.cpp; config 2: 254 bricks), and one 16-wave
// workgroup streams a whole brick with x AND the exact int64 fixed-point
// sums of the brick's region (config 2: about 25 x 21 x 5 nodes, 126 KB)
// resident in LDS from the first value load to the last.  The rows' direct
// sums go to y as each row ends (8 MB); nothing else is stored while the
// value array streams.  At the end each brick writes its region once
// ([entry][3]; 2.02 entries per row, 16 MB), and the graph kernels' run-mask
// gather (kle_sym.hip gsym_gather) adds, per row, the sums of the bricks
// whose regions hold it in ascending brick order (bitwise reproducible, as
// the fixed-point sums are order-free): per 64-row slice of the lattice, each
// brick region's stretch of one lattice line is one run of consecutive sums.  Inside a brick the waves take rows from
// an LDS counter, so the brick's end is one row long, not one wave's share.
// The value array is laid out brick by brick (rows in brick order, each row's
// upper tail in the 16-block chunk layout), so every CU streams one
// contiguous range.
#include <algorithm>
#include <climits>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "kle_brick.hpp"
#include "kle_internal.hpp"
#include "kle_sym_dev.hpp"

namespace kle {

using cint = __attribute__((address_space(4))) const int;

// a row of the brick (every field wave-uniform: SGPRs)
struct BRow {
    const double *v;
    int bnx, bnxy, k0, mu, rb0, ir;
};

// an issued item, packed in five words (SGPRs are the kernel's scarce
// registers): row P on lanes [0, s), row Q on lanes [s, 64) (s = 64: P
// alone), each from its first block kbP / kbQ; eP / eQ: the item ends row P /
// Q (its direct sum is complete); ok 0: a re-read past the brick's last unit
struct BItem {
    int ok;
    int ir;  // irP | irQ << 16
    int mu;  // muP | muQ << 16
    int kb;  // kbP | kbQ << 16
    int sf;  // s | eP << 8 | eQ << 9
};
__device__ __forceinline__ BItem bitem(int s, int muP, int muQ, int irP, int irQ, int kbP, int kbQ, int eP, int eQ)
{
    return {1, irP | irQ << 16, muP | muQ << 16, kbP | kbQ << 16, s | eP << 8 | eQ << 9};
}
constexpr int BI_NEWP = 1024;  // (sf: the item starts row P -- its x into the row registers)

// FF: the first item's registers are in flight when the item loop starts,
// which holds only while the compiler does not copy them on the way there
// (checked in the ISA; a variant with two items in flight ahead of the summed
// one -- no faster, round 5 -- had them moved, wrong products, and is gone)
// DOT (one rank, a split product whose gather the CG update does): the
// brick's share of (A x, x) in dpart[brick] -- its rows' direct sums and its
// region's transposed sums, each times the x it is added at (the gather adds
// every one of them to exactly one entry of A x), so the update's prologue
// has (A x, x) before any row is gathered (kle_ksp.hip k_sr_iter_g)
template <int WV, bool FF = true, bool DOT = false>
__global__ __launch_bounds__(64 * WV, 1) void k_nb_spmv_sym_brick(int Lx, int Ly, int Lz, int zo, int hp, int rstride,
                                                                 const BrickDesc *__restrict__ bd,
                                                                 const int2 *__restrict__ rowd,
                                                                 const double *__restrict__ sval,
                                                                 const double *__restrict__ x,
                                                                 double *__restrict__ ws, double *__restrict__ y,
                                                                 double *__restrict__ dpart,
                                                                 const int *__restrict__ istate KLE_PROBE_PARAM)
{
    KLE_PROBE_CONST
    constexpr int NT = 64 * WV;
    constexpr int D = 1;  // items in flight ahead of the summed one
    extern __shared__ double lds[];
    KLE_PROBE_TS(ts0)
#ifdef KLE_PROBE_BUILD
    __shared__ unsigned pmx[4];
    if (threadIdx.x == 0) pmx[0] = pmx[1] = pmx[2] = pmx[3] = 0;  // (racy by design: the other waves' maxima come microseconds later)
#endif
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NU = bd[b].nr / 2;  // units of two rows (kle_brick_plan.cpp)
    const int ox = bd[b].ox, oy = bd[b].oy, oz = bd[b].oz, RX = bd[b].RX, RY = bd[b].RY, RZ = bd[b].RZ;
    const int eb = bd[b].eb;
    const long long vbase = bd[b].vbase, wsoff = bd[b].wsoff;
    const int RN = RX * RY * RZ, RS = RN + 64, RXY = RX * RY;
    double *xl = lds;
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(lds + 3 * RN);
    double *wred = lds + 3 * RN + 3 * RS;
    int *ctr = reinterpret_cast<int *>(wred + 2 * WV);
    const int64_t Lxy = (int64_t)Lx * Ly;
    // 2a. x of the region into LDS (nodes off the lattice read 0), its max
    // |x|; the sums zeroed.  Line (ry, rz) of the region is 3 RX contiguous
    // doubles of x; a thread takes one position in a line and every fstep-th
    // line, FB loads in flight (unconditional: clamped addresses, masked
    // values).  FF: the first FB loads go out here, before anything waits on
    // the row descriptors and before the first items' value loads (asm,
    // waited for with vmcnt(9 D) in 2b), so they queue neither behind the
    // descriptor round trip nor behind the whole chip's first value loads.
    double xm = 0.0;
    int bad = 0;
    constexpr int FB = 12;
    const int L3 = 3 * RX, NL = RY * RZ;
    const int c3 = threadIdx.x % L3, l0 = threadIdx.x / L3, fstep = NT / L3;
    const int rx = c3 / 3, c = c3 - 3 * rx, gx = ox + rx;
    const bool xok = l0 < fstep && gx >= 0 && gx < Lx;
    // (line l = (ry, rz) and its offset in x stepped by fstep lines without
    // a division per load; offsets in 32 bits: brick_setup refuses lattices
    // of 2^29 / 3 or more ext nodes)
    const int dz = fstep / RY, dy = fstep - dz * RY, sy = 3 * Lx, sz = 3 * Lx * Ly;
    int fz = l0 / RY, fy = l0 - fz * RY, fo = 3 * gx + c + sy * (oy + fy) + sz * (oz + zo + fz);
    // (the unused loads -- lines past the region, threads past fstep lines:
    // most of a small brick's 12 per thread -- read the brick's first node,
    // not x[0]: one line of every brick's fill, not one line of the chip,
    // which every workgroup's dummies made a hot spot at kernel start)
    const int fdummy = 3 * (min(max(ox, 0), Lx - 1) + Lx * (min(max(oy, 0), Ly - 1) +
                                                           Ly * min(max(oz + zo, 0), zo + Lz + hp - 1))) + c;
    auto fnode = [&](int l, bool &ok) -> int {
        const int gy = oy + fy, gz = oz + fz;
        ok = xok & (l < NL) & (gy >= 0) & (gy < Ly) & (gz + zo >= 0) & (gz < Lz + hp);  // (no branches)
        const int off = ok ? fo : fdummy;
        fy += dy;
        fz += dz;
        fo += sy * dy + sz * dz;
        if (fy >= RY) {
            fy -= RY;
            ++fz;
            fo += sz - sy * RY;
        }
        return off;
    };
    auto fstore = [&](int lb, double *fv) {
#pragma unroll
        for (int f = 0; f < FB; ++f) {
            const int l = lb + f * fstep;
            const bool st = l0 < fstep && l < NL;
            xl[st ? c * RN + rx + RX * l : 4 * RN + lane] = fv[f];  // (else a dummy slot of the sums)
            const double a = fabs(fv[f]);
            bad |= !(a <= 1.7976931348623157e308);
            xm = fmax(xm, a);
        }
    };
    double fv0[FB];
    unsigned okm = 0;
    if constexpr (FF) {
#pragma unroll
        for (int f = 0; f < FB; ++f) {
            bool ok;
            const int off = fnode(l0 + f * fstep, ok);
            okm |= (unsigned)ok << f;
            ld_x1(fv0[f], x, 8u * (unsigned)off);
        }
    }
    KLE_PROBE_TS(tsi)
    // (read after the fill's loads are out: the compiler waits for it at once)
    const int stop = istate ? istate[I_REASON] : 0;  // (tested before the first store)
    // (the brick's rows at a fixed stride: their descriptors' address needs
    // no load, so their scalar loads go out beside bd's; address-space
    // cast: scalar loads)
    cint *rdesc = (cint *)(rowd + (int64_t)b * rstride);
    const double *vb = sval + vbase;
    // a row from its descriptor (kle_brick.hpp): packed box (dbx, dby, dbz,
    // bnx, bny, bnz: 4 bits each) + the low byte of its region index; value
    // offset / 16 doubles (23 bits) + the high byte
    auto row_setup = [&](int r, int dw, int vw, BRow &R) {
        const int dbx = dw & 15, dby = (dw >> 4) & 15, dbz = (dw >> 8) & 15;
        R.bnx = (dw >> 12) & 15;
        const int bny = (dw >> 16) & 15, bnz = (dw >> 20) & 15;
        R.bnxy = R.bnx * bny;
        R.k0 = dbx + R.bnx * (dby + bny * dbz);
        R.mu = R.bnxy * bnz - R.k0;
        R.ir = ((dw >> 24) & 255) | (((vw >> 24) & 255) << 8);
        R.rb0 = R.ir - (dbx + RX * (dby + RY * dbz));
        R.v = vb + (int64_t)(vw & (BRICK_ROW_NULL - 1)) * 16;
    };
    // the values of one item -- lanes below s from row P's blocks kbP + lane,
    // the others from row Q's blocks kbQ + lane - s (Q's values follow P's);
    // lanes past a row's end re-read its last block (their results go
    // nowhere) -- and each block's region index
    auto load_v = [&](const BRow &P, const BRow &Q, int kbP, int kbQ, int s, double *vv, int &rr) {
        const bool q = lane >= s;
        const int mu = q ? Q.mu : P.mu;
        const int kk = min(q ? kbQ + lane - s : kbP + lane, mu - 1);
        const int q16 = mu & ~15;
        const bool ch = kk < q16;
        const int o0 = ch ? (kk >> 4) * 144 + (kk & 15) : q16 * 9 + (kk - q16);
        const int st = ch ? 16 : mu - q16;
        const unsigned bo = q ? (unsigned)(Q.v - P.v) * 8u : 0u;
        unsigned o[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) o[t] = bo + (unsigned)(o0 + t * st) * 8u;
        // (the base is wave-uniform; said so, as the loads take it in SGPRs)
        const unsigned long long pb = (unsigned long long)P.v;
        const unsigned phi = (unsigned)__builtin_amdgcn_readfirstlane((int)(pb >> 32));
        const unsigned plo = (unsigned)__builtin_amdgcn_readfirstlane((int)(pb & 0xffffffffull));
        sym_ld9(vv, reinterpret_cast<const double *>(((unsigned long long)phi << 32) | plo), o);
        const int k = (q ? Q.k0 : P.k0) + kk;
        const int bnxy = q ? Q.bnxy : P.bnxy, bnx = q ? Q.bnx : P.bnx;
        const int kz = sym_div(k, bnxy, __builtin_amdgcn_rcpf((float)bnxy)), rem = k - kz * bnxy;
        const int ky = sym_div(rem, bnx, __builtin_amdgcn_rcpf((float)bnx)), kx = rem - ky * bnx;
        rr = (q ? Q.rb0 : P.rb0) + kx + RX * (ky + RY * kz);
    };
    // 1. units from an LDS counter; each wave's first D + 2 static (w, w + WV,
    // ...: the counter starts past them -- as many as the D items issued
    // before the fill can reach), so those go out before the fill
    auto grab = [&]() -> int {
        int r = 0;
        if (lane == 0) r = atomicAdd(ctr, 1);
        return __builtin_amdgcn_readfirstlane(r);
    };
    constexpr int NSTAT = D + 2;
    int snext = w + WV;
    auto take = [&]() -> int {  // (the next unit of this wave)
        if (snext < NSTAT * WV) {
            const int r = snext;
            snext += WV;
            return r;
        }
        return grab();
    };
    // The issue cursor over the wave's units: a unit (A, B) streams A's
    // passes (B absent: all of them; else its full ones), the item shared by
    // A's and B's last partial passes, then B's full passes.
    BRow A, B;
    bool hasB = false, idone = w >= NU;
    int ph = 0, ki = 0, aend = 0, bend = 0;
    auto unit_setup = [&](int u, int d0, int d1, int d2, int d3) {
        row_setup(2 * u, d0, d1, A);
        hasB = (d3 & BRICK_ROW_NULL) == 0;
        if (hasB) row_setup(2 * u + 1, d2, d3, B);
        else B = A;
        aend = hasB ? (A.mu & ~63) : A.mu;
        bend = hasB ? (B.mu & ~63) : 0;
        ph = aend > 0 ? 0 : 1;
        ki = 0;
    };
    if (!idone) {
        unit_setup(w, rdesc[4 * w], rdesc[4 * w + 1], rdesc[4 * w + 2], rdesc[4 * w + 3]);
    } else {
        A.v = vb;
        A.mu = 1;
        A.k0 = 0;
        A.bnx = A.bnxy = 1;
        A.rb0 = 0;
        A.ir = 0;
        B = A;
    }
#ifdef KLE_PROBE_BUILD
    if (probe_ts) {  // (probe: this wave's first row descriptors are in)
        asm volatile("" ::"s"(A.mu), "s"(A.k0));
        if (lane == 0) atomicMax(&pmx[0], (unsigned)(__builtin_amdgcn_s_memrealtime() - ts0));
    }
#endif
    // the next unit and its descriptors, fetched one unit ahead
    int pend = idone ? NU : take();
    // (a brick without rows, NU = 0, reads its slot's first unit: the table
    // holds at least one unit per brick)
    const int u0 = max(0, min(pend, NU - 1));
    int pd0 = rdesc[4 * u0], pd1 = rdesc[4 * u0 + 1];
    int pd2 = rdesc[4 * u0 + 2], pd3 = rdesc[4 * u0 + 3];
    // the item at the cursor: its loads into vn, its record; the cursor then
    // moves on (past the last unit it stays, re-reading the last item)
    auto issue = [&](double *vn, int &rn, BItem &itn) {
        if (idone) {  // (a re-read of A's first pass: cache hits, the results go nowhere)
            load_v(A, A, 0, 0, 64, vn, rn);
            itn.ok = 0;
            return;
        }
        if (ph == 0) {  // A's passes
            load_v(A, A, ki, 0, 64, vn, rn);
            itn = bitem(64, A.mu, A.mu, A.ir, A.ir, ki, 0, !hasB && ki + 64 >= A.mu, 0);
            if (ki == 0) itn.sf |= BI_NEWP;
            ki += 64;
            if (ki >= aend) ph = hasB ? 1 : 3;
        } else if (ph == 1) {  // A's and B's last partial passes
            const int s = A.mu - aend;
            load_v(A, B, aend, bend, s, vn, rn);
            itn = bitem(s, A.mu, B.mu, A.ir, B.ir, aend, bend, 1, bend == 0);
            if (aend == 0) itn.sf |= BI_NEWP;
            ki = 0;
            ph = bend > 0 ? 2 : 3;
        } else {  // B's full passes
            load_v(B, B, ki, 0, 64, vn, rn);
            itn = bitem(64, B.mu, B.mu, B.ir, B.ir, ki, 0, ki + 64 >= bend, 0);
            ki += 64;
            if (ki >= bend) ph = 3;
        }
        if (ph == 3) {  // the unit is done: the next one
            if (pend >= NU) {
                idone = true;
            } else {
                unit_setup(pend, pd0, pd1, pd2, pd3);
                pend = take();
                const int u = max(0, min(pend, NU - 1));
                pd0 = rdesc[4 * u];
                pd1 = rdesc[4 * u + 1];
                pd2 = rdesc[4 * u + 2];
                pd3 = rdesc[4 * u + 3];
            }
        }
    };
    double v0[9], v1[9];
    int r0 = 0, r1 = 0;
    BItem i0, i1;
#ifdef KLE_PROBE_BUILD
    unsigned long long tsf = 0;
#endif
    // 2b. the first item's value loads, then the fill's first loads landed
    // (vmcnt(9): the value loads stay in flight), into LDS; further lines
    // (regions of more than FB x fstep lines) after them
    {
        int lb = l0;
        if constexpr (FF) {
            issue(v0, r0, i0);
#ifdef KLE_PROBE_BUILD
            if (probe_ts && lane == 0) {
                atomicMax(&pmx[2], (unsigned)(__builtin_amdgcn_s_memrealtime() - ts0));
                atomicMax(&pmx[3], (unsigned)ts0);  // (the latest wave's start)
            }
#endif
            wait_x12<9 * D>(fv0);
#ifdef KLE_PROBE_BUILD
            tsf = probe_ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
#endif
#pragma unroll
            for (int f = 0; f < FB; ++f) fv0[f] = (okm >> f) & 1u ? fv0[f] : 0.0;
            fstore(lb, fv0);
            lb += FB * fstep;
        } else {
            issue(v0, r0, i0);
        }
        for (; lb < NL; lb += FB * fstep) {
            double fv[FB];
#pragma unroll
            for (int f = 0; f < FB; ++f) {
                bool ok;
                const int off = fnode(lb + f * fstep, ok);
                const double v = x[off];
                fv[f] = ok ? v : 0.0;
            }
            fstore(lb, fv);
        }
    }
    for (int k = threadIdx.x; k < 3 * RS; k += NT) acc[k] = 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) xm = fmax(xm, __shfl_xor(xm, o, 64));
    const unsigned long long anybad = __ballot(bad);
    if (lane == 0) {
        wred[w] = xm;
        wred[WV + w] = anybad ? 1.0 : 0.0;
    }
    if (threadIdx.x == 0) *ctr = NSTAT * WV;
#ifdef KLE_PROBE_BUILD
    // (probe: the latest wave's fill landed and its arrival at the barrier)
    if (probe_ts && lane == 0) {
        atomicMax(&pmx[1], (unsigned)(__builtin_amdgcn_s_memrealtime() - ts0));
    }
#endif
    __builtin_amdgcn_s_waitcnt(0xC07F);  // LDS stores done (lgkmcnt 0); the value loads stay in flight
    __builtin_amdgcn_s_barrier();
    if (__builtin_amdgcn_readfirstlane(stop) != 0) return;  // (nothing written yet)
    // the brick's scale: 2^(61 - E), 2^E > (its sums' bound, k_brick_bound) x
    // max |x|, as two factors S1 S2 (and 1 / S as T1 T2), each a normal
    // double, so that x near the bottom of the exponent range (2^(61 - E) >
    // 2^1023) keeps its 61 bits too
    double S1 = 1.0, S2 = 1.0, T1 = 1.0, T2 = 1.0;
    {
        double m = 0.0, nb = 0.0;
#pragma unroll
        for (int q = 0; q < WV; ++q) {
            m = fmax(m, wred[q]);
            nb += wred[WV + q];
        }
        if (nb != 0.0) {
            S1 = 0.0;  // non-finite x: NaN sums, as a floating-point product would give
            T1 = __builtin_nan("");
        } else if (m > 0.0) {
            int em;
            (void)frexp(m, &em);
            const int E = min(max(eb + em, -1070), 1020);
            const int e1 = min(61 - E, 1000), e2 = 61 - E - e1;
            S1 = ldexp(1.0, e1);
            S2 = ldexp(1.0, e2);
            T1 = ldexp(1.0, -e1);
            T2 = ldexp(1.0, -e2);
        }
    }
    KLE_PROBE_TS(ts1)
    // 3. The issue cursor runs D items in front of the compute cursor; each
    // issued item leaves a record (rows, lengths, region indices, first
    // blocks, which rows it ends), so the compute cursor needs no state of
    // the issue cursor.  Past the brick's last unit the issue cursor re-reads
    // its last item under a record r = -1, so every step issues 9 loads and
    // the wait for the summed item is a fixed vmcnt(9 D).
    double dr = 0.0;  // DOT: this lane's share of its rows' (direct sum, x)
    if (i0.ok) {
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
        double cx0 = 0.0, cx1 = 0.0, cx2 = 0.0;  // x of the current row, kept across its items
        // the row's direct sum (fixed-order DPP, fp64), one writer, into y --
        // the gather adds the bricks' transposed sums to it (8 MB of stores
        // at config 2: the only ones before the end)
        // DOT: each lane's part of the row's sum times the row's x, c (the
        // lanes of other rows hold 0 of this row's sum), before the lanes'
        // sum -- all in VGPRs (SGPRs are the kernel's scarce registers)
        auto row_out = [&](int ir, double a0, double a1, double a2, double xr0, double xr1, double xr2) {
            if constexpr (DOT) dr += (a0 * xr0 + a1 * xr1) + a2 * xr2;
            wsum3_dpp(a0, a1, a2);
            // (the row's lattice node from its region index: bricks may be
            // ragged, kle_brick_plan.cpp)
            const int irz = ir / RXY, irem = ir - irz * RXY, iry = irem / RX, irx = irem - iry * RX;
            const int64_t j = (ox + irx) + (int64_t)Lx * (oy + iry) + Lxy * (oz + irz);
            if (lane < 3) y[3 * j + lane] = lane == 0 ? a0 : lane == 1 ? a1 : a2;
        };
        // one step: issue the next item into vn, wait for vv (the D newer
        // items stay in flight), sum it
        auto step = [&](double *vv, const int rr, const BItem &it, double *vn, int &rn, BItem &itn) {
            issue(vn, rn, itn);
            if (!it.ok) return false;
            const int is = it.sf & 255, irP = it.ir & 0xFFFF, irQ = (int)((unsigned)it.ir >> 16);
            const bool q = lane >= is;
            // x of the lane's row (P's below s, Q's from s on); the row
            // registers hold P's from its first item on, Q's after a shared
            // one (0.35 % ahead of reading it per item, profiles/r05/pair/)
            double p0, p1, p2;
            if (it.sf & BI_NEWP) {
                p0 = uni_d(xl[irP]);
                p1 = uni_d(xl[RN + irP]);
                p2 = uni_d(xl[2 * RN + irP]);
                cx0 = p0, cx1 = p1, cx2 = p2;
            } else {
                p0 = cx0, p1 = cx1, p2 = cx2;
            }
            double c0 = p0, c1 = p1, c2 = p2;
            if (is < 64) {
                const double q0 = uni_d(xl[irQ]), q1 = uni_d(xl[RN + irQ]), q2 = uni_d(xl[2 * RN + irQ]);
                c0 = q ? q0 : p0;
                c1 = q ? q1 : p1;
                c2 = q ? q2 : p2;
                cx0 = q0, cx1 = q1, cx2 = q2;
            }
            const double xj0 = xl[rr], xj1 = xl[RN + rr], xj2 = xl[2 * RN + rr];
            sym_wait9<9 * D>(vv);
            // B x_j into the row, B^T x_i into row j (lanes past the row's end
            // and the diagonal block add into their dummy slot)
            const int kk = q ? (int)((unsigned)it.kb >> 16) + lane - is : (it.kb & 0xFFFF) + lane;
            const bool live = kk < (q ? (int)((unsigned)it.mu >> 16) : (it.mu & 0xFFFF));
            const int rt = live && kk > 0 ? rr : RN + lane;
            const double s0 = vv[0] * xj0 + vv[1] * xj1 + vv[2] * xj2;
            const double s1 = vv[3] * xj0 + vv[4] * xj1 + vv[5] * xj2;
            const double s2 = vv[6] * xj0 + vv[7] * xj1 + vv[8] * xj2;
            const double t0 = vv[0] * c0 + vv[3] * c1 + vv[6] * c2;
            const double t1 = vv[1] * c0 + vv[4] * c1 + vv[7] * c2;
            const double t2 = vv[2] * c0 + vv[5] * c1 + vv[8] * c2;
            if (!(probe & 1)) {  // (timing probe 1: no transposed adds)
                atomicAdd(&acc[rt], fx_of(t0 * S1, S2));
                atomicAdd(&acc[RS + rt], fx_of(t1 * S1, S2));
                atomicAdd(&acc[2 * RS + rt], fx_of(t2 * S1, S2));
            } else if (!live) {
                acc[RN + lane] += (unsigned long long)(t0 + t1 + t2);
            }
            const bool mine = live && !q;  // (P's lanes)
            acc0 += mine ? s0 : 0.0;
            acc1 += mine ? s1 : 0.0;
            acc2 += mine ? s2 : 0.0;
            if (it.sf & 256) {
                row_out(irP, acc0, acc1, acc2, c0, c1, c2);
                // (Q's lanes start Q's sum)
                const bool qs = live && q;
                acc0 = qs ? s0 : 0.0;
                acc1 = qs ? s1 : 0.0;
                acc2 = qs ? s2 : 0.0;
                if (it.sf & 512) {
                    row_out(irQ, acc0, acc1, acc2, c0, c1, c2);
                    acc0 = acc1 = acc2 = 0.0;
                }
            }
            return true;
        };
        while (step(v0, r0, i0, v1, r1, i1) && step(v1, r1, i1, v0, r0, i0)) {
        }
    }
    // the last (re-read) loads land before their registers are reused
    sym_wait9<0>(v0);
    sym_wait9<0>(v1);
    __syncthreads();
    KLE_PROBE_TS(ts2)
    // 4. the region's transposed sums, once, [entry][3] (coalesced; nodes
    // off the lattice are never read)
    double *dst = ws + wsoff;
    double ds = 0.0;  // DOT: this thread's (region sum, x)
    for (int t = threadIdx.x; t < 3 * RN; t += NT) {
        const int k = t / 3, c = t - 3 * k;
        const int rz = k / (RX * RY), rem = k - rz * RX * RY, ry = rem / RX, rx = rem - ry * RX;
        const int gx = ox + rx, gy = oy + ry, gz = oz + rz;
        if (gx < 0 || gx >= Lx || gy < 0 || gy >= Ly || gz + zo < 0 || gz >= Lz + hp) continue;
        const double v = fx_to_d(acc[c * RS + k]) * T1 * T2;
        dst[t] = v;
        if constexpr (DOT) ds += v * xl[c * RN + k];
    }
    if constexpr (DOT) {
        // fixed order: lanes (xor tree), then waves in order
        double s = ds + dr;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) wred[w] = s;  // (wred's scale inputs were read before the item loop)
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
#pragma unroll
            for (int q = 0; q < WV; ++q) t += wred[q];
            dpart[b] = t;
        }
    }
    KLE_PROBE_TS_END5(b, ts0, ts1, ts2, ts0 + pmx[0], ts0 + pmx[1], ts0 + pmx[2])
#ifdef KLE_PROBE_BUILD
    if (probe_ts && threadIdx.x == 0 && (int64_t)b < probe_cap)  // (the waves' start spread, 10 ns units)
        probe_ts[8 * (int64_t)b] |= (unsigned long long)(pmx[3] - (unsigned)ts0) << 32;
#endif
}

// y[0 .. n) += r: the lower neighbour's sums for this slab's lowest nodes
// (the reverse halo), added last -- after the bricks', in a fixed order
__global__ void k_brick_add_recv(int64_t n, const double *__restrict__ r, double *__restrict__ y,
                                 const int *__restrict__ istate)
{
    if (istate && istate[I_REASON] != 0) return;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) y[t] += r[t];
}

// Per brick: eb with 2^eb > the largest, over its region nodes j, of
//   sum over the brick's rows i != j with j in i's stored blocks of
//   max_b sum_a |B_ij[a][b]|   (the transposed adds, each <= that x max|x|)
// + (j owned by the brick) max_a sum over row j's stored blocks of sum_b |B[a][b]|
// (its direct sum), so no region sum can exceed 2^61 at the scale 2^(61-E),
// E = eb + (exponent of max |x| over the region).  Fixed summation order.
__global__ __launch_bounds__(256) void k_brick_bound(int Lx, int Ly, int Lz, int zo, int hp,
                                                     const BrickDesc *__restrict__ bd, const int *__restrict__ rowbox,
                                                     const int *__restrict__ smu, const int64_t *__restrict__ svptr,
                                                     const double *__restrict__ sval, int P,
                                                     const int *__restrict__ owner, int *__restrict__ ebo)
{
    __shared__ double wred[256];
    const int b = blockIdx.x;
    const BrickDesc D = bd[b];
    const int RN = D.RX * D.RY * D.RZ;
    const int64_t Lxy = (int64_t)Lx * Ly;
    double wm = 0.0;
    for (int k = threadIdx.x; k < RN; k += 256) {
        const int rz = k / (D.RX * D.RY), rem = k - rz * D.RX * D.RY, ry = rem / D.RX, rx = rem - ry * D.RX;
        const int gx = D.ox + rx, gy = D.oy + ry, gz = D.oz + rz;  // (owned z)
        if (gx < 0 || gx >= Lx || gy < 0 || gy >= Ly || gz + zo < 0 || gz >= Lz + hp) continue;
        double s = 0.0;
        // rows i of the brick whose boxes may hold j: within P of it, not above it
        for (int iz = max(D.z0, gz - P); iz <= min(D.z0 + D.nz - 1, gz); ++iz)
            for (int iy = max(D.y0, gy - P); iy <= min(D.y0 + D.ny - 1, gy + P); ++iy)
                for (int ix = max(D.x0, gx - P); ix <= min(D.x0 + D.nx - 1, gx + P); ++ix) {
                    const int64_t i = ix + (int64_t)Lx * iy + Lxy * iz;
                    if (owner[i] != b) continue;  // (a ragged brick's bounding box holds others' rows)
                    const int64_t base = rowbox[2 * i];
                    const int d = rowbox[2 * i + 1];
                    const int bze = (int)(base / Lxy), by = (int)((base - bze * Lxy) / Lx);
                    const int bx = (int)(base - bze * Lxy - (int64_t)by * Lx), bz = bze - zo;
                    const int bnx = d & 255, bny = (d >> 8) & 255, bnz = (d >> 16) & 255;
                    if (gx < bx || gx >= bx + bnx || gy < by || gy >= by + bny || gz < bz || gz >= bz + bnz) continue;
                    const int k0 = (ix - bx) + bnx * ((iy - by) + bny * (iz - bz));
                    const int kj = (gx - bx) + bnx * ((gy - by) + bny * (gz - bz));
                    if (kj <= k0) continue;  // (lower triangle or the diagonal block)
                    const int mu = bnx * bny * bnz - k0, kk = kj - k0;
                    const double *v = sval + svptr[i];
                    double bmax = 0.0;
#pragma unroll
                    for (int bb = 0; bb < 3; ++bb) {
                        double cs = 0.0;
#pragma unroll
                        for (int a = 0; a < 3; ++a) cs += fabs(v[vofs(1, 9, a * 3 + bb, kk, mu, mu)]);
                        bmax = fmax(bmax, cs);
                    }
                    s += bmax;
                }
        if (gz < Lz && owner[gx + (int64_t)Lx * gy + Lxy * gz] == b) {
            // the row's own direct sum
            const int64_t j = gx + (int64_t)Lx * gy + Lxy * gz;
            const int mu = smu[j];  // (stored blocks of row j)
            const double *v = sval + svptr[j];
            double rmax = 0.0;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double rs = 0.0;
                for (int kk = 0; kk < mu; ++kk)
#pragma unroll
                    for (int bb = 0; bb < 3; ++bb) rs += fabs(v[vofs(1, 9, a * 3 + bb, kk, mu, mu)]);
                rmax = fmax(rmax, rs);
            }
            s += rmax;
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
        int e = -1000;  // (an all-zero brick)
        if (wred[0] > 0.0) (void)frexp(wred[0], &e);
        ebo[b] = e;
    }
}

// ---------------------------------------------------------------------------
// host side

int brick_setup(kle_mat *A, const std::vector<int> &rb, const std::vector<int> &cnt, const std::vector<int> &srow,
                int P, std::vector<int64_t> &svptr_out, std::string &why, void **plan_out)
{
    auto *bp = new BrickPlan;
    bp->singles = g_tune.spmv_brick_singles;
    bp->pair = g_tune.spmv_brick_pair;
    const int64_t plane3 = 3 * A->row_lat[0] * A->row_lat[1];
    if (A->ghost_lo + 3 * A->nrows + A->ghost_hi >= (int64_t)1 << 29) {  // (the fill's 32-bit byte offsets)
        delete bp;
        why = "brick SpMV: 2^29 / 3 ext nodes or more";
        *plan_out = nullptr;
        return 0;
    }
    // k whole rounds of one brick per CU, k from spmv_brick_rounds up to the
    // fewest whose largest region fits the LDS (config 4, p = 6 on one GPU:
    // 4 rounds; one round at p = 4 and for p = 6 z slabs of 8 ranks)
    for (int rounds = std::max(1, g_tune.spmv_brick_rounds); rounds <= BRICK_MAX_ROUNDS; ++rounds) {
        try {  // (no exception may cross the C ABI: a planner failure is a refusal)
            why = brick_plan((int)A->row_lat[0], (int)A->row_lat[1], (int)A->row_lat[2],
                             (int)(A->ghost_hi / plane3), std::max(1, A->ctx->num_cus), g_tune.spmv_brick_max, rounds,
                             g_tune.spmv_brick_split, cnt, srow, P, *bp);
        } catch (const std::exception &e) {
            why = std::string("brick planner: ") + e.what();
        }
        if (why.empty() || g_tune.spmv_brick_max > 0 || g_tune.spmv_brick_split > 0 ||
            why.find("fits the LDS") == std::string::npos)
            break;
        *bp = BrickPlan{};
        bp->singles = g_tune.spmv_brick_singles;
        bp->pair = g_tune.spmv_brick_pair;
    }
    if (!why.empty()) {
        delete bp;
        *plan_out = nullptr;
        return 0;
    }
    svptr_out = bp->svb;
    *plan_out = bp;
    return 0;
}

// after the values are in place (d_sval, d_svptr in brick layout): the brick
// tables on the device, the workspace, the bound exponents
int brick_finish(kle_mat *A, void *plan)
{
    std::unique_ptr<BrickPlan> bp(reinterpret_cast<BrickPlan *>(plan));
    kle_ctx *c = A->ctx;
    const int NB = (int)bp->bricks.size();
    // every address the kernel forms from the tables, checked on the host
    // first (a bad plan is an error, never a launch)
    {
        const char *bad = brick_validate(*bp, A->row_lat[0], A->row_lat[1], A->row_lat[2], A->snvals, (int64_t)bp->lds);
        if (bad) return fail(KLE_ERR_SUP, "brick plan: %s", bad);
    }
    int rstride = 0;  // rows per brick in the descriptor table (the most of any brick)
    for (const BrickDesc &D : bp->bricks) rstride = std::max(rstride, D.nr);
    rstride = std::max(2, (rstride + 1) & ~1);  // (whole units of two rows, at least one)
    const int64_t n = A->nrows;
    int *dmu = nullptr;
    std::vector<int> hmu(2 * n, 0);  // stored blocks per row | owning brick per row (-1: a one-block row)
    int *howner = hmu.data() + n;
    std::fill(howner, howner + n, -1);
    for (int64_t i : bp->srows) hmu[i] = 1;
    bool nomem = hipMalloc(&A->d_bdesc, sizeof(BrickDesc) * std::max(NB, 1)) != hipSuccess ||
                 hipMalloc(&A->d_browd, sizeof(int) * 2 * std::max<int64_t>(1, (int64_t)NB * rstride)) != hipSuccess ||
                 (A->ghost_hi && hipMalloc(&A->d_sgsend, sizeof(double) * A->ghost_hi) != hipSuccess) ||
                 (A->send_lo && hipMalloc(&A->d_sgrecv, sizeof(double) * A->send_lo) != hipSuccess) ||
                 hipMalloc(&A->d_sws, sizeof(double) * std::max<int64_t>(bp->ws_doubles, 1)) != hipSuccess ||
                 hipMalloc(&A->d_stile_e, sizeof(int) * std::max(NB, 1)) != hipSuccess ||
                 hipMalloc(&dmu, sizeof(int) * 2 * n) != hipSuccess;
    (void)hipGetLastError();
    if (nomem) {
        if (dmu) (void)hipFree(dmu);
        return fail(KLE_ERR_MEM, "out of device memory for the symmetric SpMV bricks");
    }
    A->sws_bytes = sizeof(double) * std::max<int64_t>(bp->ws_doubles, 1);
    // stored blocks per row (the bound's direct sums) from the row descriptors
    {
        for (int q = 0; q < NB; ++q) {
            const BrickDesc &D = bp->bricks[q];
            for (int r = 0; r < D.nr; ++r) {
                const int64_t rr = (int64_t)D.rstart + r;
                if (brick_row_null(bp->rowd.data(), rr)) continue;
                const int d = bp->rowd[2 * rr];
                const int dbx = d & 15, dby = (d >> 4) & 15, dbz = (d >> 8) & 15;
                const int bnx = (d >> 12) & 15, bny = (d >> 16) & 15, bnz = (d >> 20) & 15;
                const int64_t i = brick_ir_node(D, brick_row_ir(bp->rowd.data(), rr), A->row_lat[0], A->row_lat[1]);
                hmu[i] = bnx * bny * bnz - (dbx + bnx * (dby + bny * dbz));
                howner[i] = q;
            }
        }
    }
    KLE_TRY(h2d(A->d_bdesc, bp->bricks.data(), sizeof(BrickDesc) * NB));
    {
        // the row descriptors, brick q's at row q rstride (the kernel's
        // address needs no load); the rows past a brick's own repeat its
        // last unit (never read: every read is of a unit < nr / 2)
        std::vector<int> pad((size_t)2 * std::max<int64_t>(1, (int64_t)NB * rstride), 0);
        for (int q = 0; q < NB; ++q) {
            const BrickDesc &D = bp->bricks[q];
            int *dst = pad.data() + 2 * (int64_t)q * rstride;
            std::copy(bp->rowd.begin() + 2 * (int64_t)D.rstart, bp->rowd.begin() + 2 * ((int64_t)D.rstart + D.nr), dst);
            for (int r = D.nr; r < rstride && D.nr >= 2; ++r) {
                dst[2 * r] = dst[2 * (D.nr - 2 + (r & 1))];
                dst[2 * r + 1] = dst[2 * (D.nr - 2 + (r & 1)) + 1];
            }
        }
        KLE_TRY(h2d(A->d_browd, pad.data(), sizeof(int) * pad.size()));
    }
    A->brick_rstride = rstride;
    {
        // the gather's runs (kle_sym.hip gsym_gather, the graph kernels'
        // gather): per 64-row slice of [owned | upper ghost planes] in lattice
        // order, per real brick in ascending order, each stretch of one
        // lattice line that the brick's region holds -- consecutive region
        // entries ([entry][3] at wsoff) -- as (first sum, 64-bit row mask)
        const int64_t Lx = A->row_lat[0], Ly = A->row_lat[1], Lz = A->row_lat[2];
        const int64_t p3 = 3 * Lx * Ly;
        const int64_t zo = A->ghost_lo / p3, hp = A->ghost_hi / p3;
        const int64_t ntot = n + hp * Lx * Ly, ns = (ntot + 63) / 64;
        std::vector<std::vector<std::pair<int64_t, unsigned long long>>> sr(ns);
        for (int q = 0; q < NB; ++q) {
            const BrickDesc &D = bp->bricks[q];
            for (int rz = 0; rz < D.RZ; ++rz)
                for (int ry = 0; ry < D.RY; ++ry) {
                    const int64_t gy = D.oy + ry, gz = D.oz + rz;
                    if (gy < 0 || gy >= Ly || gz + zo < 0 || gz >= Lz + hp) continue;
                    const int64_t x0 = std::max<int64_t>(D.ox, 0), x1 = std::min<int64_t>(D.ox + D.RX, Lx);
                    if (x1 <= x0) continue;
                    const int64_t j0 = x0 + Lx * (gy + Ly * gz), j1 = j0 + (x1 - x0);
                    const int64_t k0 = (x0 - D.ox) + (int64_t)D.RX * (ry + (int64_t)D.RY * rz);
                    for (int64_t a = j0; a < j1;) {
                        const int64_t sl = a >> 6, b2 = std::min(j1, (sl + 1) * 64);
                        unsigned long long m = 0;
                        for (int64_t jj = a; jj < b2; ++jj) m |= 1ull << (jj & 63);
                        sr[sl].push_back({D.wsoff + 3 * (k0 + (a - j0)), m});
                        a = b2;
                    }
                }
        }
        std::vector<int> runptr(ns + 1, 0), rstart;
        std::vector<unsigned long long> rmask;
        for (int64_t sl = 0; sl < ns; ++sl) {
            runptr[sl + 1] = runptr[sl] + (int)sr[sl].size();
            for (auto &r : sr[sl]) {
                if (r.first > INT_MAX) return fail(KLE_ERR_SUP, "brick sums beyond 2^31 doubles");
                rstart.push_back((int)r.first);
                rmask.push_back(r.second);
            }
        }
        if (rstart.empty()) {
            rstart.push_back(0);
            rmask.push_back(0);
        }
        if (hipMalloc(&A->d_sgptr, sizeof(int) * (ns + 1)) != hipSuccess ||
            hipMalloc(&A->d_sgidx, sizeof(int) * rstart.size()) != hipSuccess ||
            hipMalloc(&A->d_sgmask, sizeof(unsigned long long) * rmask.size()) != hipSuccess) {
            (void)hipGetLastError();
            if (dmu) (void)hipFree(dmu);
            return fail(KLE_ERR_MEM, "out of device memory for the brick gather runs");
        }
        KLE_TRY(h2d(A->d_sgptr, runptr.data(), sizeof(int) * (ns + 1)));
        KLE_TRY(h2d(A->d_sgidx, rstart.data(), sizeof(int) * rstart.size()));
        KLE_TRY(h2d(A->d_sgmask, rmask.data(), sizeof(unsigned long long) * rmask.size()));
        A->brick_gparts = (int)(runptr[ns] / std::max<int64_t>(ns, 1));  // (runs per 64 rows, for the log)
        A->gather_rps = (int)((runptr[ns] + ns - 1) / std::max<int64_t>(ns, 1));
    }
    if (!bp->srows.empty()) {
        // the one-block rows per 64-row slice of the owned rows (the gather
        // forms their B_ii x_i)
        const int64_t nso = (n + 63) / 64;
        std::vector<unsigned long long> sm(nso, 0ull);
        for (int64_t i : bp->srows) sm[i >> 6] |= 1ull << (i & 63);
        if (hipMalloc(&A->d_ssingle, sizeof(unsigned long long) * nso) != hipSuccess) {
            (void)hipGetLastError();
            A->d_ssingle = nullptr;
            if (dmu) (void)hipFree(dmu);
            return fail(KLE_ERR_MEM, "out of device memory for the brick gather's one-block rows");
        }
        KLE_TRY(h2d(A->d_ssingle, sm.data(), sizeof(unsigned long long) * nso));
    }
    KLE_TRY(h2d(dmu, hmu.data(), sizeof(int) * 2 * n));
    const int64_t plane3 = 3 * A->row_lat[0] * A->row_lat[1];
    const int zo = (int)(A->ghost_lo / plane3), hp = (int)(A->ghost_hi / plane3);
    if (NB > 0)  // (every row of one block: no brick at all, the gather forms y)
        hipLaunchKernelGGL(k_brick_bound, dim3((unsigned)NB), dim3(256), 0, c->stream, (int)A->row_lat[0],
                           (int)A->row_lat[1], (int)A->row_lat[2], zo, hp,
                           reinterpret_cast<const BrickDesc *>(A->d_bdesc), A->d_rowbox, dmu, A->d_svptr, A->d_sval,
                           A->sym_P, dmu + n, A->d_stile_e);
    KLE_HIP(hipGetLastError());
    // the exponents into the descriptors
    std::vector<int> eb(NB);
    KLE_HIP(hipStreamSynchronize(c->stream));
    KLE_HIP(hipMemcpy(eb.data(), A->d_stile_e, sizeof(int) * NB, hipMemcpyDeviceToHost));
    (void)hipFree(dmu);
    for (int q = 0; q < NB; ++q) bp->bricks[q].eb = eb[q];
    KLE_TRY(h2d(A->d_bdesc, bp->bricks.data(), sizeof(BrickDesc) * NB));
    A->nbricks = NB;
    {
        // (bricks along each axis: distinct first coordinates)
        std::vector<int> u[3];
        for (const BrickDesc &D : bp->bricks) {
            u[0].push_back(D.x0);
            u[1].push_back(D.y0);
            u[2].push_back(D.z0);
        }
        for (int k = 0; k < 3; ++k) {
            std::sort(u[k].begin(), u[k].end());
            A->brick_dims[k] = (int)(std::unique(u[k].begin(), u[k].end()) - u[k].begin());
        }
    }
    A->brick_model_us = bp->model_us;
    A->brick_lds = (int)bp->lds;
    A->sws_entries = bp->ws_entries;
    A->sym_brick = 1;
    if (const char *e = getenv("KLE_TIMING"))
        if (atoi(e) && NB > 0) {
            const BrickDesc &D = bp->bricks[0];
            fprintf(stderr, "[kle brick] %d bricks (first %d x %d x %d rows, region %d x %d x %d), LDS %zu B, "
                            "region entries %lld (%.2f per row)\n",
                    NB, D.nx, D.ny, D.nz, D.RX, D.RY, D.RZ, bp->lds, (long long)bp->ws_entries,
                    (double)bp->ws_entries / n);
        }
    return 0;
}

void brick_plan_free(void *plan) { delete reinterpret_cast<BrickPlan *>(plan); }

void brick_drop(kle_mat *A)
{
    for (void *q : {A->d_bdesc, (void *)A->d_browd})
        if (q) (void)hipFree(q);
    brick_forget(A);
}

void brick_forget(kle_mat *A)
{
    A->d_bdesc = nullptr;
    A->d_browd = nullptr;
    A->nbricks = 0;
    A->brick_gparts = 0;
    A->brick_dims[0] = A->brick_dims[1] = A->brick_dims[2] = 0;
    A->brick_model_us = 0.0;
    A->brick_lds = 0;
    A->sym_brick = 0;
    A->sym_gbrick = 0;
    A->brick_lds_u = 0;
}

int brick_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, double *dpart, bool split)
{
    kle_ctx *c = A->ctx;
    const int64_t plane3 = 3 * A->row_lat[0] * A->row_lat[1];
    const int zo = (int)(A->ghost_lo / plane3), hp = (int)(A->ghost_hi / plane3);
    const BrickDesc *bd = reinterpret_cast<const BrickDesc *>(A->d_bdesc);
    auto go = [&](auto kern, int slot, int wv) {
        (void)slot;
        dyn_lds(c, reinterpret_cast<const void *>(kern), (size_t)A->brick_lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)A->nbricks), dim3(64 * wv), (size_t)A->brick_lds, c->stream,
                           (int)A->row_lat[0], (int)A->row_lat[1], (int)A->row_lat[2], zo, hp, A->brick_rstride, bd,
                           reinterpret_cast<const int2 *>(A->d_browd), A->d_sval, x->base, A->d_sws, y->d,
                           dpart, istate KLE_PROBE_ARG);
    };
    const bool dist = c->nranks > 1 && (A->lo_rank >= 0 || A->hi_rank >= 0);
    // N > 1 (z slabs): the x ghost planes first (every brick's region fill
    // may read them); after the bricks, the upper ghost nodes' sums go to the
    // upper neighbour (MPISBAIJ's reverse scatter) on the comm stream while
    // the owned rows are summed; the lower neighbour's sums for the lowest
    // rows are added last (fixed order: y stays bitwise reproducible).  All
    // RCCL calls in the same order on every rank: forward, then reverse halo.
    if (dist)
        KLE_TRY(halo_exchange(c, x->base, x->ghost_lo, x->n_local, x->ghost_hi, x->lo_rank, x->hi_rank, x->send_lo,
                              x->send_hi, c->stream, nullptr));
    if (A->nbricks == 0) {
        // (no brick: every row of one block, formed by the gather)
    } else {
        // (a split product's (A x, x): the bricks' shares, DOT; else the gather's)
        if (split && dpart && !dist) go(k_nb_spmv_sym_brick<BRICK_WV, true, true>, 0, BRICK_WV);
        else go(k_nb_spmv_sym_brick<BRICK_WV, true, false>, 0, BRICK_WV);
    }
    KLE_HIP(hipGetLastError());
    // the gather (kle_sym.hip gsym_gather): per row its direct sum in y, then
    // the runs of the regions holding it, in ascending brick order
    const int64_t n = A->nrows, ntot = n + A->ghost_hi / 3, nlo = n / 64 * 64;
    const double *xs = A->d_ssingle ? x->d : nullptr;  // (rows of one stored block: the gather's)
    if (!dist) {
        if (split) return 0;  // (the consumer gathers every row: BrickGather)
        return gsym_gather(A, y->d, 0, n, istate, dpart ? x->d : nullptr, dpart, 1, c->stream, xs);
    }
    // the slices holding upper ghost rows first (their sums: d_sgsend)
    KLE_TRY(gsym_gather(A, y->d, nlo, ntot, istate, nullptr, nullptr, 1, c->stream, xs));
    const int64_t nrecv = A->lo_rank >= 0 ? A->send_lo : 0;
    const bool ovl = A->halo_overlap != 0;
    hipStream_t cs = ovl ? c->comm_stream : c->stream;
    if (ovl) {
        KLE_HIP(hipEventRecord(c->ev_x_ready, c->stream));
        KLE_HIP(hipStreamWaitEvent(cs, c->ev_x_ready, 0));
    }
    KLE_TRY(halo_reverse(c, A->d_sgsend, A->ghost_hi, A->hi_rank, A->d_sgrecv, nrecv, A->lo_rank, cs));
    if (ovl) KLE_HIP(hipEventRecord(c->ev_halo_done, cs));
    if (split) return 0;  // (the owned rows below nlo and the received sums: the consumer's)
    return brick_gather_rest(A, x, y, istate);
}

// The rank-local part of a box-brick product, for timing it
// (kle_mat_time_local_spmv): the bricks and the gather of every row they
// touch, owned and upper ghost, with no halo either way -- the ghost x as
// they are, the upper ghost rows' sums left in the send buffer.  A slab
// part's kernel time without its neighbours (ranks sharing one GPU take
// turns); on one rank the product itself.
int brick_spmv_local(kle_mat *A, const kle_vec *x, kle_vec *y)
{
    kle_ctx *c = A->ctx;
    const int64_t plane3 = 3 * A->row_lat[0] * A->row_lat[1];
    const int zo = (int)(A->ghost_lo / plane3), hp = (int)(A->ghost_hi / plane3);
    if (A->nbricks > 0) {
        auto kern = k_nb_spmv_sym_brick<BRICK_WV, true, false>;
        dyn_lds(c, reinterpret_cast<const void *>(kern), (size_t)A->brick_lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)A->nbricks), dim3(64 * BRICK_WV), (size_t)A->brick_lds, c->stream,
                           (int)A->row_lat[0], (int)A->row_lat[1], (int)A->row_lat[2], zo, hp, A->brick_rstride,
                           reinterpret_cast<const BrickDesc *>(A->d_bdesc),
                           reinterpret_cast<const int2 *>(A->d_browd), A->d_sval, x->base, A->d_sws, y->d,
                           nullptr, nullptr KLE_PROBE_ARG);
        KLE_HIP(hipGetLastError());
    }
    const int64_t ntot = A->nrows + A->ghost_hi / 3;
    return gsym_gather(A, y->d, 0, ntot, nullptr, nullptr, nullptr, 1, c->stream, A->d_ssingle ? x->d : nullptr);
}

// The rest of a split product (brick_spmv with split): the rows [0, nlo)
// (every row on one rank) gathered, then the received reverse-halo sums added
// last -- the same operations, in the same order, as the unsplit product
// (wps_force 1: each row's runs summed in k_pipe_iter_g's order).
int brick_gather_rest(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate, int wps_force)
{
    kle_ctx *c = A->ctx;
    const bool dist = c->nranks > 1 && (A->lo_rank >= 0 || A->hi_rank >= 0);
    const int64_t n = A->nrows, nlo = dist ? n / 64 * 64 : n;
    const double *xs = A->d_ssingle ? x->d : nullptr;
    KLE_TRY(gsym_gather(A, y->d, 0, nlo, istate, nullptr, nullptr, 1, c->stream, xs, wps_force));
    if (!dist) return 0;
    const int64_t nrecv = A->lo_rank >= 0 ? A->send_lo : 0;
    if (A->halo_overlap) KLE_HIP(hipStreamWaitEvent(c->stream, c->ev_halo_done, 0));
    if (nrecv)
        hipLaunchKernelGGL(k_brick_add_recv, dim3((unsigned)((nrecv + 255) / 256)), dim3(256), 0, c->stream, nrecv,
                           A->d_sgrecv, y->d, istate);
    KLE_HIP(hipGetLastError());
    return 0;
}

// What a consumer of a split product gathers itself (k_pipe_iter_g,
// kle_ksp.hip): the run lists of the rows [0, ng), the one-block rows, and
// the received sums of the lowest rows (after the reverse halo, which the
// consumer's stream must have waited for: see brick_split_wait)
BrickGather brick_gather_src(const kle_mat *A, const kle_vec *x)
{
    const kle_ctx *c = A->ctx;
    const bool dist = c->nranks > 1 && (A->lo_rank >= 0 || A->hi_rank >= 0);
    BrickGather g;
    g.runptr = A->d_sgptr;
    g.rstart = A->d_sgidx;
    g.rmask = A->d_sgmask;
    g.ws = A->d_sws;
    g.single = A->d_ssingle;
    g.sval = A->d_sval;
    g.svptr = A->d_svptr;
    g.xs = x->d;
    g.nrows = A->nrows;
    g.ng = dist ? A->nrows / 64 * 64 : A->nrows;
    g.recv = A->d_sgrecv;
    g.nrecv = dist && A->lo_rank >= 0 ? A->send_lo : 0;
    return g;
}

}  // namespace kle
