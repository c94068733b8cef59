// kle_gbrick.hip -- the unstructured symmetric SpMV on row bricks (round 5).
//
// Config 5's K (graph-numbered, Hilbert-ordered node rows, columns streamed;
// MatFS.buildFS, mat_fs.py:150-192; the product is the MatMult inside
// KSPSolve, kle_solver.py:35) in symmetric storage: block (i, j), j >= i,
// serves row i (B x_j) and row j (B^T x_i).  Round 3's kernel (kle_sym.hip
// k_nb_spmv_gsym) takes 64-row groups and writes each group's dictionary
// partials to HBM in the middle of the value stream (7.9 entries per row at
// 1M DoF).  Here, as for the box (kle_brick.hip), the rows are cut into one
// contiguous range per CU -- a "brick" of ~n / 256 Hilbert-ordered rows,
// spatially compact -- whose dictionary (its rows, then the upper-triangle
// columns past them; ~2 entries per row) holds x and the exact int64
// fixed-point transposed sums in LDS from the first value load to the last.
// A 16-wave workgroup streams the brick: rows from an LDS counter, items =
// (row, 64-block pass), nine nontemporal value loads and the blocks' 2-byte
// dictionary positions in flight one item ahead of the summed one.  B x_j
// goes to the row's fp64 register sum, written to y when the row ends; B^T
// x_i to the entry's fixed-point slot.  At the end the brick writes its
// dictionary sums once ([entry][3], the round-3 partial layout), and
// k_nb_gsym_gather (kle_sym.hip, preload) adds them to y in ascending brick
// order -- bitwise reproducible, the fixed-point sums being order-free.
// Host side: the ranges and dictionaries are planned in kle_sym.hip
// gsym_build (the round-3 group machinery with variable row ranges).
#include <algorithm>
#include <cmath>

#include "kle_brick.hpp"
#include "kle_internal.hpp"
#include "kle_sym_dev.hpp"

namespace kle {

using cint = __attribute__((address_space(4))) const int;

// one more load than sym_ld9's nine in flight per item: the blocks' 2-byte
// dictionary positions (nontemporal, whole lines per 64 lanes)
__device__ __forceinline__ void gb_ldpos(int &p, const uint16_t *base, unsigned o)
{
    asm volatile("global_load_ushort %0, %1, %2 nt" : "=&v"(p) : "v"(o), "s"(base) : "memory");
}

template <int N>
__device__ __forceinline__ void gb_wait10(double *v, int &p)
{
    asm volatile("s_waitcnt vmcnt(%10)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8]), "+v"(p)
                 : "i"(N));
}

// an issued item: the row (r < 0: a re-read past the brick's last row), its
// stored blocks, the pass's first block
struct GItem {
    int r, mu, kb;
};

template <int WV, int D>
__global__ __launch_bounds__(64 * WV, 1) void k_nb_spmv_gsym_brick(const GBrickDesc *__restrict__ bd,
                                                                  const int4 *__restrict__ rowd,
                                                                  const uint16_t *__restrict__ slid,
                                                                  const int *__restrict__ dict,
                                                                  const double *__restrict__ sval,
                                                                  const double *__restrict__ x,
                                                                  double *__restrict__ ws, double *__restrict__ y,
                                                                  const int *__restrict__ istate)
{
    constexpr int NT = 64 * WV;
    static_assert(D == 1 || D == 2, "one or two items ahead");
    extern __shared__ double lds[];
    const int stop = istate ? istate[I_REASON] : 0;  // (tested before the first store)
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r0 = bd[b].r0, NR = bd[b].nr, U = bd[b].U, eb = bd[b].eb;
    const long long d0 = bd[b].d0, vbase = bd[b].vbase, sbase = bd[b].sbase, wsoff = bd[b].wsoff;
    const int RS = U + 64;
    double *xl = lds;
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(lds + 3 * U);
    double *wred = lds + 3 * U + 3 * RS;
    int *ctr = reinterpret_cast<int *>(wred + 2 * WV);
    cint *rdesc = (cint *)(rowd + r0);  // (address-space cast: scalar loads)
    const double *vb = sval + vbase;
    const uint16_t *sb = slid + sbase;
    // the row's values and positions from its descriptor (value offset / 16,
    // position offset, stored blocks)
    struct GRow {
        const double *v;
        const uint16_t *s;
        int mu, r;
    };
    auto row_setup = [&](int r, GRow &R) {
        R.v = vb + (int64_t)rdesc[4 * r] * 16;
        R.s = sb + rdesc[4 * r + 1];
        R.mu = rdesc[4 * r + 2];
        R.r = rdesc[4 * r + 3];  // (the row's dictionary entry: the brick's rows lead it)
    };
    // the values of one 64-block pass (lanes past the row's end re-read its
    // last block; their results go nowhere) and the blocks' positions
    auto load_v = [&](const GRow &R, int kb, double *vv, int &pos) {
        const int kk = min(kb + lane, R.mu - 1);
        const int q16 = R.mu & ~15;
        const bool ch = kk < q16;
        const int o0 = ch ? (kk >> 4) * 144 + (kk & 15) : q16 * 9 + (kk - q16);
        const int st = ch ? 16 : R.mu - q16;
        unsigned o[9];
#pragma unroll
        for (int s = 0; s < 9; ++s) o[s] = (unsigned)(o0 + s * st) * 8u;
        sym_ld9(vv, R.v, o);
        gb_ldpos(pos, R.s, (unsigned)kk * 2u);
    };
    auto grab = [&]() -> int {
        int r = 0;
        if (lane == 0) r = atomicAdd(ctr, 1);
        return __builtin_amdgcn_readfirstlane(r);
    };
    // 1. the wave's first rows are static (w, w + WV, w + 2 WV: the counter
    // starts past them), so its first item goes out before the fill
    int snext = w + WV;
    auto take = [&]() -> int {
        if (snext < 3 * WV) {
            const int r = snext;
            snext += WV;
            return r;
        }
        return grab();
    };
    GRow I;
    int ki = 0;
    bool idone = w >= NR;
    double v0[9], v1[9], v2[9];
    int p0 = 0, p1 = 0, p2 = 0;
    GItem i0, i1, i2;
    if (!idone) {
        row_setup(w, I);
    } else {
        I.v = vb;
        I.s = sb;
        I.mu = 1;
        I.r = -1;
    }
    load_v(I, 0, v0, p0);
    i0 = {idone ? -1 : I.r, I.mu, 0};
    int pend = take();
    auto issue = [&](double *vn, int &pn, GItem &itn) {
        if (!idone) {
            if (ki + 64 < I.mu) {
                ki += 64;
            } else if (pend >= NR) {
                idone = true;
            } else {
                row_setup(pend, I);
                ki = 0;
                pend = take();
            }
        }
        load_v(I, ki, vn, pn);
        itn = {idone ? -1 : I.r, I.mu, ki};
    };
    if (D == 2) issue(v1, p1, i1);
    // 2. x of the dictionary into LDS (entry ids, then the x loads, FB per
    // thread in flight), its max |x|; the sums zeroed
    double xm = 0.0;
    int bad = 0;
    {
        constexpr int FB = 8;
        const int n3 = 3 * U;
        for (int t0 = 0; t0 < n3; t0 += FB * NT) {
            int id[FB];
#pragma unroll
            for (int f = 0; f < FB; ++f) {
                const int t = min(t0 + f * NT + (int)threadIdx.x, n3 - 1);
                id[f] = dict[d0 + t / 3];
            }
            double fv[FB];
#pragma unroll
            for (int f = 0; f < FB; ++f) {
                const int t = min(t0 + f * NT + (int)threadIdx.x, n3 - 1);
                fv[f] = x[(int64_t)id[f] * 3 + (t - 3 * (t / 3))];
            }
#pragma unroll
            for (int f = 0; f < FB; ++f) {
                const int t = t0 + f * NT + (int)threadIdx.x;
                const bool on = t < n3;
                const int e = t / 3, c = t - 3 * e;
                xl[on ? c * U + e : 3 * U + 3 * RS - 64 + lane] = fv[f];  // (else a dummy slot of the sums)
                const double a = on ? fabs(fv[f]) : 0.0;
                bad |= !(a <= 1.7976931348623157e308);
                xm = fmax(xm, a);
            }
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
    if (threadIdx.x == 0) *ctr = 3 * WV;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // LDS stores done (lgkmcnt 0); the value loads stay in flight
    __builtin_amdgcn_s_barrier();
    if (__builtin_amdgcn_readfirstlane(stop) != 0) {
        sym_wait9<0>(v0);
        sym_wait9<0>(v1);
        return;  // (nothing written yet)
    }
    // the brick's scale: 2^(61 - E), 2^E > (its sums' bound, k_gbrick_bound)
    // x max |x|, as two normal factors (x near the bottom of the exponent
    // range keeps its 61 bits)
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
    // 3. the items, D in flight ahead of the summed one
    if (i0.r >= 0) {
        double cx0 = 0.0, cx1 = 0.0, cx2 = 0.0;
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
        auto step = [&](double *vv, int &pp, const GItem &it, double *vn, int &pn, GItem &itn) {
            issue(vn, pn, itn);
            if (it.r < 0) return false;
            if (it.kb == 0) {  // a new row: its x (the rows lead the dictionary)
                cx0 = uni_d(xl[it.r]);
                cx1 = uni_d(xl[U + it.r]);
                cx2 = uni_d(xl[2 * U + it.r]);
            }
            gb_wait10<10 * D>(vv, pp);
            const int rr = pp;
            const double xj0 = xl[rr], xj1 = xl[U + rr], xj2 = xl[2 * U + rr];
            const int kk = it.kb + lane;
            const bool live = kk < it.mu;
            const int rt = live && kk > 0 ? rr : U + lane;
            const double s0 = vv[0] * xj0 + vv[1] * xj1 + vv[2] * xj2;
            const double s1 = vv[3] * xj0 + vv[4] * xj1 + vv[5] * xj2;
            const double s2 = vv[6] * xj0 + vv[7] * xj1 + vv[8] * xj2;
            acc0 += live ? s0 : 0.0;
            acc1 += live ? s1 : 0.0;
            acc2 += live ? s2 : 0.0;
            const double t0 = vv[0] * cx0 + vv[3] * cx1 + vv[6] * cx2;
            const double t1 = vv[1] * cx0 + vv[4] * cx1 + vv[7] * cx2;
            const double t2 = vv[2] * cx0 + vv[5] * cx1 + vv[8] * cx2;
            atomicAdd(&acc[rt], fx_of(t0 * S1, S2));
            atomicAdd(&acc[RS + rt], fx_of(t1 * S1, S2));
            atomicAdd(&acc[2 * RS + rt], fx_of(t2 * S1, S2));
            if (it.kb + 64 >= it.mu) {
                // the row is done: its direct sum (fixed-order DPP, fp64), one
                // writer, into y; the gather adds the bricks' transposed sums
                wsum3_dpp(acc0, acc1, acc2);
                const int64_t j = (int64_t)r0 + it.r;
                if (lane < 3) y[3 * j + lane] = lane == 0 ? acc0 : lane == 1 ? acc1 : acc2;
                acc0 = acc1 = acc2 = 0.0;
            }
            return true;
        };
        if constexpr (D == 1) {
            while (step(v0, p0, i0, v1, p1, i1) && step(v1, p1, i1, v0, p0, i0)) {
            }
        } else {
            while (step(v0, p0, i0, v2, p2, i2) && step(v1, p1, i1, v0, p0, i0) &&
                   step(v2, p2, i2, v1, p1, i1)) {
            }
        }
    }
    // the last (re-read) loads land before their registers are reused
    gb_wait10<0>(v0, p0);
    gb_wait10<0>(v1, p1);
    if (D == 2) gb_wait10<0>(v2, p2);
    __syncthreads();
    // 4. the dictionary's transposed sums, once: [entry][3]
    double *dst = ws + wsoff;
    for (int t = threadIdx.x; t < 3 * U; t += NT) {
        const int e = t / 3, c = t - 3 * e;
        dst[t] = fx_to_d(acc[c * RS + e]) * T1 * T2;
    }
}

// Per brick: eb with 2^eb > the largest, over its dictionary entries e, of
// the sum over its rows' blocks that add to e (the diagonal blocks excepted)
// of max_b sum_a |B[a][b]|.  The sums are exact int64 fixed-point adds of
// each term rounded up (scale 2^sh, every term < 2^50), so the bound is
// order-free: the same eb on every build.
__global__ __launch_bounds__(256) void k_gbrick_bound(const GBrickDesc *__restrict__ bd, const int4 *__restrict__ rowd,
                                                      const uint16_t *__restrict__ slid,
                                                      const double *__restrict__ sval, int sh,
                                                      int *__restrict__ ebo)
{
    extern __shared__ unsigned long long bsum[];
    __shared__ unsigned long long wmax[4];
    const GBrickDesc B = bd[blockIdx.x];
    for (int e = threadIdx.x; e < B.U; e += 256) bsum[e] = 0ull;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int r = w; r < B.nr; r += 4) {
        const int4 d = rowd[B.r0 + r];
        const double *v = sval + B.vbase + (int64_t)d.x * 16;
        const uint16_t *s = slid + B.sbase + d.y;
        const int mu = d.z;
        for (int kk = lane; kk < mu; kk += 64) {
            if (kk == 0) continue;  // (the row's own diagonal block: its direct sum)
            double bmax = 0.0;
#pragma unroll
            for (int bb = 0; bb < 3; ++bb) {
                double cs = 0.0;
#pragma unroll
                for (int a = 0; a < 3; ++a) cs += fabs(v[vofs(1, 9, a * 3 + bb, kk, mu, mu)]);
                bmax = fmax(bmax, cs);
            }
            const double f = ceil(ldexp(bmax, sh));
            atomicAdd(&bsum[s[kk]], (unsigned long long)f);
        }
    }
    __syncthreads();
    unsigned long long m = 0ull;
    for (int e = threadIdx.x; e < B.U; e += 256) m = max(m, bsum[e]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor((long long)m, o, 64));
    if (lane == 0) wmax[w] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        int e = -1000;  // (no transposed adds in this brick)
        // (the int64 -> double conversion may round down: one ulp up)
        if (m) (void)frexp(ldexp((double)m * (1.0 + 0x1p-50), -sh), &e);
        ebo[blockIdx.x] = e;
    }
}

// ---------------------------------------------------------------------------
// host side (the plan itself: kle_sym.hip gsym_build)

int gbrick_bound(kle_mat *A, double vmax_all)
{
    kle_ctx *c = A->ctx;
    const int NB = A->nbricks;
    // every term max_b sum_a |B[a][b]| <= 3 vmax_all < 2^(ev): scale 2^(50 - ev)
    int ev = 0;
    (void)frexp(3.0 * std::max(vmax_all, 1e-300), &ev);
    const int sh = 50 - ev;
    const int umax = A->brick_lds_u;
    const size_t lds = sizeof(unsigned long long) * (size_t)std::max(umax, 1);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_gbrick_bound),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_gbrick_bound, dim3((unsigned)NB), dim3(256), lds, c->stream,
                       reinterpret_cast<const GBrickDesc *>(A->d_bdesc), reinterpret_cast<const int4 *>(A->d_browd),
                       A->d_slid, A->d_sval, sh, A->d_stile_e);
    KLE_HIP(hipGetLastError());
    std::vector<int> eb(NB);
    KLE_HIP(hipStreamSynchronize(c->stream));
    KLE_HIP(hipMemcpy(eb.data(), A->d_stile_e, sizeof(int) * NB, hipMemcpyDeviceToHost));
    std::vector<GBrickDesc> hb(NB);
    KLE_HIP(hipMemcpy(hb.data(), A->d_bdesc, sizeof(GBrickDesc) * NB, hipMemcpyDeviceToHost));
    for (int q = 0; q < NB; ++q) hb[q].eb = eb[q];
    KLE_TRY(h2d(A->d_bdesc, hb.data(), sizeof(GBrickDesc) * NB));
    return 0;
}

int gbrick_launch(kle_mat *A, const kle_vec *x, kle_vec *y, const int *istate)
{
    kle_ctx *c = A->ctx;
    auto kern = k_nb_spmv_gsym_brick<BRICK_WV, 1>;
    dyn_lds(c, reinterpret_cast<const void *>(kern), (size_t)A->brick_lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)A->nbricks), dim3(64 * BRICK_WV),
                       (size_t)A->brick_lds, c->stream, reinterpret_cast<const GBrickDesc *>(A->d_bdesc),
                       reinterpret_cast<const int4 *>(A->d_browd), A->d_slid, A->d_sdict, A->d_sval, x->base, A->d_sws,
                       y->d, istate);
    KLE_HIP(hipGetLastError());
    return 0;
}

}  // namespace kle
