// Prototype (tool, not product), second layout: symmetric position-class
// storage with UNIFORM class sub-lattices.
//
// Every class c = (ix mod p, iy mod p, iz mod p) gets the same sub-lattice
// (tx, ty, tz) in [0,nel)^3 (node ix = px + p*tx), so a block offset d maps
// class-c row r to class-c' row r + shift(d) with one constant linear shift:
// for a wave of 64 consecutive class rows every stream load (values, the
// partner's transposed values, x) is 64 consecutive doubles.  A (class, d)
// stream covers the whole sub-lattice, zero where the block does not exist
// (boundary clipping, Dirichlet rows; their diagonal block is I).  Rows on
// the ix = L-1 (iy, iz) planes are Dirichlet and not part of the class
// lattice (identity rows, handled outside this kernel).
//   hipcc --offload-arch=gfx950 -O3 -o sym_proto2 sym_proto2.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("%s: %s\n", #x, hipGetErrorString(e));                          \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

struct Term {
    long long vofs;  // first double of the 9 streams + partner shift (transposed terms)
    int xofs;        // x index of the target for class row r: xofs + r
    int fx, fy, fz;  // sub-lattice shift of the target (mask for transposed terms)
    int tr;          // read the block transposed (partner's stored stream)
    int pad[2];
};

template <bool NT, int SPLIT, int B>
__global__ __launch_bounds__(256) void k_sym(int nwaves, int CS, int NX, int NY, int NZ, const int *__restrict__ wcls,
                                             const int *__restrict__ ct0, const Term *__restrict__ terms,
                                             const double *__restrict__ val, const double *__restrict__ x,
                                             double *__restrict__ y, long long nP)
{
    constexpr int GROUPS = 4 / SPLIT;
    __shared__ double part[SPLIT > 1 ? 4 : 1][3][64];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = wv % SPLIT, g = wv / SPLIT;
    const int w = blockIdx.x * GROUPS + g;
    const int lane = threadIdx.x & 63;
    const bool live = w < nwaves;
    const int wc = wcls[live ? w : 0];  // class | (row0 / 64) << 8
    const int c = wc & 255, r = ((wc >> 8) << 6) + lane;
    const int tx = r % NX, qq = r / NX, ty = qq % NY, tz = qq / NY;
    double a0 = 0, a1 = 0, a2 = 0;
    const int t0 = ct0[c], t1 = live ? ct0[c + 1] : t0;
    const long long CSL = CS;
    for (int k0 = t0 + q; k0 < t1; k0 += SPLIT * B) {
        double bv[B][9], xv[B][3];
        bool okv[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int k = k0 + u * SPLIT;
            const bool tv = k < t1;
            const Term &T = terms[tv ? k : t0];
            const bool ok = tv & ((unsigned)(tx + T.fx) < (unsigned)NX) & ((unsigned)(ty + T.fy) < (unsigned)NY) &
                            ((unsigned)(tz + T.fz) < (unsigned)NZ);
            okv[u] = ok;
            const double *v = val + T.vofs + r;
            const long long s1 = T.tr ? 3 * CSL : CSL, s3 = T.tr ? CSL : 3 * CSL;
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    const double *pp = v + a * s3 + cc * s1;
                    bv[u][3 * a + cc] = NT ? __builtin_nontemporal_load(pp) : *pp;
                }
            const long long xi = T.xofs + r;
            xv[u][0] = x[xi];
            xv[u][1] = x[xi + nP];
            xv[u][2] = x[xi + 2 * nP];
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const double m = okv[u] ? 1.0 : 0.0;
            const double x0 = m * xv[u][0], x1 = m * xv[u][1], x2 = m * xv[u][2];
            a0 += bv[u][0] * x0 + bv[u][1] * x1 + bv[u][2] * x2;
            a1 += bv[u][3] * x0 + bv[u][4] * x1 + bv[u][5] * x2;
            a2 += bv[u][6] * x0 + bv[u][7] * x1 + bv[u][8] * x2;
        }
    }
    if constexpr (SPLIT > 1) {
        part[wv][0][lane] = a0;
        part[wv][1][lane] = a1;
        part[wv][2][lane] = a2;
        __syncthreads();
        if (q != 0) return;
#pragma unroll
        for (int j = 1; j < SPLIT; ++j) {
            a0 += part[wv + j][0][lane];
            a1 += part[wv + j][1][lane];
            a2 += part[wv + j][2][lane];
        }
    }
    if (live) {
        const long long o = (long long)c * CS + r;
        y[o] = a0;
        y[nP + o] = a1;
        y[2 * nP + o] = a2;
    }
}

static int fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

int main(int argc, char **argv)
{
    int nel[3] = {20, 16, 16}, p = 4, full = 0, check = 0, nt = 1, order = 1, reps = 200, split = 4, bat = 4;
    if (argc > 3) for (int k = 0; k < 3; ++k) nel[k] = atoi(argv[1 + k]);
    if (argc > 4) p = atoi(argv[4]);
    if (argc > 5) full = atoi(argv[5]);
    if (argc > 6) check = atoi(argv[6]);
    if (argc > 7) nt = atoi(argv[7]);
    if (argc > 8) order = atoi(argv[8]);
    if (argc > 9) reps = atoi(argv[9]);
    if (argc > 10) split = atoi(argv[10]);
    if (argc > 11) bat = atoi(argv[11]);
    const int NX = nel[0], NY = nel[1], NZ = nel[2];
    const long long L[3] = {(long long)NX * p + 1, (long long)NY * p + 1, (long long)NZ * p + 1};
    const int CS0 = NX * NY * NZ, CS = (CS0 + 63) & ~63;
    const int ncls = p * p * p;
    const long long G = (long long)NX * NY + NX + 1;  // guard so shifted x reads stay inside the allocation
    const long long nP = G + (long long)ncls * CS + G;  // per component: guard | classes | guard
    auto free_node = [&](const long long *ix) {
        for (int k = 0; k < 3; ++k)
            if (ix[k] < 1 || ix[k] > L[k] - 2) return false;
        return true;
    };
    auto omin = [&](int pc) { return pc == 0 ? -p : -pc; };
    auto omax = [&](int pc) { return pc == 0 ? p : p - pc; };
    auto idoff = [&](int dx, int dy, int dz) { return dx + L[0] * (dy + L[1] * dz); };
    // stored streams (class, d >= 0)
    std::map<std::pair<int, long long>, long long> seg;
    long long nval = 0;
    std::vector<Term> terms;
    std::vector<int> ct0(ncls + 1);
    struct Cand { long long off; int d[3]; };
    std::vector<std::vector<Cand>> cands(ncls);
    for (int c = 0; c < ncls; ++c) {
        const int pc[3] = {c % p, (c / p) % p, c / (p * p)};
        for (int dz = omin(pc[2]); dz <= omax(pc[2]); ++dz)
            for (int dy = omin(pc[1]); dy <= omax(pc[1]); ++dy)
                for (int dx = omin(pc[0]); dx <= omax(pc[0]); ++dx) cands[c].push_back({idoff(dx, dy, dz), {dx, dy, dz}});
        if (order) std::sort(cands[c].begin(), cands[c].end(), [](const Cand &a, const Cand &b) {
            long long aa = std::llabs(a.off), bb = std::llabs(b.off);
            return aa != bb ? aa < bb : a.off > b.off;
        });
        for (const Cand &cd : cands[c])
            if (cd.off >= 0 || full) {
                seg[{c, cd.off}] = nval;
                nval += 9LL * CS;
            }
    }
    auto cls_shift = [&](const int *pc, const int *d, int *pt, int *f) {
        for (int k = 0; k < 3; ++k) {
            f[k] = fdiv(pc[k] + d[k], p);
            pt[k] = pc[k] + d[k] - f[k] * p;
        }
    };
    long long nstored = 0;
    for (int c = 0; c < ncls; ++c) {
        const int pc[3] = {c % p, (c / p) % p, c / (p * p)};
        ct0[c] = (int)terms.size();
        for (const Cand &cd : cands[c]) {
            int pt[3], f[3];
            cls_shift(pc, cd.d, pt, f);
            const int ctg = pt[0] + p * (pt[1] + p * pt[2]);
            const int sh = f[0] + NX * (f[1] + NY * f[2]);
            Term T{};
            T.fx = f[0], T.fy = f[1], T.fz = f[2];
            T.xofs = (int)(G + (long long)ctg * CS + sh);
            if (cd.off >= 0 || full) {
                T.vofs = seg.at({c, cd.off});
                T.tr = 0;
                ++nstored;
            } else {
                T.vofs = seg.at({ctg, -cd.off}) + sh;
                T.tr = 1;
            }
            terms.push_back(T);
        }
    }
    ct0[ncls] = (int)terms.size();
    // values: random where row and target are free nodes of the lattice
    std::vector<double> hv(nval, 0.0);
    std::mt19937_64 rng(0x5EED);
    std::uniform_real_distribution<double> U(-1, 1);
    long long real_blocks = 0;
    for (int c = 0; c < ncls; ++c) {
        const int pc[3] = {c % p, (c / p) % p, c / (p * p)};
        for (const Cand &cd : cands[c]) {
            if (!(cd.off >= 0 || full)) continue;
            const long long base = seg.at({c, cd.off});
            for (int r = 0; r < CS0; ++r) {
                const long long t[3] = {r % NX, (r / NX) % NY, r / (NX * NY)};
                const long long I[3] = {pc[0] + p * t[0], pc[1] + p * t[1], pc[2] + p * t[2]};
                const long long J[3] = {I[0] + cd.d[0], I[1] + cd.d[1], I[2] + cd.d[2]};
                const bool fi = free_node(I), fj = free_node(J);
                if (fi && fj) {
                    ++real_blocks;
                    for (int e = 0; e < 9; ++e) hv[base + (long long)e * CS + r] = U(rng);
                } else if (!fi && cd.off == 0) {
                    for (int e = 0; e < 3; ++e) hv[base + (long long)(4 * e) * CS + r] = 1.0;
                }
            }
        }
    }
    // wave list: (class, row group), ordered by (z row of the group's first row, class)
    std::vector<int> wl;
    for (int c = 0; c < ncls; ++c)
        for (int r0 = 0; r0 < CS; r0 += 64) wl.push_back(c | ((r0 / 64) << 8));
    if (order) std::stable_sort(wl.begin(), wl.end(), [&](int a, int b) {
        const int ra = (a >> 8) * 64, rb = (b >> 8) * 64;
        return ra / (NX * NY) < rb / (NX * NY);
    });
    printf("nel %d %d %d p %d: class rows %d (x%d), terms %zu, stored streams %lld, values %.3f GB (real blocks %lld = %.3f GB), waves %zu\n",
           NX, NY, NZ, p, CS0, ncls, terms.size(), nstored, nval * 8e-9, real_blocks, real_blocks * 72e-9, wl.size());
    std::vector<double> hx(3 * nP, 0.0), hy(3 * nP, 0.0);
    for (int b = 0; b < 3; ++b)
        for (int c = 0; c < ncls; ++c)
            for (int r = 0; r < CS0; ++r) hx[b * nP + G + (long long)c * CS + r] = U(rng);
    double *dv, *dx, *dy;
    Term *dt;
    int *dw, *dct;
    CK(hipMalloc(&dv, nval * 8));
    CK(hipMalloc(&dx, 3 * nP * 8));
    CK(hipMalloc(&dy, 3 * nP * 8));
    CK(hipMalloc(&dt, terms.size() * sizeof(Term)));
    CK(hipMalloc(&dw, wl.size() * 4));
    CK(hipMalloc(&dct, ct0.size() * 4));
    CK(hipMemcpy(dv, hv.data(), nval * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx, hx.data(), 3 * nP * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dy, 0, 3 * nP * 8));
    CK(hipMemcpy(dt, terms.data(), terms.size() * sizeof(Term), hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, wl.data(), wl.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dct, ct0.data(), ct0.size() * 4, hipMemcpyHostToDevice));
    const int nw = (int)wl.size();
    double *ybase = dy + G, *xbase = dx;
    auto launch = [&]() {
#define L_(NTV, S, BB) hipLaunchKernelGGL((k_sym<NTV, S, BB>), dim3((nw + 4 / S - 1) / (4 / S)), dim3(256), 0, 0, nw, CS, NX, NY, NZ, dw, dct, dt, dv, xbase, ybase, nP)
#define LB_(NTV, S) { if (bat == 1) L_(NTV, S, 1); else if (bat == 2) L_(NTV, S, 2); else L_(NTV, S, 4); }
        if (split == 1) { if (nt) LB_(true, 1) else LB_(false, 1) }
        else if (split == 2) { if (nt) LB_(true, 2) else LB_(false, 2) }
        else { if (nt) LB_(true, 4) else LB_(false, 4) }
#undef LB_
#undef L_
    };
    for (int i = 0; i < 10; ++i) launch();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double stored = 8.0 * nval, vec = 8.0 * 3 * ncls * CS * 2;
    printf("%s split=%d B=%d nt=%d order=%d: %.4f ms/SpMV; stored %.3f GB -> %.2f TB/s; full-matrix (real blocks x2 - diag) equiv %.2f TB/s\n",
           full ? "FULL" : "SYM", split, bat, nt, order, ms, stored * 1e-9, (stored + vec) / (ms * 1e-3) * 1e-12,
           (real_blocks * (full ? 72.0 : 144.0)) / (ms * 1e-3) * 1e-12);
    if (check && !full) {
        CK(hipMemcpy(hy.data(), dy, 3 * nP * 8, hipMemcpyDeviceToHost));
        double maxerr = 0, maxv = 0;
        for (int c = 0; c < ncls; ++c) {
            const int pc[3] = {c % p, (c / p) % p, c / (p * p)};
            for (int r = 0; r < CS0; ++r) {
                const long long t[3] = {r % NX, (r / NX) % NY, r / (NX * NY)};
                double acc[3] = {0, 0, 0};
                for (const Cand &cd : cands[c]) {
                    int pt[3], f[3];
                    cls_shift(pc, cd.d, pt, f);
                    const long long tt[3] = {t[0] + f[0], t[1] + f[1], t[2] + f[2]};
                    if (tt[0] < 0 || tt[0] >= NX || tt[1] < 0 || tt[1] >= NY || tt[2] < 0 || tt[2] >= NZ) continue;
                    const int ctg = pt[0] + p * (pt[1] + p * pt[2]);
                    const long long rt = tt[0] + NX * (tt[1] + NY * tt[2]);
                    double blk[9];
                    if (cd.off >= 0) {
                        const long long base = seg.at({c, cd.off});
                        for (int e = 0; e < 9; ++e) blk[e] = hv[base + (long long)e * CS + r];
                    } else {
                        const long long base = seg.at({ctg, -cd.off});
                        for (int a = 0; a < 3; ++a)
                            for (int b = 0; b < 3; ++b) blk[3 * a + b] = hv[base + (long long)(3 * b + a) * CS + rt];
                    }
                    for (int a = 0; a < 3; ++a)
                        for (int b = 0; b < 3; ++b) acc[a] += blk[3 * a + b] * hx[b * nP + G + (long long)ctg * CS + rt];
                }
                for (int a = 0; a < 3; ++a) {
                    maxerr = std::max(maxerr, std::fabs(acc[a] - hy[a * nP + G + (long long)c * CS + r]));
                    maxv = std::max(maxv, std::fabs(acc[a]));
                }
            }
        }
        printf("check: max |err| %.3e (max |y| %.3e)\n", maxerr, maxv);
    }
    return 0;
}
