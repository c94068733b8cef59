// Prototype (tool, not product): symmetric "position-class" block-diagonal
// storage of the box-mesh KLE matrix and its SpMV.
//
// Free rows of a p-order GLL box lattice fall into p^3 classes by their
// position inside the element, (ix mod p, iy mod p, iz mod p).  Rows of one
// class form a regular sub-lattice and share one set of block offsets d, so
// for a fixed (class, d) the blocks A(i, i+d) of consecutive class rows are
// consecutive in memory (SoA, one stream per block entry).  Only d >= 0
// (node-id order) is stored; row i reads its lower blocks A(i, i+e), e < 0,
// as A(i+e, i)^T from the partner class's stream, whose rows i+e are again
// consecutive -> every load is coalesced and the matrix stream is halved.
// The partner read re-touches bytes another wave streamed shortly before
// (terms are ordered by |offset|, waves by element layer), which is what
// this prototype measures: hipcc --offload-arch=gfx950 -O3 sym_proto.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
    long long vbase;  // first double of the 9 streams
    int vlen;         // stream stride (doubles)
    int ax, ay, az, nx, ny, nz;  // valid row box in the row class's coordinates
    int xbase, xsy, xsz;         // P-space index of x(i+d) = xbase + sx + xsy*sy + xsz*sz
    int tr;                      // read the block transposed
    int pad[3];
};
struct ClassInfo {
    int NX, NY, NZ, cnt, off, t0, t1, pad;
};
struct WaveItem {
    int cls, r0;
};

// SPLIT waves share one group of 64 class rows; wave q takes terms
// t0+q, t0+q+SPLIT, ...; the partial sums are added in wave order
// (deterministic).  Each wave issues the loads of B terms before it uses any.
template <bool NT, int SPLIT, int B>
__global__ __launch_bounds__(256) void k_sym(const WaveItem *__restrict__ waves, int nwaves,
                                             const ClassInfo *__restrict__ cls, const Term *__restrict__ terms,
                                             const double *__restrict__ val, const double *__restrict__ x,
                                             double *__restrict__ y, long long nP)
{
    constexpr int GROUPS = 4 / SPLIT;
    __shared__ double part[SPLIT > 1 ? 4 : 1][3][64];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = wv % SPLIT, g = wv / SPLIT;
    const int w = blockIdx.x * GROUPS + g;
    const int lane = threadIdx.x & 63;
    const bool live = w < nwaves;
    const WaveItem wi = waves[live ? w : 0];
    const ClassInfo ci = cls[wi.cls];
    const int r = wi.r0 + lane;
    const bool act = live & (r < ci.cnt);
    const int sx = r % ci.NX, qq = r / ci.NX, sy = qq % ci.NY, sz = qq / ci.NY;
    double a0 = 0, a1 = 0, a2 = 0;
    const int t1 = live ? ci.t1 : ci.t0;
    for (int k0 = ci.t0 + q; k0 < t1; k0 += SPLIT * B) {
        double bv[B][9], xv[B][3];
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int k = k0 + u * SPLIT;
            const bool tv = k < t1;
            const Term &T = terms[tv ? k : ci.t0];
            const unsigned ux = sx - T.ax, uy = sy - T.ay, uz = sz - T.az;
            const bool ok = tv & act & (ux < (unsigned)T.nx) & (uy < (unsigned)T.ny) & (uz < (unsigned)T.nz);
            const long long li = ok ? ux + (long long)T.nx * (uy + (long long)T.ny * uz) : 0;
            const double *v = val + T.vbase + li;
            const long long st = T.vlen;
            const long long s1 = T.tr ? 3 * st : st, s3 = T.tr ? st : 3 * st;
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const double *pp = v + a * s3 + c * s1;
                    bv[u][3 * a + c] = NT ? __builtin_nontemporal_load(pp) : *pp;
                }
            const long long xi = ok ? T.xbase + sx + (long long)T.xsy * sy + (long long)T.xsz * sz : 0;
            xv[u][0] = x[xi];
            xv[u][1] = x[xi + nP];
            xv[u][2] = x[xi + 2 * nP];
            if (!ok) xv[u][0] = xv[u][1] = xv[u][2] = 0.0;
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
            a0 += bv[u][0] * xv[u][0] + bv[u][1] * xv[u][1] + bv[u][2] * xv[u][2];
            a1 += bv[u][3] * xv[u][0] + bv[u][4] * xv[u][1] + bv[u][5] * xv[u][2];
            a2 += bv[u][6] * xv[u][0] + bv[u][7] * xv[u][1] + bv[u][8] * xv[u][2];
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
    if (act) {
        y[ci.off + r] = a0;
        y[nP + ci.off + r] = a1;
        y[2 * nP + ci.off + r] = a2;
    }
}

// ---- host-side lattice bookkeeping (one dimension)
struct Dim1 {
    int nel, p;
    int tlo(int px) const { return px == 0 ? 1 : 0; }
    int count(int px) const { return nel - tlo(px); }
    int omin(int px) const { return px == 0 ? -p : -px; }
    int omax(int px) const { return px == 0 ? p : p - px; }
    static int fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
    // valid row range [lo, hi) of class px for offset d, and the target (class, shift)
    bool term(int px, int d, int &lo, int &hi, int &pt, int &shift) const
    {
        const int f = fdiv(px + d, p);
        pt = px + d - f * p;
        shift = tlo(px) + f - tlo(pt);  // s_target = s + shift
        lo = std::max(0, -shift);
        hi = std::min(count(px), count(pt) - shift);
        return hi > lo;
    }
};

int main(int argc, char **argv)
{
    int nel[3] = {20, 16, 16}, p = 4, reps = 200, full = 0, check = 0, nt = 1, order = 1, split = 4, bat = 2;
    if (argc > 3) for (int k = 0; k < 3; ++k) nel[k] = atoi(argv[1 + k]);
    if (argc > 4) p = atoi(argv[4]);
    if (argc > 5) full = atoi(argv[5]);
    if (argc > 6) check = atoi(argv[6]);
    if (argc > 7) nt = atoi(argv[7]);
    if (argc > 8) order = atoi(argv[8]);
    if (argc > 9) reps = atoi(argv[9]);
    if (argc > 10) split = atoi(argv[10]);
    if (argc > 11) bat = atoi(argv[11]);
    Dim1 D[3] = {{nel[0], p}, {nel[1], p}, {nel[2], p}};
    const long long L[3] = {(long long)nel[0] * p + 1, (long long)nel[1] * p + 1, (long long)nel[2] * p + 1};
    const int ncls = p * p * p;
    std::vector<ClassInfo> cls(ncls);
    long long nP = 0;
    for (int c = 0; c < ncls; ++c) {
        const int px = c % p, py = (c / p) % p, pz = c / (p * p);
        ClassInfo &ci = cls[c];
        ci.NX = D[0].count(px), ci.NY = D[1].count(py), ci.NZ = D[2].count(pz);
        ci.cnt = ci.NX * ci.NY * ci.NZ;
        ci.off = (int)nP;
        nP += ci.cnt;
    }
    // stored segments: (class, d>=0) -> vbase
    struct Seg { long long vbase; int vlen; };
    std::map<std::pair<int, long long>, Seg> seg;  // key (class, id offset)
    long long nval = 0, nstored_blocks = 0, nblocks_full = 0;
    auto idoff = [&](int dx, int dy, int dz) { return dx + L[0] * (dy + L[1] * dz); };
    std::vector<Term> terms;
    for (int c = 0; c < ncls; ++c) {
        const int pc[3] = {c % p, (c / p) % p, c / (p * p)};
        struct Cand { long long off; int d[3]; };
        std::vector<Cand> cand;
        for (int dz = D[2].omin(pc[2]); dz <= D[2].omax(pc[2]); ++dz)
            for (int dy = D[1].omin(pc[1]); dy <= D[1].omax(pc[1]); ++dy)
                for (int dx = D[0].omin(pc[0]); dx <= D[0].omax(pc[0]); ++dx) cand.push_back({idoff(dx, dy, dz), {dx, dy, dz}});
        if (order) std::sort(cand.begin(), cand.end(), [](const Cand &a, const Cand &b) {
            long long aa = std::llabs(a.off), bb = std::llabs(b.off);
            return aa != bb ? aa < bb : a.off > b.off;
        });
        cls[c].t0 = (int)terms.size();
        for (const Cand &cd : cand) {
            int lo[3], hi[3], pt[3], sh[3];
            bool ok = true;
            for (int k = 0; k < 3; ++k) ok = ok && D[k].term(pc[k], cd.d[k], lo[k], hi[k], pt[k], sh[k]);
            if (!ok) continue;
            Term T{};
            T.ax = lo[0], T.ay = lo[1], T.az = lo[2];
            T.nx = hi[0] - lo[0], T.ny = hi[1] - lo[1], T.nz = hi[2] - lo[2];
            const int ct = pt[0] + p * (pt[1] + p * pt[2]);
            const ClassInfo &tc = cls[ct];
            T.xsy = tc.NX, T.xsz = tc.NX * tc.NY;
            T.xbase = tc.off + sh[0] + tc.NX * (sh[1] + tc.NY * sh[2]);
            const long long vol = (long long)T.nx * T.ny * T.nz;
            nblocks_full += vol;
            if (cd.off >= 0 || full) {
                Seg s{nval, (int)((vol + 15) & ~15LL)};
                nval += 9LL * s.vlen;
                nstored_blocks += vol;
                seg[{c, cd.off}] = s;
                T.vbase = s.vbase, T.vlen = s.vlen, T.tr = 0;
            } else {
                T.vbase = -1;  // resolved below (partner segment may not exist yet)
                T.tr = 1;
                T.vlen = ct;  // temporarily: partner class
                T.pad[0] = (int)(-cd.off);  // |offset| fits int for these sizes
            }
            terms.push_back(T);
        }
        cls[c].t1 = (int)terms.size();
    }
    for (Term &T : terms)
        if (T.vbase < 0) {
            const Seg &s = seg.at({T.vlen, (long long)T.pad[0]});
            T.vbase = s.vbase, T.vlen = s.vlen, T.pad[0] = 0;
        }
    // wave list ordered by (element layer, class)
    std::vector<WaveItem> waves;
    for (int c = 0; c < ncls; ++c)
        for (int r0 = 0; r0 < cls[c].cnt; r0 += 64) waves.push_back({c, r0});
    if (order) std::stable_sort(waves.begin(), waves.end(), [&](const WaveItem &a, const WaveItem &b) {
        const int za = a.r0 / (cls[a.cls].NX * cls[a.cls].NY), zb = b.r0 / (cls[b.cls].NX * cls[b.cls].NY);
        const int pa = a.cls / (p * p), pb = b.cls / (p * p);
        const int la = za + (pa == 0 ? 1 : 0), lb = zb + (pb == 0 ? 1 : 0);  // element layer of the row
        return la < lb;
    });
    printf("nel %d %d %d p %d: free rows %lld, classes %d, terms %zu, blocks full %lld stored %lld, values %.3f GB, waves %zu\n",
           nel[0], nel[1], nel[2], p, nP, ncls, terms.size(), nblocks_full, nstored_blocks, nval * 8e-9, waves.size());

    std::vector<double> hv(nval, 0.0), hx(3 * nP), hy(3 * nP);
    std::mt19937_64 rng(0x5EED);
    std::uniform_real_distribution<double> U(-1, 1);
    for (auto &kv : seg) {
        const Seg &s = kv.second;
        for (long long t = 0; t < 9LL * s.vlen; ++t) hv[s.vbase + t] = U(rng);
    }
    if (full) {  // make the explicitly stored lower blocks the transposes of the upper ones
        for (int c = 0; c < ncls; ++c)
            for (int k = cls[c].t0; k < cls[c].t1; ++k) (void)k;  // values are independent; checked only in sym mode
    }
    for (auto &v : hx) v = U(rng);
    double *dv, *dx, *dy;
    Term *dt;
    ClassInfo *dc;
    WaveItem *dw;
    CK(hipMalloc(&dv, nval * 8));
    CK(hipMalloc(&dx, 3 * nP * 8));
    CK(hipMalloc(&dy, 3 * nP * 8));
    CK(hipMalloc(&dt, terms.size() * sizeof(Term)));
    CK(hipMalloc(&dc, cls.size() * sizeof(ClassInfo)));
    CK(hipMalloc(&dw, waves.size() * sizeof(WaveItem)));
    CK(hipMemcpy(dv, hv.data(), nval * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx, hx.data(), 3 * nP * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, terms.data(), terms.size() * sizeof(Term), hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, cls.data(), cls.size() * sizeof(ClassInfo), hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, waves.data(), waves.size() * sizeof(WaveItem), hipMemcpyHostToDevice));
    const int nw = (int)waves.size();
    auto launch = [&]() {
#define L_(NTV, S, BB) hipLaunchKernelGGL((k_sym<NTV, S, BB>), dim3((nw + 4 / S - 1) / (4 / S)), dim3(256), 0, 0, dw, nw, dc, dt, dv, dx, dy, nP)
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
    const double stored = 72.0 * nstored_blocks, vec = 8.0 * 3 * nP * 2;
    printf("%s split=%d B=%d nt=%d order=%d: %.4f ms/SpMV; stored value bytes %.3f GB -> %.2f TB/s of stored bytes; full-matrix bytes %.3f GB -> %.2f TB/s equiv\n",
           full ? "FULL" : "SYM", split, bat, nt, order, ms, stored * 1e-9, (stored + vec) / (ms * 1e-3) * 1e-12, 72.0 * nblocks_full * 1e-9,
           (72.0 * nblocks_full + vec) / (ms * 1e-3) * 1e-12);
    if (check && !full) {
        CK(hipMemcpy(hy.data(), dy, 3 * nP * 8, hipMemcpyDeviceToHost));
        // independent CPU product over the lattice
        auto cls_of = [&](const long long *ix, int &c, long long &pidx) {
            int pc[3];
            long long s[3];
            for (int k = 0; k < 3; ++k) {
                pc[k] = (int)(ix[k] % p);
                s[k] = ix[k] / p - D[k].tlo(pc[k]);
            }
            c = pc[0] + p * (pc[1] + p * pc[2]);
            pidx = s[0] + cls[c].NX * (s[1] + (long long)cls[c].NY * s[2]);
        };
        double maxerr = 0, maxv = 0;
        for (long long iz = 1; iz < L[2] - 1; ++iz)
            for (long long iy = 1; iy < L[1] - 1; ++iy)
                for (long long ixx = 1; ixx < L[0] - 1; ++ixx) {
                    const long long I[3] = {ixx, iy, iz};
                    int c;
                    long long pi;
                    cls_of(I, c, pi);
                    const int pc[3] = {c % p, (c / p) % p, c / (p * p)};
                    double acc[3] = {0, 0, 0};
                    for (int dz = D[2].omin(pc[2]); dz <= D[2].omax(pc[2]); ++dz)
                        for (int dy = D[1].omin(pc[1]); dy <= D[1].omax(pc[1]); ++dy)
                            for (int dx = D[0].omin(pc[0]); dx <= D[0].omax(pc[0]); ++dx) {
                                const long long J[3] = {ixx + dx, iy + dy, iz + dz};
                                bool fr = true;
                                for (int k = 0; k < 3; ++k) fr = fr && J[k] >= 1 && J[k] <= L[k] - 2;
                                if (!fr) continue;
                                const long long off = idoff(dx, dy, dz);
                                int cj;
                                long long pj;
                                cls_of(J, cj, pj);
                                // block (I, J): stored with the row of the smaller id
                                const bool up = off >= 0;
                                const long long *R = up ? I : J;
                                int cr;
                                long long pr;
                                cls_of(R, cr, pr);
                                const Seg &s = seg.at({cr, up ? off : -off});
                                // local index of R inside the segment's valid box
                                const int prc[3] = {cr % p, (cr / p) % p, cr / (p * p)};
                                const int dd[3] = {up ? dx : -dx, up ? dy : -dy, up ? dz : -dz};
                                long long li = 0, mul = 1;
                                for (int k = 0; k < 3; ++k) {
                                    int lo, hi, pt, sh;
                                    D[k].term(prc[k], dd[k], lo, hi, pt, sh);
                                    const long long sr = R[k] / p - D[k].tlo(prc[k]);
                                    li += (sr - lo) * mul;
                                    mul *= hi - lo;
                                }
                                double b[9];
                                for (int t = 0; t < 9; ++t) b[t] = hv[s.vbase + li + (long long)t * s.vlen];
                                for (int a = 0; a < 3; ++a)
                                    for (int bb = 0; bb < 3; ++bb)
                                        acc[a] += (up ? b[a * 3 + bb] : b[bb * 3 + a]) * hx[bb * nP + cls[cj].off + pj];
                            }
                    for (int a = 0; a < 3; ++a) {
                        maxerr = std::max(maxerr, std::fabs(acc[a] - hy[a * nP + cls[c].off + pi]));
                        maxv = std::max(maxv, std::fabs(acc[a]));
                    }
                }
        printf("check: max |err| %.3e (max |y| %.3e)\n", maxerr, maxv);
    }
    return 0;
}
