// kle_brick_plan.cpp -- host planner of the brick symmetric SpMV
// (kle_brick.hip): where to cut the owned lattice so that every CU streams
// one brick of the same bytes and its region fits the LDS.
#include <algorithm>
#include <climits>
#include <cmath>

#include "kle_brick.hpp"
#include "kle_internal.hpp"

namespace kle {

// cuts of [0, L) into n parts of near-equal weight w[c], each cut moved to a
// multiple of q where that keeps every part non-empty
static bool split_axis(const std::vector<double> &w, int n, int q, std::vector<int> &cut)
{
    const int L = (int)w.size();
    if (n < 1 || n > L) return false;
    std::vector<double> pre(L + 1, 0.0);
    for (int c = 0; c < L; ++c) pre[c + 1] = pre[c] + w[c];
    cut.assign(n + 1, 0);
    cut[n] = L;
    for (int k = 1; k < n; ++k) {
        const double t = pre[L] * k / n;
        int c = (int)(std::lower_bound(pre.begin(), pre.end(), t) - pre.begin());
        if (c > 0 && t - pre[c - 1] < pre[c] - t) --c;  // (the nearer prefix)
        if (q > 1) {
            const int lo = c / q * q, hi = lo + q;
            c = (c - lo <= hi - c) ? lo : hi;
        }
        c = std::max(c, cut[k - 1] + 1);
        c = std::min(c, L - (n - k));
        cut[k] = c;
    }
    return true;
}


// Plan bricks for the owned lattice (one rank, no ghosts): split counts
// (nbx, nby, nbz) with at most ncu bricks (one round: every brick's sums are
// written after the whole value stream) and cut variants per axis, whose
// regions fit the LDS; the shortest modelled time, then the fewest region
// entries.
std::string brick_plan(int Lx, int Ly, int Lz, int ncu, int fs, const std::vector<int> &cnt,
                       const std::vector<int> &srow, int P, BrickPlan &bp, int ncu_all)
{
    if (ncu_all <= 0) ncu_all = ncu;
    const int64_t n = (int64_t)Lx * Ly * Lz, Lxy = (int64_t)Lx * Ly;
    // per row: stored blocks (upper tail) and its byte weight
    std::vector<int> mu(n);
    std::vector<double> wx(Lx, 0.0), wy(Ly, 0.0), wz(Lz, 0.0);
    std::vector<int> xlo(Lx, INT_MAX), xhi(Lx, INT_MIN), ylo(Ly, INT_MAX), yhi(Ly, INT_MIN), zhi(Lz, INT_MIN);
    double total = 0.0;  // (all rows; KLE_TIMING)
    for (int64_t i = 0; i < n; ++i) {
        const int z = (int)(i / Lxy), y = (int)((i % Lxy) / Lx), x = (int)(i % Lx);
        const int d = srow[i];
        const int dbx = d & 15, dby = (d >> 4) & 15, dbz = (d >> 8) & 15;
        const int bnx = (d >> 12) & 15, bny = (d >> 16) & 15, bnz = (d >> 20) & 15;
        const int k0 = dbx + bnx * (dby + bny * dbz);
        mu[i] = cnt[i] - k0;
        const double wgt = 72.0 * mu[i] + 64.0;
        wx[x] += wgt;
        wy[y] += wgt;
        wz[z] += wgt;
        total += wgt;
        // the upper triangle's extent: planes above take the whole box, the
        // row's own plane the lines from its own on
        const int bx = x - dbx, by = y - dby, bz = z - dbz;
        const int uz1 = bz + bnz - 1, uy1 = by + bny - 1, ux1 = bx + bnx - 1;
        const int uy0 = uz1 > z ? by : y, ux0 = uz1 > z || uy1 > y ? bx : x;
        xlo[x] = std::min(xlo[x], ux0);
        xhi[x] = std::max(xhi[x], ux1);
        ylo[y] = std::min(ylo[y], uy0);
        yhi[y] = std::max(yhi[y], uy1);
        zhi[z] = std::max(zhi[z], uz1);
    }
    // 3-D prefix sums of the row weights: box_sum over [x0,x1) x [y0,y1) x [z0,z1)
    const int64_t PX1 = Lx + 1, PXY1 = PX1 * (Ly + 1);
    std::vector<double> pw((size_t)PXY1 * (Lz + 1), 0.0);
    for (int z = 0; z < Lz; ++z)
        for (int y = 0; y < Ly; ++y)
            for (int x = 0; x < Lx; ++x) {
                const int64_t i = x + (int64_t)Lx * y + Lxy * z;
                const double v = 72.0 * mu[i] + 64.0;
                const int64_t q = (x + 1) + PX1 * (y + 1) + PXY1 * (z + 1);
                pw[q] = v + pw[q - 1] + pw[q - PX1] + pw[q - PXY1] - pw[q - 1 - PX1] - pw[q - 1 - PXY1] -
                        pw[q - PX1 - PXY1] + pw[q - 1 - PX1 - PXY1];
            }
    auto box_sum = [&](int x0, int x1, int y0, int y1, int z0, int z1) {
        auto at = [&](int x, int y, int z) { return pw[x + PX1 * y + PXY1 * z]; };
        return at(x1, y1, z1) - at(x0, y1, z1) - at(x1, y0, z1) - at(x1, y1, z0) + at(x0, y0, z1) + at(x0, y1, z0) +
               at(x1, y0, z0) - at(x0, y0, z0);
    };
    auto region = [&](const std::vector<int> &lo, const std::vector<int> &hi, int c0, int c1, int &o, int &R) {
        int a = INT_MAX, bmax = INT_MIN;
        for (int c = c0; c < c1; ++c) {
            a = std::min(a, lo.empty() ? c : lo[c]);
            bmax = std::max(bmax, hi[c]);
        }
        o = a;
        R = bmax - a + 1;
    };
    const std::vector<int> zlo_none;
    // Time model of one plan: every brick starts at once, the active CUs
    // share the stream at the per-CU rate r(k) measured with k of 256 CUs
    // streaming (tools/stream_cus.py: 61 GB/s alone .. 26.8 GB/s all busy,
    // chip 6.87 TB/s; profiles/r05/stream_cus.jsonl) but at most the item
    // loop's own cap, so the light bricks' early end speeds the heavy ones up
    // a little; bricks sorted by bytes end in order.
    auto rate_pc = [&](int k) {
        static const double kk[] = {0, 16, 32, 64, 128, 192, 256}, tb[] = {0, 0.98, 1.90, 3.51, 6.00, 7.11, 6.87};
        const double f = 256.0 * k / ncu_all;
        int j = 1;
        while (j < 6 && kk[j] < f) ++j;
        const double R = tb[j - 1] + (tb[j] - tb[j - 1]) * (std::min(f, 256.0) - kk[j - 1]) / (kk[j] - kk[j - 1]);
        // (per CU, TB/s; the SpMV's item loop itself tops out near 1.06x its
        // all-busy rate: 24.7 -> 27.5 GB/s per CU from 256 to 224 bricks,
        // profiles/r05/phase_bricks_*.jsonl)
        return std::min(R / std::max(f, 1e-9), 1.06 * 6.87 / 256.0);
    };
    auto model = [&](std::vector<double> w) {
        std::sort(w.begin(), w.end());
        double t = 0.0, done = 0.0;
        const int NB = (int)w.size();
        for (int j = 0; j < NB; ++j) {
            t += (w[j] - done) / rate_pc(NB - j);
            done = w[j];
        }
        return t;
    };
    double best_t = 1e300;
    int64_t best_ent = INT64_MAX;
    std::vector<int> bcx, bcy, bcz;
    // (fs: forced split counts nbx + 100 nby + 10000 nbz; + 1000000: cuts by
    // equal node counts only; + 10000000: weighted cuts at any node only)
    const int fmode = fs / 1000000;
    fs %= 1000000;
    const std::vector<double> ux(Lx, 1.0), uy(Ly, 1.0), uz(Lz, 1.0);
    // per axis the cut variants tried: equal weights at element boundaries,
    // equal weights at any node (x, y: a region grows by at most p - 1
    // nodes), equal node counts at element boundaries
    struct Var {
        const std::vector<double> *w;
        int q;
    };
    std::vector<Var> vx, vy, vz;
    if (fmode == 0 || fmode == 1) vx.push_back({fmode ? &ux : &wx, P});
    if (fmode == 0 || fmode == 10) vx.push_back({&wx, 1});
    if (fmode == 0) vx.push_back({&ux, P});
    if (fmode == 0 || fmode == 1) vy.push_back({fmode ? &uy : &wy, P});
    if (fmode == 0 || fmode == 10) vy.push_back({&wy, 1});
    if (fmode == 0) vy.push_back({&uy, P});
    vz.push_back({fmode == 1 ? &uz : &wz, P});
    if (fmode == 0) vz.push_back({&uz, P});
    // (at least an element per brick along each axis: regions then reach the
    // neighbouring bricks only)
    const int ex = std::max(1, (Lx - 1) / std::max(P, 1)), ey = std::max(1, (Ly - 1) / std::max(P, 1)),
              ez = std::max(1, (Lz - 1) / std::max(P, 1));
    for (int nbz = 1; nbz <= std::min(ez, ncu); ++nbz)
        for (int nby = 1; nby <= std::min(ey, ncu / nbz); ++nby)
            for (int nbx = 1; nbx <= std::min(ex, ncu / (nbz * nby)); ++nbx) {
                if (fs && fs != nbx + 100 * nby + 10000 * nbz) continue;
                for (const Var &VX : vx)
                    for (const Var &VY : vy)
                        for (const Var &VZ : vz) {
                            std::vector<int> cx, cy, cz;
                            if (!split_axis(*VX.w, nbx, VX.q, cx) || !split_axis(*VY.w, nby, VY.q, cy) ||
                                !split_axis(*VZ.w, nbz, VZ.q, cz))
                                continue;
                            int64_t ent = 0;
                            std::vector<int> RXs(nbx), RYs(nby), RZs(nbz);
                            int o;
                            for (int a = 0; a < nbx; ++a) region(xlo, xhi, cx[a], cx[a + 1], o, RXs[a]);
                            for (int a = 0; a < nby; ++a) region(ylo, yhi, cy[a], cy[a + 1], o, RYs[a]);
                            for (int a = 0; a < nbz; ++a) region(zlo_none, zhi, cz[a], cz[a + 1], o, RZs[a]);
                            bool fits = true;
                            std::vector<double> w;
                            w.reserve((size_t)nbx * nby * nbz);
                            for (int e = 0; e < nbz && fits; ++e)
                                for (int c = 0; c < nby && fits; ++c)
                                    for (int a = 0; a < nbx && fits; ++a) {
                                        const int RN = RXs[a] * RYs[c] * RZs[e];
                                        if (RN > 65535 || brick_lds(RN) > BRICK_LDS_CAP) fits = false;
                                        ent += RN;
                                        // bytes: the values, plus x and the sums of the region
                                        w.push_back(box_sum(cx[a], cx[a + 1], cy[c], cy[c + 1], cz[e], cz[e + 1]) +
                                                    72.0 * RN);
                                    }
                            if (!fits) continue;
                            const double t = model(w);
                            if (t < best_t * 0.999 || (t <= best_t * 1.001 && ent < best_ent)) {
                                best_t = t;
                                best_ent = ent;
                                bcx = cx;
                                bcy = cy;
                                bcz = cz;
                            }
                        }
            }
    bp.model_us = best_t * 1e-6;  // (bytes / (TB/s) = us)
    (void)total;
    if (bcx.empty()) return "no brick decomposition fits the LDS";
    const int nbx = (int)bcx.size() - 1, nby = (int)bcy.size() - 1, nbz = (int)bcz.size() - 1, NB = nbx * nby * nbz;
    bp.bricks.assign(NB, BrickDesc{});
    bp.rowd.assign(2 * n, 0);
    bp.svb.assign(n + 1, 0);
    int64_t voff = 0, rows = 0, wsd = 0;
    bp.lds = 0;
    bp.ws_entries = 0;
    for (int e = 0; e < nbz; ++e)
        for (int c = 0; c < nby; ++c)
            for (int a = 0; a < nbx; ++a) {
                BrickDesc &D = bp.bricks[((size_t)e * nby + c) * nbx + a];
                D.x0 = bcx[a];
                D.nx = bcx[a + 1] - bcx[a];
                D.y0 = bcy[c];
                D.ny = bcy[c + 1] - bcy[c];
                D.z0 = bcz[e];
                D.nz = bcz[e + 1] - bcz[e];
                region(xlo, xhi, bcx[a], bcx[a + 1], D.ox, D.RX);
                region(ylo, yhi, bcy[c], bcy[c + 1], D.oy, D.RY);
                region(zlo_none, zhi, bcz[e], bcz[e + 1], D.oz, D.RZ);
                const int RN = D.RX * D.RY * D.RZ;
                D.rstart = (int)rows;
                D.eb = 0;
                D.vbase = voff;
                D.wsoff = wsd;
                wsd += ((int64_t)3 * RN + 15) & ~int64_t(15);
                bp.lds = std::max(bp.lds, brick_lds(RN));
                for (int z = D.z0; z < D.z0 + D.nz; ++z)
                    for (int y = D.y0; y < D.y0 + D.ny; ++y)
                        for (int x = D.x0; x < D.x0 + D.nx; ++x) {
                            const int64_t i = x + (int64_t)Lx * y + Lxy * z;
                            bp.svb[i] = voff;
                            const int64_t o = voff - D.vbase;
                            if ((o >> 4) >= (1 << 24)) return "brick values beyond 2^28 doubles";
                            const int ir = (x - D.ox) + D.RX * ((y - D.oy) + D.RY * (z - D.oz));
                            bp.rowd[2 * rows] = (srow[i] & 0xFFFFFF) | ((ir & 255) << 24);
                            bp.rowd[2 * rows + 1] = (int)((o >> 4) | ((int64_t)((ir >> 8) & 255) << 24));
                            voff += ((int64_t)mu[i] * 9 + 15) & ~int64_t(15);
                            ++rows;
                        }
                // lattice entries of the region (written by the brick, read by the gather)
                for (int z = D.oz; z < D.oz + D.RZ; ++z)
                    for (int y = D.oy; y < D.oy + D.RY; ++y)
                        for (int x = D.ox; x < D.ox + D.RX; ++x)
                            bp.ws_entries += x >= 0 && x < Lx && y >= 0 && y < Ly && z >= 0 && z < Lz;
            }
    bp.svb[n] = voff;
    bp.ws_doubles = wsd;
    // per brick, the bricks whose regions meet its owned box (ascending)
    bp.nbptr.assign(NB + 1, 0);
    bp.nblist.clear();
    for (int q = 0; q < NB; ++q) {
        const BrickDesc &D = bp.bricks[q];
        for (int q2 = 0; q2 < NB; ++q2) {
            const BrickDesc &E = bp.bricks[q2];
            const bool meet = E.ox < D.x0 + D.nx && D.x0 < E.ox + E.RX && E.oy < D.y0 + D.ny && D.y0 < E.oy + E.RY &&
                              E.oz < D.z0 + D.nz && D.z0 < E.oz + E.RZ;
            if (meet) bp.nblist.push_back(q2);
        }
        bp.nbptr[q + 1] = (int)bp.nblist.size();
        if (bp.nbptr[q + 1] - bp.nbptr[q] > BG_MAXNB) return "a brick's rows meet more than 64 brick regions";
    }
    bp.lds = std::max(bp.lds, BRICK_LDS_MIN);
    return "";
}

}  // namespace kle

// Diagnostic (host only, no device): the brick plan of an Lx x Ly x Lz box
// lattice of p-node elements (element-aligned row boxes, the pattern of
// MatFS.buildFS on a box mesh, mat_fs.py:21-94) for ncu CUs -- what the
// symmetric storage of such a K would run (kle_sym.hip, one rank).
// dirichlet: every boundary node is a Dirichlet node -- its row the diagonal
// block alone, its column in no other row (the K of buildFS with Dirichlet
// data on all faces, as the bench's Taylor-Green case).
// info[0] bricks, [1] bricks along x, [2] y, [3] z, [4] LDS bytes;
// stats[0] bytes of the largest brick / the mean, [1] region entries per row,
// [2] stored blocks, [3] the planner's time model (us).  Returns KLE_ERR_SUP (with the reason) when no plan fits.
extern "C" int kle_brick_plan_box(int Lx, int Ly, int Lz, int p, int dirichlet, int ncu, int split, int *info,
                                  double *stats)
{
    using namespace kle;
    KLE_ARG(Lx >= 1 && Ly >= 1 && Lz >= 1 && p >= 1 && p <= 7 && ncu >= 1 && info && stats, "bad arg");
    const int64_t n = (int64_t)Lx * Ly * Lz;
    std::vector<int> cnt(n), srow(n);
    auto box = [&](int c, int L, int &b, int &nb) {  // element-aligned box of coordinate c
        const int e = c / p;
        const bool onb = c % p == 0;
        b = onb && c > 0 ? c - p : e * p;
        int hi = onb && c < L - 1 ? c + p : std::min(L - 1, e * p + p);
        if (onb && c == L - 1) hi = c;
        if (dirichlet && L > 2) {  // (free rows: only free columns)
            b = std::max(b, 1);
            hi = std::min(hi, L - 2);
        }
        nb = hi - b + 1;
    };
    int64_t blocks = 0;
    for (int z = 0; z < Lz; ++z)
        for (int y = 0; y < Ly; ++y)
            for (int x = 0; x < Lx; ++x) {
                int bx, nx, by, ny, bz, nz;
                box(x, Lx, bx, nx);
                box(y, Ly, by, ny);
                box(z, Lz, bz, nz);
                if (dirichlet && (x == 0 || y == 0 || z == 0 || x == Lx - 1 || y == Ly - 1 || z == Lz - 1)) {
                    bx = x, by = y, bz = z;
                    nx = ny = nz = 1;
                }
                const int64_t i = x + (int64_t)Lx * (y + (int64_t)Ly * z);
                cnt[i] = nx * ny * nz;
                srow[i] = (x - bx) | (y - by) << 4 | (z - bz) << 8 | nx << 12 | ny << 16 | nz << 20;
                blocks += cnt[i] - ((x - bx) + nx * ((y - by) + ny * (z - bz)));
            }
    BrickPlan bp;
    const std::string why = brick_plan(Lx, Ly, Lz, ncu, split, cnt, srow, p, bp, ncu);
    if (!why.empty()) return fail(KLE_ERR_SUP, "%s", why.c_str());
    const int NB = (int)bp.bricks.size();
    double tot = 0.0, mx = 0.0;
    for (const BrickDesc &D : bp.bricks) {
        double w = 0.0;
        for (int r = 0; r < D.nx * D.ny * D.nz; ++r) {
            const int rz = r / (D.nx * D.ny), rem = r - rz * D.nx * D.ny, ry = rem / D.nx, rx = rem - ry * D.nx;
            const int64_t i = (D.x0 + rx) + (int64_t)Lx * ((D.y0 + ry) + (int64_t)Ly * (D.z0 + rz));
            const int d = srow[i];
            const int k0 = (d & 15) + ((d >> 12) & 15) * (((d >> 4) & 15) + ((d >> 16) & 15) * ((d >> 8) & 15));
            w += 72.0 * (cnt[i] - k0) + 64.0;
        }
        tot += w;
        mx = std::max(mx, w);
    }
    int cx = 0, cy = 0, cz = 0;
    for (const BrickDesc &D : bp.bricks) {
        cx += D.y0 == 0 && D.z0 == 0;
        cy += D.x0 == 0 && D.z0 == 0;
        cz += D.x0 == 0 && D.y0 == 0;
    }
    info[0] = NB;
    info[1] = cx;
    info[2] = cy;
    info[3] = cz;
    info[4] = (int)bp.lds;
    stats[0] = mx / (tot / NB);
    stats[1] = (double)bp.ws_entries / n;
    stats[2] = (double)blocks;
    stats[3] = bp.model_us;
    return 0;
}
