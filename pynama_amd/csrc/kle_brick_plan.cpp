// kle_brick_plan.cpp -- host planner of the brick symmetric SpMV
// (kle_brick.hip): where to cut the owned lattice so that every CU streams
// one brick of the same bytes and its region fits the LDS.
#include <algorithm>
#include <climits>
#include <cmath>
#include <functional>

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


// Plan bricks for the owned lattice (one rank, no ghosts) on ncu CUs: up to
// `rounds` bricks per CU (nfix > 0: exactly at most nfix bricks), from three
// generators -- one tensor grid of split counts and cut variants per axis,
// per-slab grids, per-slab recursive bisection -- whose regions fit the
// LDS; the shortest modelled time, then the fewest region entries.  One
// brick per CU writes every brick's sums after the whole value stream; more
// balance the CUs (heaviest first to the first free CU) at the price of a
// refill and sums written mid-stream.
// What a row costs a brick, in bytes of streaming: its 64-block passes
// ("items"), each as if full.  With the memory system saturated every item in
// flight is served in about the same time whatever its bytes: the measured
// loop time of 512 config-2 bricks follows their item counts (correlation
// 0.93, 0.138 us per 1000 items) and not their bytes (0.26), so bricks full
// of short rows -- the one-block Dirichlet rows of a boundary face -- would
// end last (profiles/r05/brick_items_vs_bytes.txt).
static double row_cost(int mu) { return 4608.0 * ((mu + 63) / 64); }

std::string brick_plan(int Lx, int Ly, int Lz, int hp, int ncu, int nfix, int rounds, int fs, const std::vector<int> &cnt,
                       const std::vector<int> &srow, int P, BrickPlan &bp)
{
    const int ncu_all = ncu;
    const int64_t n = (int64_t)Lx * Ly * Lz, Lxy = (int64_t)Lx * Ly;
    // per row: stored blocks (upper tail) and its byte weight
    std::vector<int> mu(n);
    // (a row of one stored block costs a brick nothing when the gather forms
    // it)
    auto rcost = [&](int64_t i) {
        if (bp.singles && mu[i] == 1) return 0.0;
        return row_cost(mu[i]);
    };
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
        const double wgt = rcost(i);
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
                const double v = rcost(i);
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
        // (x 1.246: the rates are of bytes, the costs of full-item bytes --
        // 33.4 GB/s of them per CU with every CU busy, against 26.8 GB/s)
        return 1.246 * std::min(R / std::max(f, 1e-9), 1.06 * 6.87 / 256.0);
    };
    // bricks are dispatched in descending bytes to the first free CU (one per
    // CU: each asks for more than half the LDS); every brick after a CU's
    // first pays a refill (x fill, first loads) of about 100 KB of streaming
    auto model = [&](std::vector<double> w) {
        std::sort(w.rbegin(), w.rend());
        const int NB = (int)w.size();
        std::vector<double> act;
        int q = 0;
        for (; q < NB && q < ncu; ++q) act.push_back(w[q]);
        double t = 0.0;
        while (!act.empty()) {
            const double r = rate_pc((int)act.size());
            const double m = *std::min_element(act.begin(), act.end());
            t += m / r;
            std::vector<double> nx;
            for (double v : act)
                if (v - m > 1e-6) nx.push_back(v - m);
                else if (q < NB) nx.push_back(w[q++] + 1.0e5);
            act.swap(nx);
        }
        return t;
    };
    double best_t = 1e300;
    int64_t best_ent = INT64_MAX;
    struct Box {
        int x0, x1, y0, y1, z0, z1;
    };
    // a brick: its rows (lattice indices) in streaming order; boxes and the
    // ragged bands below are both given this way
    std::vector<std::vector<int64_t>> best;
    auto box_rows = [&](const Box &B) {
        std::vector<int64_t> r;
        r.reserve((size_t)(B.x1 - B.x0) * (B.y1 - B.y0) * (B.z1 - B.z0));
        for (int z = B.z0; z < B.z1; ++z)
            for (int y = B.y0; y < B.y1; ++y)
                for (int x = B.x0; x < B.x1; ++x) r.push_back(x + (int64_t)Lx * y + Lxy * z);
        return r;
    };
    auto consider_rows = [&](std::vector<std::vector<int64_t>> &&bx, const std::vector<double> &w, int64_t ent) {
        const double t = model(w);
        if (t < best_t * 0.999 || (t <= best_t * 1.001 && ent < best_ent)) {
            best_t = t;
            best_ent = ent;
            // (dispatch order: the heaviest brick first)
            std::vector<int> ord(bx.size());
            for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return w[a] > w[b]; });
            best.clear();
            for (int k : ord) best.push_back(std::move(bx[k]));
        }
    };
    auto consider = [&](const std::vector<Box> &bx, const std::vector<double> &w, int64_t ent) {
        const double t = model(w);
        if (t < best_t * 0.999 || (t <= best_t * 1.001 && ent < best_ent)) {
            std::vector<std::vector<int64_t>> r;
            for (const Box &B : bx) r.push_back(box_rows(B));
            consider_rows(std::move(r), w, ent);
        }
    };
    // the region of a row set: the bounding box of its rows' reach
    auto row_region = [&](const std::vector<int64_t> &rows, int &ox, int &RX, int &oy, int &RY, int &oz, int &RZ) {
        int x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN, z0 = INT_MAX, z1 = INT_MIN;
        for (int64_t i : rows) {
            const int z = (int)(i / Lxy), y = (int)((i % Lxy) / Lx), x = (int)(i % Lx);
            x0 = std::min(x0, x), x1 = std::max(x1, x + 1);
            y0 = std::min(y0, y), y1 = std::max(y1, y + 1);
            z0 = std::min(z0, z), z1 = std::max(z1, z + 1);
        }
        region(xlo, xhi, x0, x1, ox, RX);
        region(ylo, yhi, y0, y1, oy, RY);
        region(zlo_none, zhi, z0, z1, oz, RZ);
    };
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
    for (int bpc = 1; bpc <= std::max(1, rounds); ++bpc) {
        const int nmax = nfix > 0 ? nfix : bpc * ncu;
    for (int nbz = 1; nbz <= std::min(ez, nmax); ++nbz)
        for (int nby = 1; nby <= std::min(ey, nmax / nbz); ++nby)
            for (int nbx = 1; nbx <= std::min(ex, nmax / (nbz * nby)); ++nbx) {
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
                            std::vector<Box> bx;
                            for (int e = 0; e < nbz; ++e)
                                for (int c = 0; c < nby; ++c)
                                    for (int a = 0; a < nbx; ++a)
                                        bx.push_back({cx[a], cx[a + 1], cy[c], cy[c + 1], cz[e], cz[e + 1]});
                            consider(bx, w, ent);
                        }
            }
    // Per-slab grids: z slabs of one or two element layers, each with its own
    // nbx x nby grid and cuts, the CUs allotted to the slabs by weight (the
    // Dirichlet top and bottom layers of a box carry 0.66 / 0.71 of an
    // interior layer's bytes, the x / y face columns 0.91-0.93: one tensor
    // grid leaves those CUs idle early).  Per slab, the best max brick weight
    // for every brick count; then greedily more bricks to the slab whose
    // largest brick is the largest, while the total stays <= nmax.
    if (fs == 0) {
        for (int t = 1; t <= 2; ++t) {
            const int ns = std::max(1, ez / t);
            std::vector<int> cz;
            if (!split_axis(uz, ns, P, cz)) continue;
            struct Opt {
                double m = 1e300;
                int64_t ent = 0;
                std::vector<int> cx, cy;
            };
            std::vector<std::vector<Opt>> opt(ns, std::vector<Opt>(nmax + 1));
            bool ok = true;
            for (int sl = 0; sl < ns && ok; ++sl) {
                const int z0 = cz[sl], z1 = cz[sl + 1];
                int o, RZ;
                region(zlo_none, zhi, z0, z1, o, RZ);
                std::vector<double> sx(Lx), sy(Ly);
                for (int xx = 0; xx < Lx; ++xx) sx[xx] = box_sum(xx, xx + 1, 0, Ly, z0, z1);
                for (int yy = 0; yy < Ly; ++yy) sy[yy] = box_sum(0, Lx, yy, yy + 1, z0, z1);
                const std::vector<Var> wvx = {{&sx, P}, {&sx, 1}, {&ux, P}}, wvy = {{&sy, P}, {&sy, 1}, {&uy, P}};
                for (int nby = 1; nby <= std::min(ey, nmax); ++nby)
                    for (int nbx = 1; nbx <= std::min(ex, nmax / nby); ++nbx)
                        for (const Var &VX : wvx)
                            for (const Var &VY : wvy) {
                                std::vector<int> cx, cy;
                                if (!split_axis(*VX.w, nbx, VX.q, cx) || !split_axis(*VY.w, nby, VY.q, cy)) continue;
                                std::vector<int> RXs(nbx), RYs(nby);
                                for (int a = 0; a < nbx; ++a) region(xlo, xhi, cx[a], cx[a + 1], o, RXs[a]);
                                for (int a = 0; a < nby; ++a) region(ylo, yhi, cy[a], cy[a + 1], o, RYs[a]);
                                double m = 0.0;
                                int64_t ent = 0;
                                bool fits = true;
                                for (int c = 0; c < nby && fits; ++c)
                                    for (int a = 0; a < nbx && fits; ++a) {
                                        const int RN = RXs[a] * RYs[c] * RZ;
                                        if (RN > 65535 || brick_lds(RN) > BRICK_LDS_CAP) fits = false;
                                        ent += RN;
                                        m = std::max(m, box_sum(cx[a], cx[a + 1], cy[c], cy[c + 1], z0, z1) + 72.0 * RN);
                                    }
                                Opt &O = opt[sl][nbx * nby];
                                if (fits && (m < O.m * 0.999 || (m <= O.m * 1.001 && ent < O.ent))) {
                                    O.m = m;
                                    O.ent = ent;
                                    O.cx = cx;
                                    O.cy = cy;
                                }
                            }
                // (prefix minima: the best plan with at most n bricks)
                int first = -1;
                for (int k = 1; k <= nmax; ++k) {
                    if (first < 0 && opt[sl][k].m < 1e300) first = k;
                    if (k > 1 && opt[sl][k - 1].m < opt[sl][k].m) opt[sl][k] = opt[sl][k - 1];
                }
                if (first < 0) ok = false;
            }
            if (!ok) continue;
            std::vector<int> cnt_s(ns);
            int tot = 0;
            for (int sl = 0; sl < ns; ++sl) {
                int k = 1;
                while (opt[sl][k].m >= 1e300) ++k;
                cnt_s[sl] = k;
                tot += k;
            }
            if (tot > nmax) continue;
            for (;;) {
                int worst = 0;
                for (int sl = 1; sl < ns; ++sl)
                    if (opt[sl][cnt_s[sl]].m > opt[worst][cnt_s[worst]].m) worst = sl;
                int k = cnt_s[worst] + 1;
                while (k <= nmax && opt[worst][k].m >= opt[worst][cnt_s[worst]].m * 0.9999) ++k;
                if (k > nmax || tot + k - cnt_s[worst] > nmax) break;
                tot += k - cnt_s[worst];
                cnt_s[worst] = k;
            }
            std::vector<Box> bx;
            std::vector<double> w;
            int64_t ent = 0;
            for (int sl = 0; sl < ns; ++sl) {
                const Opt &O = opt[sl][cnt_s[sl]];
                int o, RZ;
                region(zlo_none, zhi, cz[sl], cz[sl + 1], o, RZ);
                for (size_t c = 0; c + 1 < O.cy.size(); ++c)
                    for (size_t a = 0; a + 1 < O.cx.size(); ++a) {
                        int RX, RY;
                        region(xlo, xhi, O.cx[a], O.cx[a + 1], o, RX);
                        region(ylo, yhi, O.cy[c], O.cy[c + 1], o, RY);
                        bx.push_back({O.cx[a], O.cx[a + 1], O.cy[c], O.cy[c + 1], cz[sl], cz[sl + 1]});
                        w.push_back(box_sum(O.cx[a], O.cx[a + 1], O.cy[c], O.cy[c + 1], cz[sl], cz[sl + 1]) +
                                    72.0 * RX * RY * RZ);
                        ent += (int64_t)RX * RY * RZ;
                    }
            }
            consider(bx, w, ent);
        }
    }
    // Recursive bisection inside z slabs of one or two element layers: each
    // slab gets bricks in proportion to its bytes (largest remainders), and a
    // rectangle of n bricks is cut across its longer side at the node that
    // splits its bytes n1 : n - n1 -- the face columns' light rows go to
    // wider bricks without widening the others.
    if (fs == 0) {
        for (int t = 1; t <= 2; ++t) {
            const int ns = std::max(1, ez / t);
            std::vector<int> cz;
            if (!split_axis(uz, ns, P, cz) || ns > nmax) continue;
            const double W = box_sum(0, Lx, 0, Ly, 0, Lz);
            std::vector<int> nsl(ns);
            std::vector<std::pair<double, int>> rem;
            int tot = 0;
            for (int sl = 0; sl < ns; ++sl) {
                const double q = box_sum(0, Lx, 0, Ly, cz[sl], cz[sl + 1]) / W * nmax;
                nsl[sl] = std::max(1, (int)q);
                tot += nsl[sl];
                rem.push_back({q - (int)q, sl});
            }
            std::sort(rem.rbegin(), rem.rend());
            for (size_t k = 0; k < rem.size() && tot < nmax; ++k, ++tot) ++nsl[rem[k].second];
            if (tot > nmax) continue;
            std::vector<Box> bx;
            std::function<void(int, int, int, int, int, int, int)> cut = [&](int x0, int x1, int y0, int y1, int z0,
                                                                            int z1, int nb) {
                // (both halves keep at least an element along the cut side)
                const bool cx_ok = x1 - x0 >= 2 * P, cy_ok = y1 - y0 >= 2 * P;
                if (nb <= 1 || (!cx_ok && !cy_ok)) {
                    bx.push_back({x0, x1, y0, y1, z0, z1});
                    return;
                }
                const int n1 = nb / 2;
                const double target = box_sum(x0, x1, y0, y1, z0, z1) * n1 / nb;
                const bool alongx = cx_ok && (!cy_ok || x1 - x0 >= y1 - y0);
                const int lo = alongx ? x0 : y0, hi = alongx ? x1 : y1;
                int bestc = lo + P;
                double bestd = 1e300;
                for (int c = lo + P; c <= hi - P; ++c) {
                    const double wl = alongx ? box_sum(x0, c, y0, y1, z0, z1) : box_sum(x0, x1, y0, c, z0, z1);
                    if (std::fabs(wl - target) < bestd) {
                        bestd = std::fabs(wl - target);
                        bestc = c;
                    }
                }
                if (alongx) {
                    cut(x0, bestc, y0, y1, z0, z1, n1);
                    cut(bestc, x1, y0, y1, z0, z1, nb - n1);
                } else {
                    cut(x0, x1, y0, bestc, z0, z1, n1);
                    cut(x0, x1, bestc, y1, z0, z1, nb - n1);
                }
            };
            for (int sl = 0; sl < ns; ++sl) cut(0, Lx, 0, Ly, cz[sl], cz[sl + 1], nsl[sl]);
            std::vector<double> w;
            int64_t ent = 0;
            bool fits = true;
            for (const Box &B : bx) {
                int o, RX, RY, RZ;
                region(xlo, xhi, B.x0, B.x1, o, RX);
                region(ylo, yhi, B.y0, B.y1, o, RY);
                region(zlo_none, zhi, B.z0, B.z1, o, RZ);
                const int RN = RX * RY * RZ;
                if (RN > 65535 || brick_lds(RN) > BRICK_LDS_CAP) fits = false;
                ent += RN;
                w.push_back(box_sum(B.x0, B.x1, B.y0, B.y1, B.z0, B.z1) + 72.0 * RN);
            }
            if (getenv("KLE_BRICK_DEBUG")) {
                double mx = 0, sm = 0;
                for (double v : w) mx = std::max(mx, v), sm += v;
                fprintf(stderr, "bisect t=%d bricks %zu fits %d max/mean %.4f model %.1f\n", t, bx.size(), (int)fits,
                        mx / (sm / w.size()), model(w) * 1e-6);
            }
            if (fits) consider(bx, w, ent);
        }
    }
        if (nfix > 0) break;
    }
    bp.model_us = best_t * 1e-6;  // (bytes / (TB/s) = us)
    (void)total;
    if (best.empty()) return "no brick decomposition fits the LDS";
    // Rows of one stored block (the diagonal: Dirichlet rows and the free rows
    // at the far corner of their box) leave the bricks (bp.singles): a 64-lane
    // item would carry one block, and the gather forms B_ii x_i for them
    // instead (28,675 of 342,225 rows at config 2: 4.3 % of the items, 0.09 %
    // of the blocks).  Their values follow the bricks', 9 doubles each.
    bp.srows.clear();
    if (bp.singles) {
        std::vector<std::vector<int64_t>> kept;
        for (std::vector<int64_t> &R : best) {
            std::vector<int64_t> m;
            m.reserve(R.size());
            for (int64_t i : R) {
                if (i < 0 || i >= n) return "bricks overlap or leave the lattice";
                (mu[i] == 1 ? bp.srows : m).push_back(i);
            }
            if (!m.empty()) kept.push_back(std::move(m));  // (a brick of one-block rows only: none left)
        }
        best.swap(kept);
        std::sort(bp.srows.begin(), bp.srows.end());
    }
    const int NB = (int)best.size();
    bp.bricks.assign(NB, BrickDesc{});
    bp.rowd.assign(4 * n, 0);  // (units of two rows: a row and its partner or a null row)
    bp.svb.assign(n + 1, 0);
    int64_t voff = 0, rows = 0, wsd = 0, nreal = 0;
    bp.lds = 0;
    bp.ws_entries = 0;
    std::vector<char> seen(n, 0);
    for (int q = 0; q < NB; ++q) {
        const std::vector<int64_t> &R = best[q];
        for (int64_t i : R) {  // (each row in exactly one brick, checked before anything is written)
            if (i < 0 || i >= n || seen[i]) return "bricks overlap or leave the lattice";
            seen[i] = 1;
        }
        BrickDesc &D = bp.bricks[q];
        row_region(R, D.ox, D.RX, D.oy, D.RY, D.oz, D.RZ);
        // (the rows' bounding box, informational)
        int x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN, z0 = INT_MAX, z1 = INT_MIN;
        for (int64_t i : R) {
            const int z = (int)(i / Lxy), y = (int)((i % Lxy) / Lx), x = (int)(i % Lx);
            x0 = std::min(x0, x), x1 = std::max(x1, x + 1);
            y0 = std::min(y0, y), y1 = std::max(y1, y + 1);
            z0 = std::min(z0, z), z1 = std::max(z1, z + 1);
        }
        D.x0 = x0;
        D.nx = x1 - x0;
        D.y0 = y0;
        D.ny = y1 - y0;
        D.z0 = z0;
        D.nz = z1 - z0;
        // Units of two rows (bp.pair): row B's last partial pass shares row
        // A's (tails tA + tB <= 64 -- one 64-lane item instead of two: 22 %
        // fewer items at config 2), the unit streamed as A's full passes, the
        // shared item, B's full passes; B's values follow A's.  A row without
        // a partner takes a null descriptor as its B.  Pairs by two pointers
        // over the tails (the largest with the smallest that fits); units in
        // the lattice order of their first row.
        std::vector<std::pair<int64_t, int64_t>> units;
        {
            std::vector<int64_t> tl;
            for (int64_t i : R)
                if (bp.pair && mu[i] % 64 != 0) tl.push_back(i);
                else units.push_back({i, -1});
            std::stable_sort(tl.begin(), tl.end(), [&](int64_t a, int64_t b) { return mu[a] % 64 < mu[b] % 64; });
            size_t lo = 0, hi = tl.size();
            while (lo < hi) {
                const int64_t big = tl[hi - 1];
                if (lo + 1 < hi && mu[tl[lo]] % 64 + mu[big] % 64 <= 64) {
                    units.push_back({std::min(big, tl[lo]), std::max(big, tl[lo])});
                    ++lo;
                } else {
                    units.push_back({big, -1});
                }
                --hi;
            }
            std::sort(units.begin(), units.end());
        }
        D.nr = 2 * (int)units.size();
        const int RN = D.RX * D.RY * D.RZ;
        D.rstart = (int)rows;
        D.eb = 0;
        D.vbase = voff;
        D.wsoff = wsd;
        wsd += ((int64_t)3 * RN + 15) & ~int64_t(15);
        bp.lds = std::max(bp.lds, brick_lds(RN));
        for (const auto &u : units)
            for (int64_t i : {u.first, u.second}) {
                if (i < 0) {  // (no partner: the null descriptor)
                    bp.rowd[2 * rows] = 0;
                    bp.rowd[2 * rows + 1] = BRICK_ROW_NULL;
                    ++rows;
                    continue;
                }
                const int z = (int)(i / Lxy), y = (int)((i % Lxy) / Lx), x = (int)(i % Lx);
                bp.svb[i] = voff;
                const int64_t o = voff - D.vbase;
                if ((o >> 4) >= (1 << 23)) return "brick values beyond 2^27 doubles";
                const int ir = (x - D.ox) + D.RX * ((y - D.oy) + D.RY * (z - D.oz));
                bp.rowd[2 * rows] = (srow[i] & 0xFFFFFF) | ((ir & 255) << 24);
                bp.rowd[2 * rows + 1] = (int)((o >> 4) | ((int64_t)((ir >> 8) & 255) << 24));
                voff += ((int64_t)mu[i] * 9 + 15) & ~int64_t(15);
                ++rows;
                ++nreal;
            }
        // lattice entries of the region (written by the brick, read by the gather)
        for (int z = D.oz; z < D.oz + D.RZ; ++z)
            for (int y = D.oy; y < D.oy + D.RY; ++y)
                for (int x = D.ox; x < D.ox + D.RX; ++x)
                    bp.ws_entries += x >= 0 && x < Lx && y >= 0 && y < Ly && z >= 0 && z < Lz + hp;
    }
    for (size_t k = 0; k < bp.srows.size(); ++k) {
        const int64_t i = bp.srows[k];
        if (seen[i]) return "bricks overlap or leave the lattice";
        seen[i] = 1;
        bp.svb[i] = voff;
        voff += 9;
    }
    voff = (voff + 15) & ~int64_t(15);
    if (nreal + (int64_t)bp.srows.size() != n) return "bricks do not cover the lattice";
    bp.svb[n] = voff;
    bp.ws_doubles = wsd;
    bp.lds = std::max(bp.lds, BRICK_LDS_MIN);
    return "";
}

// The plan's tables against what k_nb_spmv_sym_brick derives from them:
// units of two rows (the second may be null), every real row's box, first
// block k0 < its box's size (mu >= 1 stored blocks), region index inside the
// brick's region and its lattice node inside the owned lattice, its values
// [off 16, off 16 + 9 mu) inside the value array, a unit's second row's
// values after its first's; regions within the LDS.  nullptr: consistent.
const char *brick_validate(const BrickPlan &bp, int64_t Lx, int64_t Ly, int64_t Lz, int64_t nvals,
                                  int64_t lds_cap)
{
    for (const BrickDesc &D : bp.bricks) {
        const int64_t RN = (int64_t)D.RX * D.RY * D.RZ;
        if (D.nr < 2 || D.nr % 2 || RN < 1 || RN > 65535) return "a brick's rows or region";
        if ((int64_t)brick_lds((int)RN) > std::min<int64_t>(lds_cap, (int64_t)BRICK_LDS_CAP))
            return "a brick's region exceeds the LDS";
        if (D.rstart < 0 || 2 * ((int64_t)D.rstart + D.nr) > (int64_t)bp.rowd.size()) return "a brick's rows";
        int64_t a_v0 = 0;
        for (int r = 0; r < D.nr; ++r) {
            const int64_t rr = (int64_t)D.rstart + r;
            const int dw = bp.rowd[2 * rr], vw = bp.rowd[2 * rr + 1];
            if (vw & BRICK_ROW_NULL) {
                if (r % 2 == 0) return "a unit's first row is null";
                continue;
            }
            const int dbx = dw & 15, dby = (dw >> 4) & 15, dbz = (dw >> 8) & 15;
            const int bnx = (dw >> 12) & 15, bny = (dw >> 16) & 15, bnz = (dw >> 20) & 15;
            const int k0 = dbx + bnx * (dby + bny * dbz), mu = bnx * bny * bnz - k0;
            if (dbx >= bnx || dby >= bny || dbz >= bnz || mu < 1) return "a row's box";
            const int ir = brick_row_ir(bp.rowd.data(), rr);
            if (ir < 0 || ir >= RN) return "a row's region index";
            const int irz = ir / (D.RX * D.RY), irem = ir - irz * D.RX * D.RY, iry = irem / D.RX, irx = irem - iry * D.RX;
            const int64_t gx = D.ox + irx, gy = D.oy + iry, gz = D.oz + irz;
            if (gx < 0 || gx >= Lx || gy < 0 || gy >= Ly || gz < 0 || gz >= Lz) return "a row's lattice node";
            const int64_t v0 = D.vbase + (int64_t)(vw & (BRICK_ROW_NULL - 1)) * 16, v1 = v0 + 9 * (int64_t)mu;
            if (v0 < 0 || v1 > nvals) return "a row's values";
            if (r % 2 == 0) a_v0 = v0;
            else if (v0 < a_v0 || v0 - a_v0 > ((int64_t)1 << 26)) return "a unit's second row's values";
        }
    }
    return nullptr;
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
extern "C" int kle_brick_plan_box(int Lx, int Ly, int Lz, int p, int dirichlet, int ncu, int rounds, int split,
                                  int *info, double *stats)
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
                if (dirichlet == 1 && (x == 0 || y == 0 || z == 0 || x == Lx - 1 || y == Ly - 1 || z == Lz - 1)) {
                    bx = x, by = y, bz = z;
                    nx = ny = nz = 1;
                }
                const int64_t i = x + (int64_t)Lx * (y + (int64_t)Ly * z);
                cnt[i] = nx * ny * nz;
                srow[i] = (x - bx) | (y - by) << 4 | (z - bz) << 8 | nx << 12 | ny << 16 | nz << 20;
                blocks += cnt[i] - ((x - bx) + nx * ((y - by) + ny * (z - bz)));
            }
    BrickPlan bp;
    bp.singles = g_tune.spmv_brick_singles;
    bp.pair = g_tune.spmv_brick_pair;
    const std::string why = brick_plan(Lx, Ly, Lz, 0, ncu, 0, rounds, split, cnt, srow, p, bp);
    if (!why.empty()) return fail(KLE_ERR_SUP, "%s", why.c_str());
    const int NB = (int)bp.bricks.size();
    // every row decodes (descriptor region index -> node) to a distinct node
    // of the lattice, inside its brick's region (what brick_finish and the
    // kernel rely on)
    {
        std::vector<char> seen(n, 0);
        for (const BrickDesc &D : bp.bricks)
            for (int r = 0; r < D.nr; ++r) {
                if (brick_row_null(bp.rowd.data(), (int64_t)D.rstart + r)) {
                    if (r % 2 == 0) return fail(KLE_ERR_SUP, "brick plan: a unit without its first row");
                    continue;
                }
                const int ir = brick_row_ir(bp.rowd.data(), (int64_t)D.rstart + r);
                if (ir < 0 || ir >= D.RX * D.RY * D.RZ) return fail(KLE_ERR_SUP, "brick plan: region index out of range");
                const int64_t i = brick_ir_node(D, ir, Lx, Ly);
                if (i < 0 || i >= n || seen[i]) return fail(KLE_ERR_SUP, "brick plan: row %lld decodes badly", (long long)i);
                seen[i] = 1;
            }
    }
    double tot = 0.0, mx = 0.0;
    // a brick's weight: its rows' costs (the rows from its descriptors)
    auto weight = [&](const BrickDesc &D) {
        double w = 0.0;
        for (int r = 0; r < D.nr; ++r) {
            if (brick_row_null(bp.rowd.data(), (int64_t)D.rstart + r)) continue;
            const int64_t i = brick_ir_node(D, brick_row_ir(bp.rowd.data(), (int64_t)D.rstart + r), Lx, Ly);
            const int d = srow[i];
            const int k0 = (d & 15) + ((d >> 12) & 15) * (((d >> 4) & 15) + ((d >> 16) & 15) * ((d >> 8) & 15));
            w += row_cost(cnt[i] - k0);
        }
        return w;
    };
    for (const BrickDesc &D : bp.bricks) {
        const double w = weight(D);
        tot += w;
        mx = std::max(mx, w);
    }
    // (bricks along each axis: distinct first coordinates)
    std::vector<int> ux, uy, uz;
    for (const BrickDesc &D : bp.bricks) {
        ux.push_back(D.x0);
        uy.push_back(D.y0);
        uz.push_back(D.z0);
    }
    auto distinct = [](std::vector<int> &v) {
        std::sort(v.begin(), v.end());
        return (int)(std::unique(v.begin(), v.end()) - v.begin());
    };
    const int cx = distinct(ux), cy = distinct(uy), cz = distinct(uz);
    info[0] = NB;
    info[1] = cx;
    info[2] = cy;
    info[3] = cz;
    info[4] = (int)bp.lds;
    stats[0] = NB ? mx / (tot / NB) : 0.0;
    stats[1] = (double)bp.ws_entries / n;
    stats[2] = (double)blocks;
    stats[3] = bp.model_us;
    // the items the bricks stream (a unit of two rows: their full passes and
    // one shared item) and the share of their lanes that carry a block
    {
        auto rmu = [&](int64_t r) {
            const int d = bp.rowd[2 * r];
            const int dbx = d & 15, dby = (d >> 4) & 15, dbz = (d >> 8) & 15;
            const int bnx = (d >> 12) & 15, bny = (d >> 16) & 15, bnz = (d >> 20) & 15;
            return bnx * bny * bnz - (dbx + bnx * (dby + bny * dbz));
        };
        int64_t items = 0, blocks_b = 0;
        for (const BrickDesc &D : bp.bricks)
            for (int u = 0; u < D.nr / 2; ++u) {
                const int64_t ra = (int64_t)D.rstart + 2 * u, rb = ra + 1;
                const int ma = rmu(ra);
                blocks_b += ma;
                if (brick_row_null(bp.rowd.data(), rb)) {
                    items += (ma + 63) / 64;
                } else {
                    const int mb = rmu(rb);
                    blocks_b += mb;
                    if (ma % 64 == 0 || mb % 64 == 0 || ma % 64 + mb % 64 > 64)
                        return fail(KLE_ERR_SUP, "brick plan: a unit whose tails do not share an item");
                    items += ma / 64 + mb / 64 + 1;
                }
            }
        stats[4] = (double)items;
        stats[5] = items ? (double)blocks_b / (64.0 * (double)items) : 0.0;
    }
    {
        // (the tables checked as brick_finish checks them on the device path;
        // the values: the plan's own layout)
        if (const char *bad = brick_validate(bp, Lx, Ly, Lz, bp.svb[n], (int64_t)bp.lds))
            return fail(KLE_ERR_SUP, "brick plan: %s", bad);
    }
    if (getenv("KLE_BRICK_DEBUG"))
        for (const BrickDesc &D : bp.bricks) {
            // (stored blocks, rows of one stored block, rows past one 64-block pass)
            long long sb = 0;
            int one = 0, two = 0;
            for (int r = 0; r < D.nr; ++r) {
                if (brick_row_null(bp.rowd.data(), (int64_t)D.rstart + r)) continue;
                const int64_t i = brick_ir_node(D, brick_row_ir(bp.rowd.data(), (int64_t)D.rstart + r), Lx, Ly);
                const int d = srow[i];
                const int k0 = (d & 15) + ((d >> 12) & 15) * (((d >> 4) & 15) + ((d >> 16) & 15) * ((d >> 8) & 15));
                const int mu = cnt[i] - k0;
                sb += mu;
                one += mu == 1;
                two += mu > 64;
            }
            fprintf(stderr, "brick %d %d %d  %d %d %d  rows %d  region %d %d %d  w %.4f  blocks %lld  one %d  multi %d\n",
                    D.x0, D.y0, D.z0, D.nx, D.ny, D.nz, D.nr, D.RX, D.RY, D.RZ, weight(D) / (tot / NB), sb, one, two);
        }
    return 0;
}
