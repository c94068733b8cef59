// kle_basis.cpp -- see kle_basis.hpp.
#include "kle_basis.hpp"

#include <cmath>

namespace kle {

// Legendre P_n and P_n' at x by the three-term recurrence.
static void legendre(int n, double x, double &p, double &dp, double &pm1)
{
    double p0 = 1.0, p1 = x;
    if (n == 0) {
        p = 1.0;
        dp = 0.0;
        pm1 = 0.0;
        return;
    }
    for (int k = 2; k <= n; ++k) {
        double pk = ((2.0 * k - 1.0) * x * p1 - (k - 1.0) * p0) / k;
        p0 = p1;
        p1 = pk;
    }
    p = p1;
    pm1 = p0;
    dp = (std::fabs(x) < 1.0) ? n * (p0 - x * p1) / (1.0 - x * x) : 0.5 * n * (n + 1) * std::pow(x, n - 1);
}

void gauss_legendre(int n, std::vector<double> &x, std::vector<double> &w)
{
    x.assign(n, 0.0);
    w.assign(n, 0.0);
    for (int i = 0; i < n; ++i) {
        // Chebyshev-like initial guess, i-th root from the left
        double z = -std::cos(M_PI * (i + 0.75) / (n + 0.5));
        for (int it = 0; it < 100; ++it) {
            double p, dp, pm1;
            legendre(n, z, p, dp, pm1);
            double dz = p / dp;
            z -= dz;
            if (std::fabs(dz) < 1e-17) break;
        }
        double p, dp, pm1;
        legendre(n, z, p, dp, pm1);
        x[i] = z;
        w[i] = 2.0 / ((1.0 - z * z) * dp * dp);
    }
    // exact symmetry (the reference symmetrises too, utilities.py:59-60)
    for (int i = 0; i < n / 2; ++i) {
        double a = 0.5 * (x[n - 1 - i] - x[i]), b = 0.5 * (w[i] + w[n - 1 - i]);
        x[i] = -a;
        x[n - 1 - i] = a;
        w[i] = w[n - 1 - i] = b;
    }
    if (n % 2) x[n / 2] = 0.0;
}

void gauss_lobatto(int n, std::vector<double> &x, std::vector<double> &w)
{
    x.assign(n, 0.0);
    w.assign(n, 0.0);
    int N = n - 1;
    for (int i = 0; i < n; ++i) {
        double z = -std::cos(M_PI * i / N);
        if (i > 0 && i < N) {
            // interior nodes are the roots of P_N'; Newton on q = P_N'
            for (int it = 0; it < 100; ++it) {
                double p, dp, pm1;
                legendre(N, z, p, dp, pm1);
                // P_N'' from the Legendre ODE: (1-z^2) P'' = 2 z P' - N(N+1) P
                double d2 = (2.0 * z * dp - N * (N + 1.0) * p) / (1.0 - z * z);
                double dz = dp / d2;
                z -= dz;
                if (std::fabs(dz) < 1e-17) break;
            }
        }
        double p, dp, pm1;
        legendre(N, z, p, dp, pm1);
        x[i] = z;
        w[i] = 2.0 / (N * (N + 1.0) * p * p);
    }
    for (int i = 0; i < n / 2; ++i) {
        double a = 0.5 * (x[n - 1 - i] - x[i]), b = 0.5 * (w[i] + w[n - 1 - i]);
        x[i] = -a;
        x[n - 1 - i] = a;
        w[i] = w[n - 1 - i] = b;
    }
    if (n % 2) x[n / 2] = 0.0;
}

void lagrange(const std::vector<double> &nodes, const std::vector<double> &pts, std::vector<double> &h,
              std::vector<double> &dh)
{
    const int nn = (int)nodes.size(), np = (int)pts.size();
    h.assign((size_t)np * nn, 0.0);
    dh.assign((size_t)np * nn, 0.0);
    for (int q = 0; q < np; ++q)
        for (int a = 0; a < nn; ++a) {
            double den = 1.0, num = 1.0;
            for (int j = 0; j < nn; ++j)
                if (j != a) {
                    den *= nodes[a] - nodes[j];
                    num *= pts[q] - nodes[j];
                }
            double d = 0.0;
            for (int k = 0; k < nn; ++k) {
                if (k == a) continue;
                double t = 1.0;
                for (int j = 0; j < nn; ++j)
                    if (j != a && j != k) t *= pts[q] - nodes[j];
                d += t;
            }
            h[(size_t)q * nn + a] = num / den;
            dh[(size_t)q * nn + a] = d / den;
        }
}

void element_sets(int ngl, PointSet1D &full, PointSet1D &red, PointSet1D &op)
{
    std::vector<double> nodes, nw;
    gauss_lobatto(ngl, nodes, nw);
    if (ngl > 3) {
        full.x = nodes;
        full.w = nw;
    } else {
        gauss_legendre(ngl, full.x, full.w);
    }
    gauss_legendre(ngl - 1, red.x, red.w);
    op.x = nodes;
    op.w = nw;
    lagrange(nodes, full.x, full.h, full.dh);
    lagrange(nodes, red.x, red.h, red.dh);
    lagrange(nodes, op.x, op.h, op.dh);
}

}  // namespace kle
