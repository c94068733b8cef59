// kle_basis.hpp -- 1-D quadrature and Lagrange tables (host, setup only).
//
// Product-side counterpart of utilities.py:43-92 (gaussPoints, lobattoPoints)
// and element.py:13-45 (interpFun1D).  Computed once per (ngl) on the host
// and uploaded; the per-element work runs on the GPU (kle_assemble.hip).
#pragma once
#include <vector>

namespace kle {

// Gauss-Legendre nodes/weights on [-1,1], ascending (Newton on P_n).
void gauss_legendre(int n, std::vector<double> &x, std::vector<double> &w);
// Gauss-Lobatto-Legendre nodes/weights on [-1,1], ascending.
void gauss_lobatto(int n, std::vector<double> &x, std::vector<double> &w);
// Lagrange basis of `nodes` and its derivative at `pts`: h[q*nn + a].
void lagrange(const std::vector<double> &nodes, const std::vector<double> &pts,
              std::vector<double> &h, std::vector<double> &dh);

// Point sets of the spectral element (spectral.py:67-90):
//   full: GLL(ngl) if ngl > 3 else Gauss(ngl)   (stiffness, Rw, Rd)
//   red : Gauss(ngl-1)                          (div / curl penalties)
//   op  : GLL(ngl)                              (collocation operators)
struct PointSet1D {
    std::vector<double> x, w;  // 1-D points and weights
    std::vector<double> h, dh; // Lagrange basis of the GLL nodes at x: [q][a]
};
void element_sets(int ngl, PointSet1D &full, PointSet1D &red, PointSet1D &op);

}  // namespace kle
