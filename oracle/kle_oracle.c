/*
 * kle_oracle.c -- CPU restatement of Pynama's KLE assembly + Krylov hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it;
 * the product (pynama_amd/, libkle.so) never links, calls or falls back to it.
 *
 * Pinned against golden vectors produced by the reference's own Python code
 * (tests/golden/make_golden.py -> tests/golden/ fixtures); see tests/test_oracle.py.
 *
 * Every routine cites the reference file:line (paths under /root/reference/src)
 * whose behaviour it restates.  Arithmetic is fp64 throughout.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_MAXN 16

/* ------------------------------------------------------------------------ */
/* a1: quadrature                                                            */
/* ------------------------------------------------------------------------ */

/* Cyclic Jacobi eigen-solver for a small symmetric matrix (row-major n x n).
 * On exit a holds the eigenvalues on its diagonal, v the eigenvectors in its
 * columns.  Stand-in for numpy.linalg.eig in gaussPoints (utilities.py:54). */
static void jacobi_eig(int n, double *a, double *v)
{
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) v[i * n + j] = (i == j);
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0;
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) off += a[i * n + j] * a[i * n + j];
        if (off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                double apq = a[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                double theta = (a[q * n + q] - a[p * n + p]) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                double c = 1 / sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; ++k) { /* rows/cols r != p,q */
                    if (k == p || k == q) continue;
                    double akp = a[k * n + p], akq = a[k * n + q];
                    a[k * n + p] = a[p * n + k] = c * akp - s * akq;
                    a[k * n + q] = a[q * n + k] = s * akp + c * akq;
                }
                a[p * n + p] -= t * apq;
                a[q * n + q] += t * apq;
                a[p * n + q] = a[q * n + p] = 0;
                for (int k = 0; k < n; ++k) {
                    double vkp = v[k * n + p], vkq = v[k * n + q];
                    v[k * n + p] = c * vkp - s * vkq;
                    v[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

/* gaussPoints (utilities.py:43-61): Golub-Welsch + symmetrisation. */
int orc_gauss(int n, double *x, double *w)
{
    if (n < 1 || n > ORC_MAXN) return -1;
    double a[ORC_MAXN * ORC_MAXN] = {0}, v[ORC_MAXN * ORC_MAXN];
    for (int i = 1; i < n; ++i) {
        double b = 0.5 / sqrt(1.0 - pow(2.0 * i, -2.0));
        a[(i - 1) * n + i] = b;
        a[i * n + i - 1] = b;
    }
    jacobi_eig(n, a, v);
    int idx[ORC_MAXN];
    for (int i = 0; i < n; ++i) idx[i] = i;
    for (int i = 0; i < n; ++i) /* argsort of eigenvalues */
        for (int j = i + 1; j < n; ++j)
            if (a[idx[j] * n + idx[j]] < a[idx[i] * n + idx[i]]) {
                int t = idx[i]; idx[i] = idx[j]; idx[j] = t;
            }
    double xs[ORC_MAXN], ws[ORC_MAXN];
    for (int i = 0; i < n; ++i) {
        xs[i] = a[idx[i] * n + idx[i]];
        double v0 = v[0 * n + idx[i]], nrm = 0;
        for (int k = 0; k < n; ++k) nrm += v[k * n + idx[i]] * v[k * n + idx[i]];
        ws[i] = 2 * (v0 * v0 / nrm);
    }
    for (int i = 0; i < n; ++i) {
        x[i] = (xs[i] - xs[n - 1 - i]) / 2;
        w[i] = (ws[i] + ws[n - 1 - i]) / 2;
    }
    return 0;
}

/* lobattoPoints (utilities.py:63-92): Newton on Legendre from the
 * Chebyshev-Gauss-Lobatto guess, tolerance 1e-15. */
int orc_lobatto(int N, double *xo, double *wo)
{
    if (N < 2 || N > ORC_MAXN) return -1;
    double x[ORC_MAXN], xold[ORC_MAXN], P[ORC_MAXN][ORC_MAXN];
    for (int i = 0; i < N; ++i) {
        double step = M_PI / (N - 1); /* np.linspace(0, pi, N) */
        x[i] = cos(i == N - 1 ? M_PI : i * step);
        xold[i] = 2;
    }
    for (int it = 0; it < 1000; ++it) {
        double md = 0;
        for (int i = 0; i < N; ++i) md = fmax(md, fabs(x[i] - xold[i]));
        if (!(md > 1e-15)) break;
        for (int i = 0; i < N; ++i) {
            xold[i] = x[i];
            P[i][0] = 1;
            P[i][1] = x[i];
            for (int k = 2; k < N; ++k)
                P[i][k] = ((2 * k - 1) * x[i] * P[i][k - 1] - (k - 1) * P[i][k - 2]) / k;
            x[i] = xold[i] - (x[i] * P[i][N - 1] - P[i][N - 2]) / (N * P[i][N - 1]);
        }
    }
    double w[ORC_MAXN];
    for (int i = 0; i < N; ++i) w[i] = 2.0 / ((N - 1) * N * (P[i][N - 1] * P[i][N - 1]));
    for (int i = 0; i < N; ++i) {
        xo[i] = (x[N - 1 - i] - x[i]) / 2;
        wo[i] = (w[N - 1 - i] + w[i]) / 2;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* a3: local node order (DMPlex closure order of the spectral element)       */
/* ------------------------------------------------------------------------ */

/* Label of tensor node (a,b,c) (a along r, slowest) as built by
 * Spectral.getSpectralOrder (spectral.py:356-441): returns Permlst. */
static void spectral_labels3d(int n, int *perm)
{
    if (n == 1) { perm[0] = 0; return; }
    int m = n - 2;
    int *I = calloc((size_t)n * n * n, sizeof(int));
#define ID(x, y, z) I[((x) * n + (y)) * n + (z)]
    int L = n - 1;
    ID(0, 0, 0) = 8; ID(0, 0, L) = 7; ID(0, L, 0) = 5; ID(0, L, L) = 6;
    ID(L, 0, 0) = 2; ID(L, 0, L) = 3; ID(L, L, 0) = 1; ID(L, L, L) = 4;
    if (n > 2) {
        int e = 8;
        for (int t = 0; t < m; ++t) ID(L, 1 + t, 0) = e + m - t;          /* edge1 */
        e += n - 1;
        for (int t = 0; t < m; ++t) ID(L, 0, 1 + t) = e + t;              /* edge2 */
        e += n - 2;
        for (int t = 0; t < m; ++t) ID(L, 1 + t, L) = e + t;              /* edge3 */
        e += n - 3;
        for (int t = 0; t < m; ++t) ID(L, L, 1 + t) = e + m - t;          /* edge4 */
        e += n - 1;
        for (int t = 0; t < m; ++t) ID(0, L, 1 + t) = e + t;              /* edge5 */
        e += n - 3;
        for (int t = 0; t < m; ++t) ID(0, 1 + t, L) = e + m - t;          /* edge6 */
        e += n - 2;
        for (int t = 0; t < m; ++t) ID(0, 0, 1 + t) = e + m - t;          /* edge7 */
        e += n - 1;
        for (int t = 0; t < m; ++t) ID(0, 1 + t, 0) = e + t;              /* edge8 */
        e += n - 3;
        for (int t = 0; t < m; ++t) ID(1 + t, L, L) = e + m - t;          /* edge9 */
        e += n - 1;
        for (int t = 0; t < m; ++t) ID(1 + t, L, 0) = e + t;              /* edge10 */
        e += n - 3;
        for (int t = 0; t < m; ++t) ID(1 + t, 0, 0) = e + m - t;          /* edge11 */
        e += n - 1;
        for (int t = 0; t < m; ++t) ID(1 + t, 0, L) = e + t;              /* edge12 */
        int nf = m * m, v = e + n - 2;
        for (int u = 0; u < m; ++u)                                       /* face1 */
            for (int w = 0; w < m; ++w) ID(L, 1 + u, 1 + w) = v + u * m + w;
        v = v + nf - 1;
        for (int u = 0; u < m; ++u)                                       /* face2 */
            for (int w = 0; w < m; ++w) ID(0, 1 + u, 1 + w) = v + nf - (u * m + w);
        v = v + nf;
        for (int a = 0; a < m; ++a)                                       /* face3 */
            for (int c = 0; c < m; ++c) ID(1 + a, L, 1 + c) = v + nf - (c * m + a);
        v = v + nf + 1;
        for (int a = 0; a < m; ++a)                                       /* face4 */
            for (int c = 0; c < m; ++c) ID(1 + a, 0, 1 + c) = v + c * m + a;
        v = v + nf;
        for (int u = 0; u < m; ++u)                                       /* face5 */
            for (int w = 0; w < m; ++w) ID(1 + u, 1 + w, L) = v + u * m + w;
        v = v + nf - 1;
        for (int u = 0; u < m; ++u)                                       /* face6 */
            for (int w = 0; w < m; ++w) ID(1 + u, 1 + w, 0) = v + nf - (u * m + w);
        v = v + nf + 1;
        for (int u = 0; u < m; ++u)                                       /* body */
            for (int w = 0; w < m; ++w)
                for (int z = 0; z < m; ++z) ID(1 + u, 1 + w, 1 + z) = v + (u * m + w) * m + z;
    }
    /* Permlst[a n^2 + b n + c] = Ind3d[n-1-c][n-1-b][a] - 1 */
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b)
            for (int c = 0; c < n; ++c)
                perm[(a * n + b) * n + c] = ID(L - c, L - b, a) - 1;
#undef ID
    free(I);
}

/* Label of tensor node (a,b) in 2-D: computeMats2D (spectral.py:230-310). */
static void spectral_labels2d(int n, int *perm)
{
    if (n == 1) { perm[0] = 0; return; }
    int m = n - 2, L = n - 1;
    int *I = calloc((size_t)n * n, sizeof(int));
#define ID(x, y) I[(x) * n + (y)]
    ID(0, 0) = 2; ID(0, L) = 1; ID(L, 0) = 3; ID(L, L) = 4;
    if (n > 2) {
        for (int t = 0; t < m; ++t) ID(0, 1 + t) = n + 2 - t;
        for (int t = 0; t < m; ++t) ID(1 + t, 0) = n + 3 + t;
        for (int t = 0; t < m; ++t) ID(L, 1 + t) = 2 * n + 1 + t;
        for (int t = 0; t < m; ++t) ID(1 + t, L) = 4 * n - 4 - t;
        for (int u = 0; u < m; ++u)
            for (int v = 0; v < m; ++v) ID(1 + u, 1 + v) = 4 * n - 3 + v * m + u;
    }
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) perm[a * n + b] = ID(L - b, a) - 1;
#undef ID
    free(I);
}

static void labels(int dim, int n, int *perm)
{
    if (dim == 2) spectral_labels2d(n, perm);
    else spectral_labels3d(n, perm);
}

/* invPerm as returned by getSpectralOrder / computed in computeMats2D. */
int orc_spectral_order(int dim, int n, int *inv_perm)
{
    int cnt = dim == 2 ? n * n : n * n * n;
    int *perm = malloc(sizeof(int) * cnt);
    labels(dim, n, perm);
    for (int t = 0; t < cnt; ++t) inv_perm[perm[t]] = t;
    free(perm);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* a2/a3: basis tables                                                       */
/* ------------------------------------------------------------------------ */

/* Element.interpFun1D (element.py:13-45): Lagrange basis and derivative. */
static void interp1d(const double *nodes, int nn, const double *pts, int np_,
                     double *h, double *dh)
{
    for (int e = 0; e < np_; ++e) {
        double prodDen[ORC_MAXN], prodNum[ORC_MAXN], num3[ORC_MAXN];
        for (int i = 0; i < nn; ++i) {
            double pn = 1, pd = 1;
            for (int j = 0; j < nn; ++j) {
                pn *= (i == j) ? 1 : pts[e] - nodes[j];   /* Num  (element.py:27-29) */
                pd *= (i == j) ? 1 : -nodes[j] + nodes[i]; /* Den  (element.py:32-35) */
            }
            prodNum[i] = pn;
            prodDen[i] = pd;
            num3[i] = 0;
        }
        for (int col = 0; col < nn; ++col)
            for (int i = 0; i < nn; ++i) {
                double p = 1;
                for (int j = 0; j < nn; ++j) {
                    double v = (j == col) ? (i == j ? 0.0 : 1.0)
                                          : ((i == j) ? 1 : pts[e] - nodes[j]);
                    p *= v;
                }
                num3[i] += p;
            }
        for (int i = 0; i < nn; ++i) {
            h[e * nn + i] = prodNum[i] / prodDen[i];
            dh[e * nn + i] = num3[i] / prodDen[i];
        }
    }
}

typedef struct {
    int nq, nn;          /* points, nodes (tensor counts)             */
    double *H;           /* [nq][nn]                                  */
    double *Hrs;         /* [nq][dim][nn]                             */
    double *w;           /* [nq] weights                              */
    double *pt;          /* [nq][dim] point coords (r,s,t)            */
} orc_set;

typedef struct {
    int dim, ngl, nn;
    orc_set full, red, op, coo, cooRed, cooOp;
} orc_elem;

/* computeMats2D/3D (spectral.py:230-354) for one (nodes, points) pair. */
static void build_set(int dim, const double *nodes1d, int nn1, const double *pts1d,
                      const double *wei1d, int np1, orc_set *s)
{
    int nn = dim == 2 ? nn1 * nn1 : nn1 * nn1 * nn1;
    int nq = dim == 2 ? np1 * np1 : np1 * np1 * np1;
    s->nn = nn;
    s->nq = nq;
    s->H = calloc((size_t)nq * nn, sizeof(double));
    s->Hrs = calloc((size_t)nq * dim * nn, sizeof(double));
    s->w = calloc(nq, sizeof(double));
    s->pt = calloc((size_t)nq * dim, sizeof(double));
    double h[ORC_MAXN * ORC_MAXN], dh[ORC_MAXN * ORC_MAXN];
    interp1d(nodes1d, nn1, pts1d, np1, h, dh);
    int *nlab = malloc(sizeof(int) * nn), *qlab = malloc(sizeof(int) * nq);
    labels(dim, nn1, nlab);
    labels(dim, np1, qlab);
    for (int tq = 0; tq < nq; ++tq) {
        int q = qlab[tq];
        int i = dim == 2 ? tq / np1 : tq / (np1 * np1);
        int j = dim == 2 ? tq % np1 : (tq / np1) % np1;
        int k = tq % np1;
        if (dim == 2) {
            s->w[q] = wei1d[i] * wei1d[j];
            s->pt[q * 2] = pts1d[i];
            s->pt[q * 2 + 1] = pts1d[j];
        } else {
            s->w[q] = wei1d[i] * wei1d[j] * wei1d[k];
            s->pt[q * 3] = pts1d[i];
            s->pt[q * 3 + 1] = pts1d[j];
            s->pt[q * 3 + 2] = pts1d[k];
        }
        for (int tn = 0; tn < nn; ++tn) {
            int l = nlab[tn];
            if (dim == 2) {
                int a = tn / nn1, b = tn % nn1;
                s->H[q * nn + l] = (1.0 * h[i * nn1 + a]) * h[j * nn1 + b];
                s->Hrs[(q * 2 + 0) * nn + l] = (1.0 * dh[i * nn1 + a]) * h[j * nn1 + b];
                s->Hrs[(q * 2 + 1) * nn + l] = (1.0 * h[i * nn1 + a]) * dh[j * nn1 + b];
            } else {
                int a = tn / (nn1 * nn1), b = (tn / nn1) % nn1, c = tn % nn1;
                s->H[q * nn + l] = ((1.0 * h[i * nn1 + a]) * h[j * nn1 + b]) * h[k * nn1 + c];
                s->Hrs[(q * 3 + 0) * nn + l] = ((1.0 * dh[i * nn1 + a]) * h[j * nn1 + b]) * h[k * nn1 + c];
                s->Hrs[(q * 3 + 1) * nn + l] = ((1.0 * h[i * nn1 + a]) * dh[j * nn1 + b]) * h[k * nn1 + c];
                s->Hrs[(q * 3 + 2) * nn + l] = ((1.0 * h[i * nn1 + a]) * h[j * nn1 + b]) * dh[k * nn1 + c];
            }
        }
    }
    free(nlab);
    free(qlab);
}

static void free_set(orc_set *s)
{
    free(s->H); free(s->Hrs); free(s->w); free(s->pt);
}

/* Spectral.__init__ + setUpSpectralMats2D/3D (spectral.py:17-90). */
orc_elem *orc_elem_create(int dim, int ngl)
{
    if ((dim != 2 && dim != 3) || ngl < 2 || ngl > ORC_MAXN) return NULL;
    orc_elem *e = calloc(1, sizeof(orc_elem));
    e->dim = dim;
    e->ngl = ngl;
    e->nn = dim == 2 ? ngl * ngl : ngl * ngl * ngl;
    double nodes[ORC_MAXN], opw[ORC_MAXN], gps[ORC_MAXN], fw[ORC_MAXN], gr[ORC_MAXN],
        rw[ORC_MAXN], cn[2], cw[2];
    orc_lobatto(ngl, nodes, opw);
    if (ngl <= 3) orc_gauss(ngl, gps, fw);
    else orc_lobatto(ngl, gps, fw);
    orc_gauss(ngl - 1, gr, rw);
    orc_lobatto(2, cn, cw);
    build_set(dim, nodes, ngl, gps, fw, ngl, &e->full);
    build_set(dim, nodes, ngl, gr, rw, ngl - 1, &e->red);
    build_set(dim, nodes, ngl, nodes, opw, ngl, &e->op);
    build_set(dim, cn, 2, gps, fw, ngl, &e->coo);
    build_set(dim, cn, 2, gr, rw, ngl - 1, &e->cooRed);
    build_set(dim, cn, 2, nodes, opw, ngl, &e->cooOp);
    return e;
}

void orc_elem_destroy(orc_elem *e)
{
    if (!e) return;
    free_set(&e->full); free_set(&e->red); free_set(&e->op);
    free_set(&e->coo); free_set(&e->cooRed); free_set(&e->cooOp);
    free(e);
}

/* Export a table for the golden comparison.  which: 0 full,1 red,2 op,3 coo,
 * 4 cooRed, 5 cooOp ; what: 0 H, 1 Hrs, 2 weights, 3 points. */
int orc_elem_table(const orc_elem *e, int which, int what, double *out)
{
    const orc_set *s[] = {&e->full, &e->red, &e->op, &e->coo, &e->cooRed, &e->cooOp};
    if (which < 0 || which > 5) return -1;
    const orc_set *t = s[which];
    size_t n = what == 0 ? (size_t)t->nq * t->nn
             : what == 1 ? (size_t)t->nq * e->dim * t->nn
             : what == 2 ? (size_t)t->nq : (size_t)t->nq * e->dim;
    const double *src = what == 0 ? t->H : what == 1 ? t->Hrs : what == 2 ? t->w : t->pt;
    memcpy(out, src, n * sizeof(double));
    return (int)n;
}

int orc_elem_npoints(const orc_elem *e, int which)
{
    const orc_set *s[] = {&e->full, &e->red, &e->op, &e->coo, &e->cooRed, &e->cooOp};
    return s[which]->nq;
}

/* ------------------------------------------------------------------------ */
/* a4/a5: element matrices                                                   */
/* ------------------------------------------------------------------------ */

/* J = HrsCoo[q] . X ; Hxy = inv(J) . Hrs[q] ; det(J)  (spectral.py:117-120). */
static double geometry(int dim, const orc_set *coo, const orc_set *s, int q,
                       const double *X, double *Hxy)
{
    double J[9] = {0}, Ji[9];
    int nc = coo->nn;
    for (int i = 0; i < dim; ++i)
        for (int j = 0; j < dim; ++j) {
            double acc = 0;
            for (int c = 0; c < nc; ++c) acc += coo->Hrs[(q * dim + i) * nc + c] * X[c * dim + j];
            J[i * dim + j] = acc;
        }
    double det;
    if (dim == 2) {
        det = J[0] * J[3] - J[1] * J[2];
        Ji[0] = J[3] / det; Ji[1] = -J[1] / det;
        Ji[2] = -J[2] / det; Ji[3] = J[0] / det;
    } else {
        double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8],
               c02 = J[3] * J[7] - J[4] * J[6];
        det = J[0] * c00 + J[1] * c01 + J[2] * c02;
        Ji[0] = c00 / det;
        Ji[1] = (J[2] * J[7] - J[1] * J[8]) / det;
        Ji[2] = (J[1] * J[5] - J[2] * J[4]) / det;
        Ji[3] = c01 / det;
        Ji[4] = (J[0] * J[8] - J[2] * J[6]) / det;
        Ji[5] = (J[2] * J[3] - J[0] * J[5]) / det;
        Ji[6] = c02 / det;
        Ji[7] = (J[1] * J[6] - J[0] * J[7]) / det;
        Ji[8] = (J[0] * J[4] - J[1] * J[3]) / det;
    }
    int nn = s->nn;
    for (int i = 0; i < dim; ++i)
        for (int l = 0; l < nn; ++l) {
            double acc = 0;
            for (int k = 0; k < dim; ++k) acc += Ji[i * dim + k] * s->Hrs[(q * dim + k) * nn + l];
            Hxy[i * nn + l] = acc;
        }
    return det;
}

/* curl index tables (spectral.py:26-33): rows of B_curl / Bw_curl. */
static const int IND3[6][3] = {{0, 2, 1}, {0, 1, 2}, {1, 0, 2}, {1, 2, 0}, {2, 1, 0}, {2, 0, 1}};
static const int INDC2[2][3] = {{0, 1, 0}, {0, 0, 1}};  /* indCurl 2-D  */
static const int INDW2[2][3] = {{0, 0, 1}, {1, 0, 0}};  /* indWCurl 2-D */

/* Spectral.getElemKLEMatrices (spectral.py:92-160), written out entry-wise on
 * the sparse B matrices in the same per-Gauss-point accumulation order.
 * K [dim n][dim n], Rw [dim n][dim_w n], Rd [dim n][n], row-major. */
int orc_elem_kle(const orc_elem *e, const double *X, double *K, double *Rw, double *Rd)
{
    const int dim = e->dim, nn = e->nn, dw = dim == 2 ? 1 : 3;
    const double alpha_w = 1e2, alpha_d = 1e3;
    const int nd = dim * nn;
    memset(K, 0, sizeof(double) * nd * nd);
    memset(Rw, 0, sizeof(double) * nd * dw * nn);
    memset(Rd, 0, sizeof(double) * nd * nn);
    double *Hxy = malloc(sizeof(double) * 3 * nn);
    double *Bw = malloc(sizeof(double) * dim * dw * nn);   /* Bw_curl [dim][dw n] */
    double *Bc = malloc(sizeof(double) * dw * dim * nn);   /* B_curl  [dw][dim n] */
    const int (*iw)[3] = dim == 2 ? INDW2 : IND3;
    const int (*ic)[3] = dim == 2 ? INDC2 : IND3;
    const int nind = dim == 2 ? 2 : 6;
    for (int q = 0; q < e->full.nq; ++q) {
        double detJ = geometry(dim, &e->coo, &e->full, q, X, Hxy);
        double c = e->full.w[q] * detJ;
        const double *H = e->full.H + (size_t)q * nn;
        memset(Bw, 0, sizeof(double) * dim * dw * nn);
        for (int i = 0; i < nind; ++i) {
            double sg = (i & 1) ? -1.0 : 1.0;
            for (int l = 0; l < nn; ++l) Bw[iw[i][0] * dw * nn + l * dw + iw[i][1]] = sg * Hxy[iw[i][2] * nn + l];
        }
        for (int l = 0; l < nn; ++l)
            for (int m = 0; m < nn; ++m) {
                double g = 0;
                for (int i = 0; i < dim; ++i) g += Hxy[i * nn + l] * Hxy[i * nn + m];
                for (int a = 0; a < dim; ++a) K[(l * dim + a) * nd + m * dim + a] += c * g;
            }
        for (int l = 0; l < nn; ++l)
            for (int a = 0; a < dim; ++a) {
                double *row = Rw + (size_t)(l * dim + a) * dw * nn;
                for (int j = 0; j < dw * nn; ++j) row[j] += c * (H[l] * Bw[a * dw * nn + j]);
                double *rd = Rd + (size_t)(l * dim + a) * nn;
                for (int m = 0; m < nn; ++m) rd[m] -= c * (H[l] * Hxy[a * nn + m]);
            }
    }
    for (int q = 0; q < e->red.nq; ++q) {
        double detJ = geometry(dim, &e->cooRed, &e->red, q, X, Hxy);
        double c = e->red.w[q] * detJ;
        const double *H = e->red.H + (size_t)q * nn;
        memset(Bc, 0, sizeof(double) * dw * dim * nn);
        for (int i = 0; i < nind; ++i) {
            double sg = (i & 1) ? -1.0 : 1.0;
            for (int l = 0; l < nn; ++l) Bc[ic[i][0] * dim * nn + l * dim + ic[i][1]] = sg * Hxy[ic[i][2] * nn + l];
        }
        for (int r = 0; r < nd; ++r) {
            int l = r / dim, a = r % dim;
            double divr = Hxy[a * nn + l];
            for (int s = 0; s < nd; ++s) {
                int m = s / dim, b = s % dim;
                double cc = 0;
                for (int k = 0; k < dw; ++k) cc += Bc[k * dim * nn + r] * Bc[k * dim * nn + s];
                K[r * nd + s] += c * (alpha_d * (divr * Hxy[b * nn + m]) + alpha_w * cc);
            }
            for (int k = 0; k < dw; ++k)
                for (int m = 0; m < nn; ++m)
                    Rw[(size_t)r * dw * nn + m * dw + k] += c * alpha_w * (Bc[k * dim * nn + r] * H[m]);
            /* np.outer(Hxy.flatten("F"), H): flat-F index r -> Hxy[r % dim][r / dim] */
            for (int m = 0; m < nn; ++m) Rd[(size_t)r * nn + m] += c * alpha_d * (Hxy[a * nn + l] * H[m]);
        }
    }
    free(Hxy); free(Bw); free(Bc);
    return 0;
}

/* Spectral.getElemKLEOperators (spectral.py:162-228) on the GLL collocation
 * points.  SrT [ds n][dim n], DivSrT [dim n][ds n], Curl [dw n][dim n], W [n]. */
int orc_elem_ops(const orc_elem *e, const double *X, double *SrT, double *DivSrT,
                 double *Curl, double *W)
{
    const int dim = e->dim, nn = e->nn, dw = dim == 2 ? 1 : 3, ds = dim == 2 ? 3 : 6;
    const int nd = dim * nn;
    memset(SrT, 0, sizeof(double) * ds * nn * nd);
    memset(DivSrT, 0, sizeof(double) * nd * ds * nn);
    memset(Curl, 0, sizeof(double) * dw * nn * nd);
    double *Wm = calloc((size_t)nn * nn, sizeof(double));
    double *Hxy = malloc(sizeof(double) * 3 * nn);
    double *Bs = malloc(sizeof(double) * ds * nd);       /* B_srt  [ds][dim n]  */
    double *Bd = malloc(sizeof(double) * dim * ds * nn); /* B_div  [dim][ds n]  */
    double *Bc = malloc(sizeof(double) * dw * nd);       /* B_curl [dw][dim n]  */
    static const int bdiv2[2][2] = {{0, 1}, {1, 2}};
    static const int bdiv3[3][3] = {{0, 1, 5}, {1, 2, 3}, {5, 3, 4}};
    const int (*ic)[3] = dim == 2 ? INDC2 : IND3;
    const int nind = dim == 2 ? 2 : 6;
    for (int q = 0; q < e->op.nq; ++q) {
        double detJ = geometry(dim, &e->cooOp, &e->op, q, X, Hxy);
        double c = e->op.w[q] * detJ;
        const double *H = e->op.H + (size_t)q * nn;
        memset(Bs, 0, sizeof(double) * ds * nd);
        memset(Bd, 0, sizeof(double) * dim * ds * nn);
        memset(Bc, 0, sizeof(double) * dw * nd);
        for (int i = 0; i < nind; ++i) {
            double sg = (i & 1) ? -1.0 : 1.0;
            for (int l = 0; l < nn; ++l) Bc[ic[i][0] * nd + l * dim + ic[i][1]] = sg * Hxy[ic[i][2] * nn + l];
        }
        for (int x = 0; x < dim; ++x) {
            for (int l = 0; l < nn; ++l) Bs[(2 * x) * nd + l * dim + x] = 2 * Hxy[x * nn + l];
            for (int i = 0; i < dim; ++i) {
                int col = dim == 2 ? bdiv2[x][i] : bdiv3[x][i];
                for (int l = 0; l < nn; ++l) Bd[i * ds * nn + l * ds + col] = Hxy[x * nn + l];
                if (i != x) {
                    int row = (x + i != 2) ? x + i : 5;
                    for (int l = 0; l < nn; ++l) Bs[row * nd + l * dim + i] = Hxy[x * nn + l];
                }
            }
        }
        for (int j = 0; j < ds * nd; ++j) Bs[j] *= 0.5;
        /* Hsrt^T B_srt : row (l ds + k) = H[l] * B_srt[k] */
        for (int l = 0; l < nn; ++l)
            for (int k = 0; k < ds; ++k) {
                double *row = SrT + (size_t)(l * ds + k) * nd;
                for (int j = 0; j < nd; ++j) row[j] += c * (H[l] * Bs[k * nd + j]);
            }
        for (int l = 0; l < nn; ++l)
            for (int x = 0; x < dim; ++x) {
                double *row = DivSrT + (size_t)(l * dim + x) * ds * nn;
                for (int j = 0; j < ds * nn; ++j) row[j] += c * (H[l] * Bd[x * ds * nn + j]);
            }
        for (int l = 0; l < nn; ++l)
            for (int k = 0; k < dw; ++k) {
                double *row = Curl + (size_t)(l * dw + k) * nd;
                for (int j = 0; j < nd; ++j) row[j] += c * (H[l] * Bc[k * nd + j]);
            }
        for (int l = 0; l < nn; ++l)
            for (int m = 0; m < nn; ++m) Wm[l * nn + m] += c * (H[l] * H[m]);
    }
    for (int l = 0; l < nn; ++l) {
        double s = 0;
        for (int m = 0; m < nn; ++m) s += Wm[l * nn + m];
        W[l] = s;
    }
    free(Wm); free(Hxy); free(Bs); free(Bd); free(Bc);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* a6/a7/a9: structured box mesh in the canonical numbering                  */
/* ------------------------------------------------------------------------ */

typedef struct {
    int dim, ngl, p;
    int64_t nel[3], L[3], N, E;
    double lower[3], upper[3], h[3];
    int *loc2lat;       /* [nn][dim] lattice offset of local node l */
    double xi[ORC_MAXN];/* GLL nodes mapped to [0,1], ascending        */
    int64_t *uconn;     /* unstructured: explicit [E][nn] node ids      */
    double *ucorners;   /* unstructured: [E][2^dim][dim] closure order  */
} orc_mesh;

static const int CORN2[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
static const int CORN3[8][3] = {{0, 0, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0},
                                {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};

/* Box mesh (BoxDom.create, dmplex.py:382-388) with cells x-fastest and corner
 * closure order as test_dmplex_wrapper.py:24-27,106-115. */
orc_mesh *orc_mesh_box(int dim, const int64_t *nel, const double *lo, const double *hi, int ngl)
{
    orc_mesh *m = calloc(1, sizeof(orc_mesh));
    m->dim = dim;
    m->ngl = ngl;
    m->p = ngl - 1;
    m->N = 1;
    m->E = 1;
    for (int d = 0; d < 3; ++d) { m->nel[d] = 1; m->L[d] = 1; }
    for (int d = 0; d < dim; ++d) {
        m->nel[d] = nel[d];
        m->L[d] = nel[d] * m->p + 1;
        m->lower[d] = lo[d];
        m->upper[d] = hi[d];
        m->h[d] = (hi[d] - lo[d]) / nel[d];
        m->N *= m->L[d];
        m->E *= nel[d];
    }
    double x[ORC_MAXN], w[ORC_MAXN];
    orc_lobatto(ngl, x, w);
    for (int i = 0; i < ngl; ++i) m->xi[i] = (1.0 + x[i]) / 2.0;
    orc_elem *e = orc_elem_create(dim, ngl);
    int nn = e->nn;
    m->loc2lat = malloc(sizeof(int) * nn * dim);
    for (int l = 0; l < nn; ++l)
        for (int d = 0; d < dim; ++d) {
            double v = 0;
            for (int c = 0; c < (1 << dim); ++c)
                v += e->cooOp.H[l * (1 << dim) + c] * (dim == 2 ? CORN2[c][d] : CORN3[c][d]);
            int best = 0;
            for (int i = 1; i < ngl; ++i)
                if (fabs(m->xi[i] - v) < fabs(m->xi[best] - v)) best = i;
            m->loc2lat[l * dim + d] = best;
        }
    orc_elem_destroy(e);
    return m;
}

void orc_mesh_destroy(orc_mesh *m)
{
    if (!m) return;
    free(m->loc2lat);
    free(m->uconn);
    free(m->ucorners);
    free(m);
}

/* Unstructured mesh from explicit arrays (GmshDom + the section numbering are
 * restated in oracle.py: nodes identified by coordinates). */
orc_mesh *orc_mesh_from_arrays(int dim, int ngl, int64_t N, int64_t E, const int64_t *conn,
                               const double *corners)
{
    orc_mesh *m = calloc(1, sizeof(orc_mesh));
    m->dim = dim;
    m->ngl = ngl;
    m->p = ngl - 1;
    m->N = N;
    m->E = E;
    const int nn = dim == 2 ? ngl * ngl : ngl * ngl * ngl, nc = 1 << dim;
    m->uconn = malloc(sizeof(int64_t) * E * nn);
    m->ucorners = malloc(sizeof(double) * E * nc * dim);
    memcpy(m->uconn, conn, sizeof(int64_t) * E * nn);
    memcpy(m->ucorners, corners, sizeof(double) * E * nc * dim);
    return m;
}

int64_t orc_mesh_nnodes(const orc_mesh *m) { return m->N; }
int64_t orc_mesh_nelems(const orc_mesh *m) { return m->E; }

static void elem_index(const orc_mesh *m, int64_t e, int64_t *ei)
{
    ei[0] = e % m->nel[0];
    ei[1] = (e / m->nel[0]) % m->nel[1];
    ei[2] = e / (m->nel[0] * m->nel[1]);
}

/* element -> global node ids in local spectral order (the role of
 * DMPlexDom.getGlobalNodesFromCell, dmplex.py:193-196). */
int orc_mesh_conn(const orc_mesh *m, int64_t *conn)
{
    int nn = m->dim == 2 ? m->ngl * m->ngl : m->ngl * m->ngl * m->ngl;
    if (m->uconn) {
        memcpy(conn, m->uconn, sizeof(int64_t) * m->E * nn);
        return 0;
    }
    for (int64_t e = 0; e < m->E; ++e) {
        int64_t ei[3];
        elem_index(m, e, ei);
        for (int l = 0; l < nn; ++l) {
            int64_t id = 0;
            for (int d = m->dim - 1; d >= 0; --d)
                id = id * m->L[d] + ei[d] * m->p + m->loc2lat[l * m->dim + d];
            conn[e * nn + l] = id;
        }
    }
    return 0;
}

/* corner coordinates of every cell in closure order (dmplex.py:93-100). */
int orc_mesh_corners(const orc_mesh *m, double *X)
{
    int nc = 1 << m->dim;
    if (m->ucorners) {
        memcpy(X, m->ucorners, sizeof(double) * m->E * nc * m->dim);
        return 0;
    }
    for (int64_t e = 0; e < m->E; ++e) {
        int64_t ei[3];
        elem_index(m, e, ei);
        for (int c = 0; c < nc; ++c)
            for (int d = 0; d < m->dim; ++d) {
                int o = m->dim == 2 ? CORN2[c][d] : CORN3[c][d];
                X[(e * nc + c) * m->dim + d] = m->lower[d] + (ei[d] + o) * m->h[d];
            }
    }
    return 0;
}

/* node coordinates (computeFullCoordinates, dmplex.py:62-91). */
int orc_mesh_coords(const orc_mesh *m, double *xyz)
{
    for (int64_t n = 0; n < m->N; ++n) {
        int64_t r = n;
        for (int d = 0; d < m->dim; ++d) {
            int64_t li = r % m->L[d];
            r /= m->L[d];
            int64_t e = li / m->p, o = li % m->p;
            if (li == m->L[d] - 1) { e = m->nel[d] - 1; o = m->p; }
            xyz[n * m->dim + d] = (li == m->L[d] - 1) ? m->upper[d]
                                                       : m->lower[d] + (e + m->xi[o]) * m->h[d];
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* a8/a10: FS assembly into CSR (MatFS.build/buildFS, mat_fs.py:131-192)     */
/* ------------------------------------------------------------------------ */

typedef struct {
    int64_t m, n, nnz;
    int64_t *indptr;
    int64_t *indices;
    double *data;
} orc_csr;

void orc_csr_destroy(orc_csr *a)
{
    if (!a) return;
    free(a->indptr); free(a->indices); free(a->data); free(a);
}
int64_t orc_csr_nnz(const orc_csr *a) { return a->nnz; }
int64_t orc_csr_rows(const orc_csr *a) { return a->m; }
int orc_csr_export(const orc_csr *a, int64_t *indptr, int64_t *indices, double *data)
{
    memcpy(indptr, a->indptr, sizeof(int64_t) * (a->m + 1));
    memcpy(indices, a->indices, sizeof(int64_t) * a->nnz);
    memcpy(data, a->data, sizeof(double) * a->nnz);
    return 0;
}

orc_csr *orc_csr_from(int64_t m, int64_t n, const int64_t *indptr, const int64_t *indices,
                      const double *data)
{
    orc_csr *a = calloc(1, sizeof(orc_csr));
    a->m = m; a->n = n; a->nnz = indptr[m];
    a->indptr = malloc(sizeof(int64_t) * (m + 1));
    a->indices = malloc(sizeof(int64_t) * (a->nnz ? a->nnz : 1));
    a->data = malloc(sizeof(double) * (a->nnz ? a->nnz : 1));
    memcpy(a->indptr, indptr, sizeof(int64_t) * (m + 1));
    /* first touch by the same static row partition orc_spmv uses, so each
     * thread's rows sit in its own NUMA node's memory (as with one PETSc rank
     * per core) */
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < m; ++r) {
        const int64_t k0 = indptr[r], k1 = indptr[r + 1];
        memcpy(a->indices + k0, indices + k0, sizeof(int64_t) * (k1 - k0));
        memcpy(a->data + k0, data + k0, sizeof(double) * (k1 - k0));
    }
    return a;
}

static int cmp_i64(const void *a, const void *b)
{
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* node adjacency: sorted unique neighbour nodes of every node (a8). */
static int64_t **node_adjacency(const orc_mesh *m, const int64_t *conn, int *deg_out)
{
    int nn = m->dim == 2 ? m->ngl * m->ngl : m->ngl * m->ngl * m->ngl;
    int64_t N = m->N;
    int *cnt = calloc(N, sizeof(int));
    for (int64_t e = 0; e < m->E; ++e)
        for (int l = 0; l < nn; ++l) cnt[conn[e * nn + l]] += nn;
    int64_t **adj = malloc(sizeof(int64_t *) * N);
    for (int64_t i = 0; i < N; ++i) { adj[i] = malloc(sizeof(int64_t) * cnt[i]); deg_out[i] = 0; }
    for (int64_t e = 0; e < m->E; ++e)
        for (int l = 0; l < nn; ++l) {
            int64_t i = conn[e * nn + l];
            for (int k = 0; k < nn; ++k) adj[i][deg_out[i]++] = conn[e * nn + k];
        }
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t i = 0; i < N; ++i) {
        qsort(adj[i], deg_out[i], sizeof(int64_t), cmp_i64);
        int u = 0;
        for (int k = 0; k < deg_out[i]; ++k)
            if (u == 0 || adj[i][u - 1] != adj[i][k]) adj[i][u++] = adj[i][k];
        deg_out[i] = u;
    }
    free(cnt);
    return adj;
}

static int64_t find_col(const orc_csr *a, int64_t r, int64_t c)
{
    int64_t lo = a->indptr[r], hi = a->indptr[r + 1] - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a->indices[mid] == c) return mid;
        if (a->indices[mid] < c) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

/* Build the FS matrices K, Krhs, Rw exactly as MatFS.build (mat_fs.py:131-192):
 *   free rows x free cols of K  += K_e         (mat_fs.py:179-180)
 *   free rows x dir cols of Krhs += -K_e       (mat_fs.py:174-177)
 *   K[dir,dir] += 0 per element, then += 1     (mat_fs.py:182-183, 115-120)
 *   Krhs[dir,dir] += 1                         (mat_fs.py:117)
 *   Rw[free rows, all w cols] += Rw_e          (mat_fs.py:185-186)
 * ADD order is ascending cell order (single-rank MatSetValues).  dir_flag is
 * per node.  Explicit zeros are kept in the pattern. */
int orc_assemble_fs(const orc_mesh *m, const uint8_t *dir_flag, orc_csr **Kout,
                    orc_csr **Krhsout, orc_csr **Rwout)
{
    const int dim = m->dim, dw = dim == 2 ? 1 : 3;
    const int nn = dim == 2 ? m->ngl * m->ngl : m->ngl * m->ngl * m->ngl;
    const int64_t N = m->N;
    int64_t *conn = malloc(sizeof(int64_t) * m->E * nn);
    orc_mesh_conn(m, conn);
    int *deg = malloc(sizeof(int) * N);
    int64_t **adj = node_adjacency(m, conn, deg);
    orc_csr *K = calloc(1, sizeof(orc_csr)), *Kr = calloc(1, sizeof(orc_csr)),
            *Rw = calloc(1, sizeof(orc_csr));
    K->m = K->n = Kr->m = Kr->n = Rw->m = N * dim;
    Rw->n = N * dw;
    K->indptr = calloc(N * dim + 1, sizeof(int64_t));
    Kr->indptr = calloc(N * dim + 1, sizeof(int64_t));
    Rw->indptr = calloc(N * dim + 1, sizeof(int64_t));
    for (int64_t i = 0; i < N; ++i) {
        int nfree = 0, ndir = 0;
        for (int k = 0; k < deg[i]; ++k) {
            if (dir_flag[adj[i][k]]) ++ndir;
            else ++nfree;
        }
        for (int a = 0; a < dim; ++a) {
            int64_t r = i * dim + a;
            K->indptr[r + 1] = dir_flag[i] ? 1 : (int64_t)nfree * dim;
            Kr->indptr[r + 1] = dir_flag[i] ? 1 : (int64_t)ndir * dim;
            Rw->indptr[r + 1] = dir_flag[i] ? 0 : (int64_t)deg[i] * dw;
        }
    }
    for (int64_t r = 0; r < N * dim; ++r) {
        K->indptr[r + 1] += K->indptr[r];
        Kr->indptr[r + 1] += Kr->indptr[r];
        Rw->indptr[r + 1] += Rw->indptr[r];
    }
    orc_csr *all[3] = {K, Kr, Rw};
    for (int t = 0; t < 3; ++t) {
        all[t]->nnz = all[t]->indptr[all[t]->m];
        all[t]->indices = malloc(sizeof(int64_t) * (all[t]->nnz ? all[t]->nnz : 1));
        all[t]->data = calloc(all[t]->nnz ? all[t]->nnz : 1, sizeof(double));
    }
    for (int64_t i = 0; i < N; ++i)
        for (int a = 0; a < dim; ++a) {
            int64_t r = i * dim + a;
            int64_t pk = K->indptr[r], pr = Kr->indptr[r], pw = Rw->indptr[r];
            if (dir_flag[i]) {
                K->indices[pk] = r;
                Kr->indices[pr] = r;
                continue;
            }
            for (int k = 0; k < deg[i]; ++k) {
                int64_t j = adj[i][k];
                for (int b = 0; b < dim; ++b) {
                    if (dir_flag[j]) Kr->indices[pr++] = j * dim + b;
                    else K->indices[pk++] = j * dim + b;
                }
                for (int c = 0; c < dw; ++c) Rw->indices[pw++] = j * dw + c;
            }
        }
    orc_elem *el = orc_elem_create(dim, m->ngl);
    int nd = dim * nn, nc = 1 << dim;
    double *X = malloc(sizeof(double) * m->E * nc * dim);
    orc_mesh_corners(m, X);
    /* Elements in ascending batches: the batch's element matrices in parallel
     * (orc_elem_kle is reentrant), then the ADDs in parallel over disjoint
     * node-row ranges, each range walking the batch in ascending cell order.
     * Every entry therefore receives the same additions in the same order as
     * the serial cell loop of MatFS.buildFS: the result is bitwise the serial
     * one, at any thread count. */
    const int64_t B = 256;
    const size_t kes = (size_t)nd * nd, rws = (size_t)nd * dw * nn, rds = (size_t)nd * nn;
    double *Ke = malloc(sizeof(double) * kes * B), *Rwe = malloc(sizeof(double) * rws * B),
           *Rde = malloc(sizeof(double) * rds * B);
    for (int64_t e0 = 0; e0 < m->E; e0 += B) {
        const int64_t nb = m->E - e0 < B ? m->E - e0 : B;
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t k = 0; k < nb; ++k)
            orc_elem_kle(el, X + (e0 + k) * nc * dim, Ke + kes * k, Rwe + rws * k, Rde + rds * k);
#pragma omp parallel
        {
            const int T = omp_get_num_threads(), t = omp_get_thread_num();
            const int64_t nlo = N * t / T, nhi = N * (t + 1) / T;
            for (int64_t k = 0; k < nb; ++k) {
                const int64_t *cn = conn + (e0 + k) * nn;
                const double *ke = Ke + kes * k, *rwe = Rwe + rws * k;
                for (int li = 0; li < nn; ++li) {
                    int64_t gi = cn[li];
                    if (gi < nlo || gi >= nhi || dir_flag[gi]) continue;
                    for (int a = 0; a < dim; ++a) {
                        int64_t r = gi * dim + a;
                        for (int lj = 0; lj < nn; ++lj) {
                            int64_t gj = cn[lj];
                            for (int b = 0; b < dim; ++b) {
                                double v = ke[(li * dim + a) * nd + lj * dim + b];
                                if (dir_flag[gj]) Kr->data[find_col(Kr, r, gj * dim + b)] += -v;
                                else K->data[find_col(K, r, gj * dim + b)] += v;
                            }
                            for (int c = 0; c < dw; ++c)
                                Rw->data[find_col(Rw, r, gj * dw + c)] += rwe[(li * dim + a) * dw * nn + lj * dw + c];
                        }
                    }
                }
            }
        }
    }
    for (int64_t i = 0; i < N; ++i)
        if (dir_flag[i])
            for (int a = 0; a < dim; ++a) {
                K->data[K->indptr[i * dim + a]] += 1.0;
                Kr->data[Kr->indptr[i * dim + a]] += 1.0;
            }
    orc_elem_destroy(el);
    free(X); free(Ke); free(Rwe); free(Rde); free(conn);
    for (int64_t i = 0; i < N; ++i) free(adj[i]);
    free(adj); free(deg);
    *Kout = K; *Krhsout = Kr; *Rwout = Rw;
    return 0;
}

/* a12: Operators (mat_fs.py:194-271).  Curl [dw N x dim N], SrT [ds N x dim N],
 * DivSrT [dim N x ds N] on the full node adjacency (explicit zeros kept),
 * element blocks of Spectral.getElemKLEOperators added in ascending cell order
 * (Operators.setValues, mat_fs.py:238-251); the lumped weights are summed per
 * node in the same order, inverted (Vec.reciprocal) and applied as a left
 * diagonal scaling (Mat.diagonalScale(L=), mat_fs.py:253-271). */
static orc_csr *ops_pattern(int64_t N, const int *deg, int64_t *const *adj, int R, int C)
{
    orc_csr *A = calloc(1, sizeof(orc_csr));
    A->m = N * R;
    A->n = N * C;
    A->indptr = calloc(A->m + 1, sizeof(int64_t));
    for (int64_t i = 0; i < N; ++i)
        for (int a = 0; a < R; ++a) A->indptr[i * R + a + 1] = (int64_t)deg[i] * C;
    for (int64_t r = 0; r < A->m; ++r) A->indptr[r + 1] += A->indptr[r];
    A->nnz = A->indptr[A->m];
    A->indices = malloc(sizeof(int64_t) * (A->nnz ? A->nnz : 1));
    A->data = calloc(A->nnz ? A->nnz : 1, sizeof(double));
    for (int64_t i = 0; i < N; ++i)
        for (int a = 0; a < R; ++a) {
            int64_t p = A->indptr[i * R + a];
            for (int k = 0; k < deg[i]; ++k)
                for (int b = 0; b < C; ++b) A->indices[p++] = adj[i][k] * C + b;
        }
    return A;
}

static void ops_add(orc_csr *A, const int64_t *cn, int nn, int R, int C, const double *Ae)
{
    for (int li = 0; li < nn; ++li)
        for (int a = 0; a < R; ++a) {
            int64_t r = cn[li] * R + a;
            for (int lj = 0; lj < nn; ++lj) {
                int64_t p = find_col(A, r, cn[lj] * C);
                for (int b = 0; b < C; ++b) A->data[p + b] += Ae[(size_t)(li * R + a) * nn * C + lj * C + b];
            }
        }
}

static void ops_scale(orc_csr *A, int R, const double *winv)
{
    for (int64_t r = 0; r < A->m; ++r)
        for (int64_t k = A->indptr[r]; k < A->indptr[r + 1]; ++k) A->data[k] *= winv[r / R];
}

int orc_assemble_ops(const orc_mesh *m, orc_csr **Curl, orc_csr **SrT, orc_csr **DivSrT, double *Wout)
{
    const int dim = m->dim, dw = dim == 2 ? 1 : 3, ds = dim == 2 ? 3 : 6;
    const int nn = dim == 2 ? m->ngl * m->ngl : m->ngl * m->ngl * m->ngl;
    const int64_t N = m->N;
    int64_t *conn = malloc(sizeof(int64_t) * m->E * nn);
    orc_mesh_conn(m, conn);
    int *deg = malloc(sizeof(int) * N);
    int64_t **adj = node_adjacency(m, conn, deg);
    orc_csr *Cu = ops_pattern(N, deg, adj, dw, dim), *S = ops_pattern(N, deg, adj, ds, dim),
            *D = ops_pattern(N, deg, adj, dim, ds);
    double *W = calloc(N, sizeof(double));
    orc_elem *el = orc_elem_create(dim, m->ngl);
    const int nd = dim * nn, nc = 1 << dim;
    double *X = malloc(sizeof(double) * m->E * nc * dim);
    orc_mesh_corners(m, X);
    double *Se = malloc(sizeof(double) * ds * nn * nd), *De = malloc(sizeof(double) * nd * ds * nn),
           *Ce = malloc(sizeof(double) * dw * nn * nd), *We = malloc(sizeof(double) * nn);
    for (int64_t e = 0; e < m->E; ++e) {
        orc_elem_ops(el, X + e * nc * dim, Se, De, Ce, We);
        const int64_t *cn = conn + e * nn;
        ops_add(Cu, cn, nn, dw, dim, Ce);
        ops_add(S, cn, nn, ds, dim, Se);
        ops_add(D, cn, nn, dim, ds, De);
        for (int l = 0; l < nn; ++l) W[cn[l]] += We[l];
    }
    double *winv = calloc(N ? N : 1, sizeof(double));
    for (int64_t i = 0; i < N; ++i) winv[i] = 1.0 / W[i];
    ops_scale(S, ds, winv);
    ops_scale(D, dim, winv);
    ops_scale(Cu, dw, winv);
    if (Wout) memcpy(Wout, W, sizeof(double) * N);
    orc_elem_destroy(el);
    free(X); free(Se); free(De); free(Ce); free(We); free(W); free(winv); free(conn);
    for (int64_t i = 0; i < N; ++i) free(adj[i]);
    free(adj); free(deg);
    *Curl = Cu; *SrT = S; *DivSrT = D;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* a14/a15: CSR SpMV and PETSc-3.12-style KSPCG                               */
/* ------------------------------------------------------------------------ */

/* MatMult_SeqAIJ: y = A x (row-sequential sums in column order). */
void orc_spmv(const orc_csr *A, const double *x, double *y)
{
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < A->m; ++r) {
        double s = 0;
        for (int64_t k = A->indptr[r]; k < A->indptr[r + 1]; ++k) s += A->data[k] * x[A->indices[k]];
        y[r] = s;
    }
}

static double dot(int64_t n, const double *a, const double *b)
{
    double s = 0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

static double g_cg_loop_seconds = 0.0;
/* wall time of the last orc_cg's iteration loop (setup and the exit residual
 * excluded): what the CPU baseline times */
double orc_cg_loop_seconds(void) { return g_cg_loop_seconds; }

/* KSPSolve_CG (PETSc 3.12, src/ksp/ksp/impls/cg/cg.c; reached through
 * kle_solver.py:35 with -ksp_type cg [-pc_type jacobi|none]); zero initial
 * guess (KSP default), convergence on the UNPRECONDITIONED residual norm:
 * ||r_k|| <= max(rtol ||b||, atol).  jacobi != 0 uses z = D^-1 r.
 * Returns iterations; *relres = ||b - A x|| / ||b|| recomputed at exit. */
int orc_cg(const orc_csr *A, const double *b, double *x, double rtol, double atol, int maxit,
           int jacobi, int fixed_iters, double *relres)
{
    int64_t n = A->m;
    double *r = malloc(sizeof(double) * n), *z = malloc(sizeof(double) * n),
           *p = malloc(sizeof(double) * n), *w = malloc(sizeof(double) * n),
           *dinv = malloc(sizeof(double) * n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double d = 0;
        for (int64_t k = A->indptr[i]; k < A->indptr[i + 1]; ++k)
            if (A->indices[k] == i) d = A->data[k];
        dinv[i] = (jacobi && d != 0) ? 1.0 / d : 1.0;
        x[i] = 0;
        r[i] = b[i];
        z[i] = dinv[i] * r[i];
    }
    double bnorm = sqrt(dot(n, b, b));
    double tol = fmax(rtol * bnorm, atol);
    double beta = dot(n, z, r), betaold = 0;
    int it = 0;
    double rn = sqrt(dot(n, r, r));
    const double t_loop = omp_get_wtime();
    while (it < maxit && (fixed_iters || rn > tol)) {
        if (it == 0) memcpy(p, z, sizeof(double) * n);
        else {
            double bb = beta / betaold;
#pragma omp parallel for schedule(static)
            for (int64_t i = 0; i < n; ++i) p[i] = z[i] + bb * p[i];
        }
        orc_spmv(A, p, w);
        double dpi = dot(n, p, w);
        double a = beta / dpi;
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            x[i] += a * p[i];
            r[i] -= a * w[i];
            z[i] = dinv[i] * r[i];
        }
        betaold = beta;
        beta = dot(n, z, r);
        rn = sqrt(dot(n, r, r));
        ++it;
    }
    g_cg_loop_seconds = omp_get_wtime() - t_loop;
    orc_spmv(A, x, w);
    double s = 0;
    for (int64_t i = 0; i < n; ++i) s += (b[i] - w[i]) * (b[i] - w[i]);
    *relres = bnorm > 0 ? sqrt(s) / bnorm : sqrt(s);
    free(r); free(z); free(p); free(w); free(dinv);
    return it;
}

int orc_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_num_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* Host STREAM triad a = b + s c (McCalpin's kernel; 24 B moved per element,
 * the write-allocate read of `a` not counted, as STREAM reports it) over n
 * doubles per array on the current OpenMP threads, first-touched by the same
 * static schedule.  Best of `reps` in GB/s: the host memory ceiling the CPU
 * baseline's CSR CG runs against. */
double orc_stream_triad(int64_t n, int reps)
{
    double *a = malloc(sizeof(double) * n), *b = malloc(sizeof(double) * n), *c = malloc(sizeof(double) * n);
    if (!a || !b || !c) { free(a); free(b); free(c); return -1.0; }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) { a[i] = 0.0; b[i] = 1.0; c[i] = 2.0; }
    double best = 0.0;
    for (int r = 0; r < reps; ++r) {
        double t0 = omp_get_wtime();
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) a[i] = b[i] + 3.0 * c[i];
        double dt = omp_get_wtime() - t0;
        double gbs = 24.0 * (double)n / dt * 1e-9;
        if (gbs > best) best = gbs;
    }
    volatile double sink = a[n / 2];
    (void)sink;
    free(a); free(b); free(c);
    return best;
}
