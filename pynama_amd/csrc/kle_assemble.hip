// kle_assemble.hip -- batch device assembly of the KLE system on gfx950.
//
// Replaces MatFS.build -> buildFS (mat_fs.py:131-192): the per-cell Python
// loop that calls Spectral.getElemKLEMatrices (spectral.py:92-160) and
// inserts the element blocks with MatSetValues(ADD_VALUES).
//
// Kernels (patterns: k_pat_count / k_pat_fill on box meshes, k_upat on
// unstructured ones; element matrices: k_element_mfma by default, the FP64
// MFMA form of k_element below; elements are processed in ascending batches
// bounded by KLE_ASM_SCRATCH_GB):
//   k_geometry   one thread per (element, Gauss point): Jacobian of the
//                trilinear map, c_q = w_q det J, inv(J)          (spectral.py:117-120)
//   k_element    one element x (32x32 node-pair tile) per 256-thread workgroup.
//                Gauss-point loops staged through LDS in chunks of QC points;
//                factored form of the element matrices:
//                  K_e(la,mb) = d_ab G + a_d D_ab + a_w (d_ab tr D - D_ba)
//                  G   = sum_full c grad N_l . grad N_m
//                  D_ab= sum_red  c dN_l/dx_a dN_m/dx_b
//                  Rw_e from E_d = sum_full c N_l dN_m/dx_d and F_d = sum_red c dN_l/dx_d N_m
//                (algebraically identical to B_gr^T B_gr + a_d B_div^T B_div +
//                 a_w B_curl^T B_curl of spectral.py:134,155-156)
//   k_gather     one wavefront per owned node row: for every block column the
//                lanes sum the element blocks of the cells containing both
//                nodes in ascending cell order (PETSc single-rank ADD order),
//                no atomics -> bitwise deterministic.  Dirichlet masking as
//                mat_fs.py:158-189.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <cstdlib>
#include <cmath>
#include <cstring>

#include "kle_basis.hpp"
#include "kle_internal.hpp"

namespace kle {

constexpr double ALPHA_W = 1e2;  // spectral.py:96
constexpr double ALPHA_D = 1e3;  // spectral.py:97
constexpr int TL = 32;           // node tile of k_element
constexpr int QC = 32;           // Gauss points per LDS chunk (k_element)
constexpr int QM = 16;           // Gauss points per LDS chunk (k_element_mfma: 3 workgroups / CU)

struct Tables1D {
    int np1;          // 1-D points
    const double *x;  // [np1]
    const double *w;  // [np1]
    const double *h;  // [np1][ngl]
    const double *dh; // [np1][ngl]
};

// ------------------------------------------------------------- geometry
template <int DIM>
__global__ void k_geometry(int64_t nel, int ngl, Tables1D T, const double *__restrict__ corners,
                           double *__restrict__ geo)
{
    const int nq = DIM == 2 ? T.np1 * T.np1 : T.np1 * T.np1 * T.np1;
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= nel * nq) return;
    const int64_t e = t / nq;
    const int q = (int)(t % nq);
    int qi[3] = {q % T.np1, (q / T.np1) % T.np1, DIM == 3 ? q / (T.np1 * T.np1) : 0};
    double xi[3], wq = 1.0;
    for (int d = 0; d < DIM; ++d) {
        xi[d] = T.x[qi[d]];
        wq *= T.w[qi[d]];
    }
    constexpr int NC = 1 << DIM;
    // closure order of the corners (kle_mesh.cpp CORN2/CORN3)
    const int c2[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
    const int c3[8][3] = {{0, 0, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0},
                          {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
    double J[DIM][DIM] = {};
    const double *X = corners + e * NC * DIM;
    for (int c = 0; c < NC; ++c) {
        double s[3], f[3];
        for (int d = 0; d < DIM; ++d) {
            s[d] = 2.0 * (DIM == 2 ? c2[c][d] : c3[c][d]) - 1.0;
            f[d] = 0.5 * (1.0 + s[d] * xi[d]);
        }
        for (int k = 0; k < DIM; ++k) {
            double dn = 0.5 * s[k];
            for (int d = 0; d < DIM; ++d)
                if (d != k) dn *= f[d];
            for (int j = 0; j < DIM; ++j) J[k][j] += dn * X[c * DIM + j];
        }
    }
    double det, Ji[DIM][DIM];
    if constexpr (DIM == 2) {
        det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
        Ji[0][0] = J[1][1] / det;
        Ji[0][1] = -J[0][1] / det;
        Ji[1][0] = -J[1][0] / det;
        Ji[1][1] = J[0][0] / det;
    } else {
        const double a00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
        const double a01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
        const double a02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
        det = J[0][0] * a00 + J[0][1] * a01 + J[0][2] * a02;
        Ji[0][0] = a00 / det;
        Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
        Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
        Ji[1][0] = a01 / det;
        Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
        Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
        Ji[2][0] = a02 / det;
        Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
        Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
    }
    double *g = geo + t * (1 + DIM * DIM);
    g[0] = wq * det;  // signed det J, as spectral.py:120
    for (int i = 0; i < DIM; ++i)
        for (int k = 0; k < DIM; ++k) g[1 + i * DIM + k] = Ji[i][k];
}

// Fill one LDS chunk: for points q0..q0+QC-1 and the 32 nodes of a tile,
// value H and physical gradient, optionally scaled by c_q.
template <int DIM>
__device__ __forceinline__ void fill_chunk(int ngl, int ne, int nq, const Tables1D &T,
                                           const double *__restrict__ geo, int q0, int n0,
                                           bool scale, double (*sH)[TL], double (*sG)[DIM][TL],
                                           const double (*sgeo)[1 + DIM * DIM], int tid)
{
    for (int it = tid; it < QC * TL; it += 256) {
        const int qq = it / TL, nl = it % TL;
        const int q = q0 + qq, l = n0 + nl;
        double hv = 0, g[DIM] = {};
        if (q < nq && l < ne) {
            const int qi[3] = {q % T.np1, (q / T.np1) % T.np1, DIM == 3 ? q / (T.np1 * T.np1) : 0};
            const int li[3] = {l % ngl, (l / ngl) % ngl, DIM == 3 ? l / (ngl * ngl) : 0};
            double hh[3], dd[3];
            for (int d = 0; d < DIM; ++d) {
                hh[d] = T.h[qi[d] * ngl + li[d]];
                dd[d] = T.dh[qi[d] * ngl + li[d]];
            }
            double dref[DIM];
            if constexpr (DIM == 2) {
                hv = hh[0] * hh[1];
                dref[0] = dd[0] * hh[1];
                dref[1] = hh[0] * dd[1];
            } else {
                hv = hh[0] * hh[1] * hh[2];
                dref[0] = dd[0] * hh[1] * hh[2];
                dref[1] = hh[0] * dd[1] * hh[2];
                dref[2] = hh[0] * hh[1] * dd[2];
            }
            const double *gq = sgeo[qq];
            for (int i = 0; i < DIM; ++i) {
                double s = 0;
                for (int k = 0; k < DIM; ++k) s += gq[1 + i * DIM + k] * dref[k];
                g[i] = s;
            }
            if (scale) {
                hv *= gq[0];
                for (int i = 0; i < DIM; ++i) g[i] *= gq[0];
            }
        }
        sH[qq][nl] = hv;
        for (int i = 0; i < DIM; ++i) sG[qq][i][nl] = g[i];
    }
}

// K_e, Rw_e (and Rd_e) blocks of node pair (l, m) from the factored sums
// (G, E_d, D_ab, F_d of k_element's header comment)
template <int DIM>
__device__ __forceinline__ void store_elem_blocks(int64_t e, int l, int m, int ne, double G, const double (&E)[DIM],
                                                  const double (&D)[DIM][DIM], const double (&F)[DIM],
                                                  double *__restrict__ Ke, double *__restrict__ Rwe,
                                                  double *__restrict__ Rde)
{
    constexpr int DW = DIM == 2 ? 1 : 3;
    double tr = 0;
    for (int c = 0; c < DIM; ++c) tr += D[c][c];
    double *kb = Ke + ((e * ne + l) * (int64_t)ne + m) * (DIM * DIM);
    for (int a = 0; a < DIM; ++a)
        for (int b = 0; b < DIM; ++b) {
            double val = ALPHA_D * D[a][b] - ALPHA_W * D[b][a];
            if (a == b) val += G + ALPHA_W * tr;
            kb[a * DIM + b] = val;
        }
    double rw[DIM][DW] = {};
    if constexpr (DIM == 3) {
        // (row, col, derivative) of B_curl / Bw_curl, sign (-1)^t
        // (indCurl == indWCurl, spectral.py:31-32)
        const int ind[6][3] = {{0, 2, 1}, {0, 1, 2}, {1, 0, 2}, {1, 2, 0}, {2, 1, 0}, {2, 0, 1}};
        for (int t = 0; t < 6; ++t) {
            const double sg = (t & 1) ? -1.0 : 1.0;
            const int r0 = ind[t][0], r1 = ind[t][1], d = ind[t][2];
            rw[r0][r1] += sg * E[d];             // H^T Bw_curl  (full)
            rw[r1][r0] += ALPHA_W * sg * F[d];   // a_w B_curl^T H (reduced)
        }
    } else {
        // indWCurl 2-D [[0,0,1],[1,0,0]] ; indCurl 2-D [[0,1,0],[0,0,1]]
        rw[0][0] += E[1] - ALPHA_W * F[1];
        rw[1][0] += -E[0] + ALPHA_W * F[0];
    }
    double *rb = Rwe + ((e * ne + l) * (int64_t)ne + m) * (DIM * DW);
    for (int a = 0; a < DIM; ++a)
        for (int c = 0; c < DW; ++c) rb[a * DW + c] = rw[a][c];
    if (Rde) {
        // Rd_e = -H^T B_div (full) + a_d B_div^T H (reduced)   (spectral.py:136-137,157)
        double *db = Rde + ((e * ne + l) * (int64_t)ne + m) * DIM;
        for (int a = 0; a < DIM; ++a) db[a] = -E[a] + ALPHA_D * F[a];
    }
}

// fill_chunk with the index arithmetic hoisted: the 1-D tables (th, tdh:
// [point][node]) live in LDS and every point / node of the chunk / tile comes
// pre-decomposed into lattice indices (x | y << 8 | z << 16, -1 outside), so
// an entry costs a few LDS reads and FMAs instead of six integer divisions
// and global table loads.  Same arithmetic, same values.
template <int DIM, int NQ = QC>
__device__ __forceinline__ void fill_chunk_lds(int ngl, const double *th, const double *tdh, const int *sq,
                                               const int *sn, bool scale, double (*sH)[TL], double (*sG)[DIM][TL],
                                               const double (*sgeo)[1 + DIM * DIM], int tid)
{
    for (int it = tid; it < NQ * TL; it += 256) {
        const int qq = it / TL, nl = it % TL;
        const int qp = sq[qq], lp = sn[nl];
        double hv = 0, g[DIM] = {};
        if (qp >= 0 && lp >= 0) {
            double hh[3], dd[3];
            for (int d = 0; d < DIM; ++d) {
                const int t = ((qp >> (8 * d)) & 255) * ngl + ((lp >> (8 * d)) & 255);
                hh[d] = th[t];
                dd[d] = tdh[t];
            }
            double dref[DIM];
            if constexpr (DIM == 2) {
                hv = hh[0] * hh[1];
                dref[0] = dd[0] * hh[1];
                dref[1] = hh[0] * dd[1];
            } else {
                hv = hh[0] * hh[1] * hh[2];
                dref[0] = dd[0] * hh[1] * hh[2];
                dref[1] = hh[0] * dd[1] * hh[2];
                dref[2] = hh[0] * hh[1] * dd[2];
            }
            const double *gq = sgeo[qq];
            for (int i = 0; i < DIM; ++i) {
                double s = 0;
                for (int k = 0; k < DIM; ++k) s += gq[1 + i * DIM + k] * dref[k];
                g[i] = s;
            }
            if (scale) {
                hv *= gq[0];
                for (int i = 0; i < DIM; ++i) g[i] *= gq[0];
            }
        }
        sH[qq][nl] = hv;
        for (int i = 0; i < DIM; ++i) sG[qq][i][nl] = g[i];
    }
}

__device__ __forceinline__ int pack_lattice(int v, int n, int dim)
{
    const int x = v % n, y = (v / n) % n, z = dim == 3 ? v / (n * n) : 0;
    return x | (y << 8) | (z << 16);
}

template <int DIM>
__global__ __launch_bounds__(256) void k_element(int ngl, Tables1D TF, Tables1D TR,
                                                 const double *__restrict__ geoF,
                                                 const double *__restrict__ geoR,
                                                 double *__restrict__ Ke, double *__restrict__ Rwe,
                                                 double *__restrict__ Rde)
{
    constexpr int DW = DIM == 2 ? 1 : 3;
    constexpr int G1 = 1 + DIM * DIM;
    const int ne = DIM == 2 ? ngl * ngl : ngl * ngl * ngl;
    const int nqF = DIM == 2 ? TF.np1 * TF.np1 : TF.np1 * TF.np1 * TF.np1;
    const int nqR = DIM == 2 ? TR.np1 * TR.np1 : TR.np1 * TR.np1 * TR.np1;
    const int64_t e = blockIdx.z;
    const int l0 = blockIdx.x * TL, m0 = blockIdx.y * TL;
    const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;

    __shared__ double sHL[QC][TL], sHM[QC][TL];
    __shared__ double sGL[QC][DIM][TL], sGM[QC][DIM][TL];
    __shared__ double sgeo[QC][G1];

    double G[4] = {}, E[DIM][4] = {}, D[DIM][DIM][4] = {}, F[DIM][4] = {};

    // full integration (GLL if ngl > 3 else Gauss): G and E
    for (int q0 = 0; q0 < nqF; q0 += QC) {
        for (int it = tid; it < QC * G1; it += 256) {
            int qq = it / G1, k = it % G1;
            sgeo[qq][k] = (q0 + qq < nqF) ? geoF[(e * nqF + q0 + qq) * G1 + k] : 0.0;
        }
        __syncthreads();
        fill_chunk<DIM>(ngl, ne, nqF, TF, geoF, q0, l0, true, sHL, sGL, sgeo, tid);
        fill_chunk<DIM>(ngl, ne, nqF, TF, geoF, q0, m0, false, sHM, sGM, sgeo, tid);
        __syncthreads();
        const int qn = min(QC, nqF - q0);
        for (int qq = 0; qq < qn; ++qq) {
            double gl[2][DIM], hl[2], gm[2][DIM];
            for (int u = 0; u < 2; ++u) {
                hl[u] = sHL[qq][tx + 16 * u];
                for (int i = 0; i < DIM; ++i) {
                    gl[u][i] = sGL[qq][i][tx + 16 * u];
                    gm[u][i] = sGM[qq][i][ty + 16 * u];
                }
            }
            for (int u = 0; u < 2; ++u)
                for (int v = 0; v < 2; ++v) {
                    double s = 0;
                    for (int i = 0; i < DIM; ++i) s += gl[u][i] * gm[v][i];
                    G[u * 2 + v] += s;
                    for (int d = 0; d < DIM; ++d) E[d][u * 2 + v] += hl[u] * gm[v][d];
                }
        }
        __syncthreads();
    }
    // reduced integration (Gauss ngl-1): D and F
    for (int q0 = 0; q0 < nqR; q0 += QC) {
        for (int it = tid; it < QC * G1; it += 256) {
            int qq = it / G1, k = it % G1;
            sgeo[qq][k] = (q0 + qq < nqR) ? geoR[(e * nqR + q0 + qq) * G1 + k] : 0.0;
        }
        __syncthreads();
        fill_chunk<DIM>(ngl, ne, nqR, TR, geoR, q0, l0, true, sHL, sGL, sgeo, tid);
        fill_chunk<DIM>(ngl, ne, nqR, TR, geoR, q0, m0, false, sHM, sGM, sgeo, tid);
        __syncthreads();
        const int qn = min(QC, nqR - q0);
        for (int qq = 0; qq < qn; ++qq) {
            double gl[2][DIM], gm[2][DIM], hm[2];
            for (int u = 0; u < 2; ++u) {
                hm[u] = sHM[qq][ty + 16 * u];
                for (int i = 0; i < DIM; ++i) {
                    gl[u][i] = sGL[qq][i][tx + 16 * u];
                    gm[u][i] = sGM[qq][i][ty + 16 * u];
                }
            }
            for (int u = 0; u < 2; ++u)
                for (int v = 0; v < 2; ++v) {
                    for (int a = 0; a < DIM; ++a)
                        for (int b = 0; b < DIM; ++b) D[a][b][u * 2 + v] += gl[u][a] * gm[v][b];
                    for (int d = 0; d < DIM; ++d) F[d][u * 2 + v] += gl[u][d] * hm[v];
                }
        }
        __syncthreads();
    }
    // compose and store the blocks: Ke[e][l][m][a][b], Rwe[e][l][m][a][c]
    for (int u = 0; u < 2; ++u)
        for (int v = 0; v < 2; ++v) {
            const int l = l0 + tx + 16 * u, m = m0 + ty + 16 * v;
            if (l >= ne || m >= ne) continue;
            const int pv = u * 2 + v;
            double d[DIM][DIM], ev[DIM], fv[DIM];
            for (int a = 0; a < DIM; ++a) {
                ev[a] = E[a][pv];
                fv[a] = F[a][pv];
                for (int b = 0; b < DIM; ++b) d[a][b] = D[a][b][pv];
            }
            store_elem_blocks<DIM>(e, l, m, ne, G[pv], ev, d, fv, Ke, Rwe, Rde);
        }
}

// MFMA form of k_element (the default): the Gauss-point sums are GEMMs,
//   G    = (c grad N_L)^T (grad N_M)   (K = DIM * nq_full)
//   E_d  = (c N_L)^T (dN_M/dx_d)       (K = nq_full)
//   D_ab = (c dN_L/dx_a)^T (dN_M/dx_b) (K = nq_red)
//   F_d  = (c dN_L/dx_d)^T N_M         (K = nq_red)
// run on v_mfma_f64_16x16x4_f64: each of the 4 waves owns a 16x16 (l, m)
// sub-tile of the workgroup's 32x32 tile and keeps all 1 + DIM + DIM^2 + DIM
// accumulators (double4 each) in registers; the A (l side, scaled by c_q) and
// B (m side) operands come from the same LDS chunks as k_element, four Gauss
// points per instruction (lane: A[l = lane&15][q = lane>>4], B[q = lane>>4][m
// = lane&15]; result reg r at l = (lane>>4) + 4r, m = lane&15).
typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ dbl4 mfma64(double a, double b, dbl4 c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int DIM, int MINW>
__global__ __launch_bounds__(256, MINW) void k_element_mfma(int ngl, Tables1D TF, Tables1D TR,
                                                      const double *__restrict__ geoF,
                                                      const double *__restrict__ geoR,
                                                      double *__restrict__ Ke, double *__restrict__ Rwe,
                                                      double *__restrict__ Rde)
{
    constexpr int G1 = 1 + DIM * DIM;
    const int ne = DIM == 2 ? ngl * ngl : ngl * ngl * ngl;
    const int nqF = DIM == 2 ? TF.np1 * TF.np1 : TF.np1 * TF.np1 * TF.np1;
    const int nqR = DIM == 2 ? TR.np1 * TR.np1 : TR.np1 * TR.np1 * TR.np1;
    const int64_t e = blockIdx.z;
    const int l0 = blockIdx.x * TL, m0 = blockIdx.y * TL;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ls = (wv & 1) * 16, ms = (wv >> 1) * 16;  // this wave's 16x16 sub-tile
    const int li = lane & 15, kq = lane >> 4;

    __shared__ double sHL[QM][TL], sHM[QM][TL];
    __shared__ double sGL[QM][DIM][TL], sGM[QM][DIM][TL];
    __shared__ double sgeo[QM][G1];
    __shared__ double sTab[4][64];  // full h, dh; reduced h, dh  [point * ngl + node]
    __shared__ int sLn[TL], sMn[TL], sQ[QM];
    for (int it = tid; it < 64; it += 256) {
        sTab[0][it] = it < TF.np1 * ngl ? TF.h[it] : 0.0;
        sTab[1][it] = it < TF.np1 * ngl ? TF.dh[it] : 0.0;
        sTab[2][it] = it < TR.np1 * ngl ? TR.h[it] : 0.0;
        sTab[3][it] = it < TR.np1 * ngl ? TR.dh[it] : 0.0;
    }
    if (tid < TL) {
        sLn[tid] = l0 + tid < ne ? pack_lattice(l0 + tid, ngl, DIM) : -1;
        sMn[tid] = m0 + tid < ne ? pack_lattice(m0 + tid, ngl, DIM) : -1;
    }

    const dbl4 z4 = {0.0, 0.0, 0.0, 0.0};
    dbl4 G = z4, E[DIM], D[DIM][DIM], F[DIM];
#pragma unroll
    for (int a = 0; a < DIM; ++a) {
        E[a] = z4;
        F[a] = z4;
#pragma unroll
        for (int b = 0; b < DIM; ++b) D[a][b] = z4;
    }

    // full integration: G and E (the chunk beyond nq is zero-filled)
    for (int q0 = 0; q0 < nqF; q0 += QM) {
        for (int it = tid; it < QM * G1; it += 256) {
            int qq = it / G1, k = it % G1;
            sgeo[qq][k] = (q0 + qq < nqF) ? geoF[(e * nqF + q0 + qq) * G1 + k] : 0.0;
        }
        if (tid < QM) sQ[tid] = q0 + tid < nqF ? pack_lattice(q0 + tid, TF.np1, DIM) : -1;
        __syncthreads();
        fill_chunk_lds<DIM, QM>(ngl, sTab[0], sTab[1], sQ, sLn, true, sHL, sGL, sgeo, tid);
        fill_chunk_lds<DIM, QM>(ngl, sTab[0], sTab[1], sQ, sMn, false, sHM, sGM, sgeo, tid);
        __syncthreads();
        const int qn = min(QM, nqF - q0);
        for (int qq = 0; qq < qn; qq += 4) {
            const int q = qq + kq;
            const double ah = sHL[q][ls + li];
            double ag[DIM], bg[DIM];
#pragma unroll
            for (int i = 0; i < DIM; ++i) {
                ag[i] = sGL[q][i][ls + li];
                bg[i] = sGM[q][i][ms + li];
            }
#pragma unroll
            for (int i = 0; i < DIM; ++i) G = mfma64(ag[i], bg[i], G);
#pragma unroll
            for (int d = 0; d < DIM; ++d) E[d] = mfma64(ah, bg[d], E[d]);
        }
        __syncthreads();
    }
    // reduced integration: D and F
    for (int q0 = 0; q0 < nqR; q0 += QM) {
        for (int it = tid; it < QM * G1; it += 256) {
            int qq = it / G1, k = it % G1;
            sgeo[qq][k] = (q0 + qq < nqR) ? geoR[(e * nqR + q0 + qq) * G1 + k] : 0.0;
        }
        if (tid < QM) sQ[tid] = q0 + tid < nqR ? pack_lattice(q0 + tid, TR.np1, DIM) : -1;
        __syncthreads();
        fill_chunk_lds<DIM, QM>(ngl, sTab[2], sTab[3], sQ, sLn, true, sHL, sGL, sgeo, tid);
        fill_chunk_lds<DIM, QM>(ngl, sTab[2], sTab[3], sQ, sMn, false, sHM, sGM, sgeo, tid);
        __syncthreads();
        const int qn = min(QM, nqR - q0);
        for (int qq = 0; qq < qn; qq += 4) {
            const int q = qq + kq;
            const double bh = sHM[q][ms + li];
            double ag[DIM], bg[DIM];
#pragma unroll
            for (int i = 0; i < DIM; ++i) {
                ag[i] = sGL[q][i][ls + li];
                bg[i] = sGM[q][i][ms + li];
            }
#pragma unroll
            for (int a = 0; a < DIM; ++a)
#pragma unroll
                for (int b = 0; b < DIM; ++b) D[a][b] = mfma64(ag[a], bg[b], D[a][b]);
#pragma unroll
            for (int d = 0; d < DIM; ++d) F[d] = mfma64(ag[d], bh, F[d]);
        }
        __syncthreads();
    }
    const int m = m0 + ms + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int l = l0 + ls + kq + 4 * r;
        if (l >= ne || m >= ne) continue;
        double d[DIM][DIM], ev[DIM], fv[DIM];
#pragma unroll
        for (int a = 0; a < DIM; ++a) {
            ev[a] = E[a][r];
            fv[a] = F[a][r];
#pragma unroll
            for (int b = 0; b < DIM; ++b) d[a][b] = D[a][b][r];
        }
        store_elem_blocks<DIM>(e, l, m, ne, G[r], ev, d, fv, Ke, Rwe, Rde);
    }
}

// ---------------------------------------------------------------- gather
struct MeshDev {
    int dim, p, ngl, ne;
    int64_t nel[3], L[3];
    int64_t node_begin, ext_begin, elem_begin;
};

// MODE 0: K (free cols, +K_e), 1: Krhs (Dirichlet cols, -K_e), 2: Rw (+Rw_e)
template <int R, int C, int MODE>
__global__ __launch_bounds__(256) void k_gather(MeshDev M, int64_t nrows, const int *__restrict__ rowptr,
                                                const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr,
                                                int lay, const int *__restrict__ bcol,
                                                const uint8_t *__restrict__ dir,
                                                const double *__restrict__ Eblk, double *__restrict__ val,
                                                int64_t eb0, int64_t eb1, int accum)
{
    const int lane = threadIdx.x & 63;
    const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (row >= nrows) return;
    const int64_t gi = M.node_begin + row;
    const int b0 = rowptr[row], mp = rowptr[row + 1] - b0, m = rowcnt ? rowcnt[row] : mp;
    double *v = val + vptr[row];
    if (dir[gi - M.ext_begin]) {
        // K[dir,dir] = 0 + ... + 0 + 1 and Krhs[dir,dir] = 1 (mat_fs.py:115-120,182-183)
        if (MODE != 2 && lane == 0 && m == 1 && eb0 == 0)
            for (int a = 0; a < R; ++a)
                for (int b = 0; b < C; ++b) v[vofs(lay, R * C, a * C + b, 0, m, mp)] = (a == b) ? 1.0 : 0.0;
        return;
    }
    int64_t ci[3] = {gi % M.L[0], (gi / M.L[0]) % M.L[1], M.dim == 3 ? gi / (M.L[0] * M.L[1]) : 0};
    int64_t elo[3], ehi[3];
    for (int d = 0; d < 3; ++d) {
        if (d >= M.dim) {
            elo[d] = ehi[d] = 0;
            continue;
        }
        int64_t c = ci[d];
        elo[d] = (c % M.p == 0) ? max((int64_t)0, c / M.p - 1) : c / M.p;
        ehi[d] = min(M.nel[d] - 1, c / M.p);
    }
    // element batch [eb0, eb1) (local ids, ascending = the ADD order): rows
    // with no cell in it are left as they are
    const int64_t emin = elo[0] + M.nel[0] * (elo[1] + M.nel[1] * elo[2]) - M.elem_begin;
    const int64_t emax = ehi[0] + M.nel[0] * (ehi[1] + M.nel[1] * ehi[2]) - M.elem_begin;
    if (emax < eb0 || emin >= eb1) return;
    const int ngl = M.ngl, ne = M.ne;
    for (int k = lane; k < m; k += 64) {
        const int64_t gj = M.ext_begin + bcol[b0 + k];
        int64_t cj[3] = {gj % M.L[0], (gj / M.L[0]) % M.L[1], M.dim == 3 ? gj / (M.L[0] * M.L[1]) : 0};
        double acc[R * C];
        // later batches continue the ascending-cell sum from the stored partial
#pragma unroll
        for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = 0; b < C; ++b) acc[a * C + b] = accum ? v[vofs(lay, R * C, a * C + b, k, m, mp)] : 0.0;
        for (int64_t ez = elo[2]; ez <= ehi[2]; ++ez)
            for (int64_t ey = elo[1]; ey <= ehi[1]; ++ey)
                for (int64_t ex = elo[0]; ex <= ehi[0]; ++ex) {
                    const int64_t eo[3] = {ex * M.p, ey * M.p, ez * M.p};
                    bool in = true;
                    int oj[3] = {0, 0, 0}, oi[3] = {0, 0, 0};
                    for (int d = 0; d < M.dim; ++d) {
                        int64_t o = cj[d] - eo[d];
                        in = in && o >= 0 && o <= M.p;
                        oj[d] = (int)o;
                        oi[d] = (int)(ci[d] - eo[d]);
                    }
                    const int64_t e = ex + M.nel[0] * (ey + M.nel[1] * ez) - M.elem_begin;
                    if (!in || e < eb0 || e >= eb1) continue;
                    const int li = oi[0] + ngl * (oi[1] + ngl * oi[2]);
                    const int lj = oj[0] + ngl * (oj[1] + ngl * oj[2]);
                    const double *blk = Eblk + (((e - eb0) * ne + li) * (int64_t)ne + lj) * (R * C);
#pragma unroll
                    for (int t = 0; t < R * C; ++t) acc[t] += (MODE == 1) ? -blk[t] : blk[t];
                }
#pragma unroll
        for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = 0; b < C; ++b) v[vofs(lay, R * C, a * C + b, k, m, mp)] = acc[a * C + b];
    }
}

static MeshDev mesh_dev(const kle_mesh *m)
{
    MeshDev M;
    M.dim = m->dim;
    M.p = m->p;
    M.ngl = m->ngl;
    M.ne = m->nn();
    for (int d = 0; d < 3; ++d) {
        M.nel[d] = m->nel[d];
        M.L[d] = m->L[d];
    }
    M.node_begin = m->node_begin;
    M.ext_begin = m->ext_begin;
    M.elem_begin = m->elem_begin;
    return M;
}

// KLE_TIMING=1: stream-synchronised wall time of each setup phase on stderr
struct PhaseTimer {
    kle_ctx *c;
    bool on;
    std::chrono::steady_clock::time_point t;
    explicit PhaseTimer(kle_ctx *ctx) : c(ctx)
    {
        const char *e = getenv("KLE_TIMING");
        on = e && atoi(e) != 0;
        t = std::chrono::steady_clock::now();
    }
    void lap(const char *what)
    {
        if (!on) return;
        (void)hipStreamSynchronize(c->stream);
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[kle timing r%d] %-34s %9.2f ms\n", c->rank, what,
                std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// Unstructured mesh topology on the device (kle_umesh.cpp arrays, ext-local ids)
struct UMeshDev {
    int ne;
    const int *conn;      // [e][ne] ext-local node
    const int64_t *incp;  // owned row -> [incp[i], incp[i+1])
    const int *inc;       // e * ne + l
    int64_t glo;          // ext-local id of owned row 0
};

struct UMeshBuf {
    int *conn = nullptr, *inc = nullptr;
    int64_t *incp = nullptr;
    UMeshDev dev{};
    ~UMeshBuf()
    {
        hipFree(conn);
        hipFree(inc);
        hipFree(incp);
    }
};

static int upload_umesh(kle_ctx *ctx, const kle_mesh *m, UMeshBuf &U)
{
    const int ne = m->nn();
    std::vector<int> c32(std::max<size_t>(m->u_conn.size(), 1));
    for (size_t k = 0; k < m->u_conn.size(); ++k) c32[k] = (int)(m->u_conn[k] - m->ext_begin);
    KLE_HIP(hipMalloc(&U.conn, sizeof(int) * c32.size()));
    KLE_HIP(hipMalloc(&U.incp, sizeof(int64_t) * m->u_incp.size()));
    KLE_HIP(hipMalloc(&U.inc, sizeof(int) * std::max<size_t>(m->u_inc.size(), 1)));
    KLE_HIP(hipMemcpyAsync(U.conn, c32.data(), sizeof(int) * c32.size(), hipMemcpyHostToDevice, ctx->stream));
    KLE_HIP(hipMemcpyAsync(U.incp, m->u_incp.data(), sizeof(int64_t) * m->u_incp.size(), hipMemcpyHostToDevice,
                           ctx->stream));
    if (!m->u_inc.empty())
        KLE_HIP(hipMemcpyAsync(U.inc, m->u_inc.data(), sizeof(int) * m->u_inc.size(), hipMemcpyHostToDevice,
                               ctx->stream));
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    U.dev = {ne, U.conn, U.incp, U.inc, m->node_begin - m->ext_begin};
    return 0;
}

// ------------------------------------------------------ device patterns
// Box meshes: the symbolic pattern `which` (kle_mesh.cpp row_cols: the
// preallocation of mat_fs.py:21-94 / mat_ns.py:7-45) built on the device, one
// wavefront per owned node row.  The lanes walk the row's neighbour box
// (nodes sharing a cell) in ascending node id, the Dirichlet filter of
// `which` is a ballot, and the kept columns are compacted with a popcount
// prefix -> the same ascending column list as the host enumeration, bit for
// bit, without materialising O(nnz) host arrays.
struct PatRowInfo {
    int cnt;   // kept columns
    int cmin;  // first / last kept column (ext-relative), INT_MAX / -1 when empty
    int cmax;
    int box0;  // structured-column box: base column, nx | ny<<8 | nz<<16 (-1: not a box)
    int box1;
};

__device__ __forceinline__ bool pat_keep(int which, bool di, bool dj)
{
    switch (which) {
    case 0: return !dj;
    case 1: return dj;
    case 4: return di || dj;
    case 5: return dj;
    default: return true;  // 2, 3, 6
    }
}

// neighbour box of node row gi (kle_mesh.cpp nbr_range); returns false for the
// rows whose pattern is not a box walk (Dirichlet rows of K/Krhs/Rw, free rows of Rwfs)
__device__ __forceinline__ bool pat_row_box(const MeshDev &M, int which, int64_t gi, bool di, int64_t lo[3],
                                            int64_t n[3], int &special)
{
    special = -1;
    if (which == 6 && !di) {
        special = 0;
        return false;
    }
    if (which <= 2 && di) {
        special = which != 2 ? 1 : 0;
        return false;
    }
    const int64_t c[3] = {gi % M.L[0], (gi / M.L[0]) % M.L[1], M.dim == 3 ? gi / (M.L[0] * M.L[1]) : 0};
    for (int d = 0; d < 3; ++d) {
        int64_t a = 0, b = 0;
        if (d < M.dim) {
            if (c[d] % M.p == 0) {
                a = max((int64_t)0, c[d] - M.p);
                b = min(M.L[d] - 1, c[d] + M.p);
            } else {
                a = (c[d] / M.p) * M.p;
                b = a + M.p;
            }
        }
        lo[d] = a;
        n[d] = b - a + 1;
    }
    return true;
}

__global__ __launch_bounds__(256) void k_pat_count(MeshDev M, int64_t nrows, int which,
                                                   const uint8_t *__restrict__ dir, PatRowInfo *__restrict__ info)
{
    const int lane = threadIdx.x & 63;
    const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (row >= nrows) return;
    const int64_t gi = M.node_begin + row;
    const bool di = dir[gi - M.ext_begin] != 0;
    int64_t lo[3], n[3];
    int special;
    PatRowInfo r{0, 0x7fffffff, -1, 0, 0};
    if (!pat_row_box(M, which, gi, di, lo, n, special)) {
        if (special == 1) {
            const int c = (int)(gi - M.ext_begin);
            r = PatRowInfo{1, c, c, c, 1 | (1 << 8) | (1 << 16)};
        }
        if (lane == 0) info[row] = r;
        return;
    }
    const int64_t vol = n[0] * n[1] * n[2], Lxy = M.L[0] * M.L[1];
    int cnt = 0;
    int64_t mn[3] = {INT64_MAX, INT64_MAX, INT64_MAX}, mx[3] = {-1, -1, -1};
    int64_t first = INT64_MAX, last = -1;
    for (int64_t k0 = 0; k0 < vol; k0 += 64) {
        const int64_t k = k0 + lane;
        bool keep = false;
        int64_t q[3] = {0, 0, 0}, j = 0;
        if (k < vol) {
            q[0] = lo[0] + k % n[0];
            q[1] = lo[1] + (k / n[0]) % n[1];
            q[2] = lo[2] + k / (n[0] * n[1]);
            j = q[0] + M.L[0] * q[1] + Lxy * q[2];
            keep = pat_keep(which, di, dir[j - M.ext_begin] != 0);
        }
        cnt += __popcll(__ballot(keep));
        if (keep) {
            for (int d = 0; d < 3; ++d) {
                mn[d] = min(mn[d], q[d]);
                mx[d] = max(mx[d], q[d]);
            }
            first = min(first, j);
            last = max(last, j);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        for (int d = 0; d < 3; ++d) {
            mn[d] = min(mn[d], (int64_t)__shfl_xor(mn[d], o, 64));
            mx[d] = max(mx[d], (int64_t)__shfl_xor(mx[d], o, 64));
        }
        first = min(first, (int64_t)__shfl_xor(first, o, 64));
        last = max(last, (int64_t)__shfl_xor(last, o, 64));
    }
    if (lane) return;
    r.cnt = cnt;
    if (cnt) {
        r.cmin = (int)(first - M.ext_begin);
        r.cmax = (int)(last - M.ext_begin);
        const int64_t bx = mx[0] - mn[0] + 1, by = mx[1] - mn[1] + 1, bz = mx[2] - mn[2] + 1;
        if (bx * by * bz == cnt && bx <= 255 && by <= 255 && bz <= 255) {
            r.box0 = (int)(mn[0] + M.L[0] * mn[1] + Lxy * mn[2] - M.ext_begin);
            r.box1 = (int)(bx | (by << 8) | (bz << 16));
        } else {
            r.box0 = 0;
            r.box1 = -1;
        }
    }
    info[row] = r;
}

__global__ __launch_bounds__(256) void k_pat_fill(MeshDev M, int64_t nrows, int which,
                                                  const uint8_t *__restrict__ dir, const int *__restrict__ rowptr,
                                                  int *__restrict__ bcol)
{
    const int lane = threadIdx.x & 63;
    const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (row >= nrows) return;
    const int64_t gi = M.node_begin + row;
    const bool di = dir[gi - M.ext_begin] != 0;
    int64_t lo[3], n[3];
    int special;
    int *out = bcol + rowptr[row];
    if (!pat_row_box(M, which, gi, di, lo, n, special)) {
        if (special == 1 && lane == 0) out[0] = (int)(gi - M.ext_begin);
        return;
    }
    const int64_t vol = n[0] * n[1] * n[2], Lxy = M.L[0] * M.L[1];
    const uint64_t below = (1ull << lane) - 1ull;
    int pos = 0;
    for (int64_t k0 = 0; k0 < vol; k0 += 64) {
        const int64_t k = k0 + lane;
        bool keep = false;
        int64_t j = 0;
        if (k < vol) {
            j = lo[0] + k % n[0] + M.L[0] * (lo[1] + (k / n[0]) % n[1]) + Lxy * (lo[2] + k / (n[0] * n[1]));
            keep = pat_keep(which, di, dir[j - M.ext_begin] != 0);
        }
        const uint64_t bal = __ballot(keep);
        if (keep) out[pos + __popcll(bal & below)] = (int)(j - M.ext_begin);
        pos += __popcll(bal);
    }
}

// Unstructured meshes: the columns of row i are the sorted unique nodes of
// its incident cells (kle_umesh.cpp umesh_row_nodes), filtered as row_cols.
// One wavefront per row gathers the incident cells' node lists into LDS
// (padded to a power of two), bitonic-sorts them, and keeps the first copy of
// each node that passes the filter (ballot + popcount prefix).  pass 0:
// per-row summary; pass 1: the column list at rowptr[row].
__global__ __launch_bounds__(64) void k_upat(UMeshDev U, int64_t nrows, int which, int P,
                                             const uint8_t *__restrict__ dir, PatRowInfo *__restrict__ info,
                                             const int *__restrict__ rowptr, int *__restrict__ bcol)
{
    extern __shared__ int sc[];
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    if (row >= nrows) return;
    const int il = (int)(row + U.glo);
    const bool di = dir[il] != 0;
    const bool pass1 = bcol != nullptr;
    int *out = pass1 ? bcol + rowptr[row] : nullptr;
    if ((which == 6 && !di) || (which <= 2 && di)) {
        const bool one = which <= 2 && which != 2;
        if (lane == 0) {
            if (pass1) {
                if (one) out[0] = il;
            } else {
                info[row] = one ? PatRowInfo{1, il, il, 0, -1} : PatRowInfo{0, 0x7fffffff, -1, 0, 0};
            }
        }
        return;
    }
    const int ne = U.ne;
    const int64_t q0 = U.incp[row], q1 = U.incp[row + 1];
    const int nc = (int)(q1 - q0) * ne;
    for (int k = lane; k < P; k += 64) {
        int v = 0x7fffffff;
        if (k < nc) {
            const int e = U.inc[q0 + k / ne] / ne;
            v = U.conn[(int64_t)e * ne + k % ne];
        }
        sc[k] = v;
    }
    __syncthreads();
    for (int kk = 2; kk <= P; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < P; i += 64) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int a = sc[i], b = sc[ixj];
                    if ((a > b) == ((i & kk) == 0)) {
                        sc[i] = b;
                        sc[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    const uint64_t below = (1ull << lane) - 1ull;
    int cnt = 0, first = 0x7fffffff, last = -1;
    for (int k0 = 0; k0 < nc; k0 += 64) {
        const int k = k0 + lane;
        bool keep = false;
        int v = 0;
        if (k < nc) {
            v = sc[k];
            keep = (k == 0 || sc[k - 1] != v) && pat_keep(which, di, dir[v] != 0);
        }
        const uint64_t bal = __ballot(keep);
        if (keep) {
            if (pass1) out[cnt + __popcll(bal & below)] = v;
            first = min(first, v);
            last = max(last, v);
        }
        cnt += __popcll(bal);
    }
    if (pass1) return;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        first = min(first, __shfl_xor(first, o, 64));
        last = max(last, __shfl_xor(last, o, 64));
    }
    if (lane == 0) info[row] = PatRowInfo{cnt, first, last, 0, cnt ? -1 : 0};
}

static int upat_lds(const kle_mesh *m)
{
    int64_t mx = 1;
    for (size_t i = 0; i + 1 < m->u_incp.size(); ++i) mx = std::max<int64_t>(mx, m->u_incp[i + 1] - m->u_incp[i]);
    int P = 64;
    while (P < mx * m->nn()) P <<= 1;
    return P;
}

// Per-row pattern summary of `which` on the device (box meshes); dd = device
// copy of m->dir.
static int pattern_rows_dev(kle_ctx *ctx, const kle_mesh *m, int which, const uint8_t *dd,
                            std::vector<PatRowInfo> &info, const UMeshDev *U = nullptr, int P = 0)
{
    const int64_t nrows = m->node_end - m->node_begin;
    info.resize(std::max<int64_t>(nrows, 1));
    if (nrows == 0) return 0;
    PatRowInfo *di = nullptr;
    KLE_HIP(hipMalloc(&di, sizeof(PatRowInfo) * nrows));
    if (m->kind == 1)
        hipLaunchKernelGGL(k_upat, dim3((unsigned)nrows), dim3(64), sizeof(int) * P, ctx->stream, *U, nrows, which, P,
                           dd, di, nullptr, nullptr);
    else
        hipLaunchKernelGGL(k_pat_count, dim3((unsigned)((nrows * 64 + 255) / 256)), dim3(256), 0, ctx->stream,
                           mesh_dev(m), nrows, which, dd, di);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(info.data(), di, sizeof(PatRowInfo) * nrows, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    hipFree(di);
    if (e != hipSuccess) return fail(KLE_ERR_DEVICE, "device pattern count failed: %s", hipGetErrorString(e));
    return 0;
}

// Host-built pattern (unstructured meshes, and box meshes under KLE_HOST_PATTERN=1):
// the same per-row summary plus the explicit column lists.
static int pattern_rows_host(const kle_mesh *m, int which, std::vector<PatRowInfo> &info,
                             std::vector<int64_t> &rp, std::vector<int64_t> &cols)
{
    const int64_t nrows = m->node_end - m->node_begin;
    KLE_TRY(pattern_csr(m, which, rp, cols));
    info.resize(std::max<int64_t>(nrows, 1));
    const int64_t Lx = m->L[0], Lxy = m->L[0] * m->L[1];
    parallel_for(nrows, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t b = rp[i], e = rp[i + 1];
            PatRowInfo r{(int)(e - b), 0x7fffffff, -1, 0, 0};
            if (e > b) {
                const int64_t c0 = cols[b] - m->ext_begin, c1 = cols[e - 1] - m->ext_begin;
                r.cmin = (int)c0;
                r.cmax = (int)c1;
                r.box1 = -1;
                if (m->kind != 0) {  // unstructured: no lattice (and L may be 0)
                    info[i] = r;
                    continue;
                }
                // structured columns: the list must be exactly a lattice box
                const int64_t nx = c1 % Lx - c0 % Lx + 1, ny = (c1 / Lx) % m->L[1] - (c0 / Lx) % m->L[1] + 1,
                              nz = c1 / Lxy - c0 / Lxy + 1;
                bool ok = nx >= 1 && ny >= 1 && nz >= 1 && nx <= 255 && ny <= 255 && nz <= 255 &&
                          nx * ny * nz == e - b;
                int64_t k = b;
                for (int64_t z = 0; ok && z < nz; ++z)
                    for (int64_t y = 0; ok && y < ny; ++y)
                        for (int64_t x = 0; ok && x < nx; ++x, ++k)
                            ok = cols[k] - m->ext_begin == c0 + x + Lx * y + Lxy * z;
                if (ok) {
                    r.box0 = (int)c0;
                    r.box1 = (int)(nx | (ny << 8) | (nz << 16));
                }
            }
            info[i] = r;
        }
    });
    return 0;
}

// Device node-block matrix with the symbolic pattern `which` of the mesh.
int nb_create(kle_ctx *ctx, const kle_mesh *m, int which, int R, int C, kle_mat **out, const UMeshDev *U = nullptr)
{
    const int64_t nrows = m->node_end - m->node_begin;
    PhaseTimer tm(ctx);
    // symbolic pattern on the device (KLE_HOST_PATTERN=1: the host enumeration)
    const char *hp = getenv("KLE_HOST_PATTERN");
    const int P = m->kind == 1 ? upat_lds(m) : 0;
    const bool on_dev = !(hp && atoi(hp) != 0) && P <= 32768;
    UMeshBuf Uloc;
    if (on_dev && m->kind == 1 && !U) {
        KLE_TRY(upload_umesh(ctx, m, Uloc));
        U = &Uloc.dev;
    }
    std::vector<PatRowInfo> info;
    std::vector<int64_t> rp, cols;
    struct DirBuf {
        uint8_t *p = nullptr;
        ~DirBuf() { if (p) (void)hipFree(p); }
    } dirbuf;
    uint8_t *&ddir = dirbuf.p;
    if (on_dev) {
        KLE_HIP(hipMalloc(&ddir, std::max<size_t>(m->dir.size(), 1)));
        KLE_HIP(hipMemcpyAsync(ddir, m->dir.data(), m->dir.size(), hipMemcpyHostToDevice, ctx->stream));
        KLE_TRY(pattern_rows_dev(ctx, m, which, ddir, info, U, P));
    } else {
        KLE_TRY(pattern_rows_host(m, which, info, rp, cols));
    }
    tm.lap(on_dev ? "pattern: device row summary" : "pattern: host enumeration");
    int64_t nb = 0;
    for (int64_t i = 0; i < nrows; ++i) nb += info[i].cnt;
    if (nb >= (1ll << 31)) return fail(KLE_ERR_SUP, "pattern too large for int32 block offsets");
    // structured columns? each row's column list must be exactly a lattice box
    const int64_t Lx = m->L[0], Lxy = m->L[0] * m->L[1];
    bool is_box = nrows > 0 && m->kind == 0;
    std::vector<int> box(2 * std::max<int64_t>(nrows, 1), 0);
    int box_max = 0;
    for (int64_t i = 0; i < nrows && is_box; ++i) {
        if (info[i].box1 < 0) is_box = false;
        box[2 * i] = info[i].box0;
        box[2 * i + 1] = info[i].box1;
        const int b1 = info[i].box1;
        box_max = std::max({box_max, b1 & 255, (b1 >> 8) & 255, (b1 >> 16) & 255});
    }
    const int lay = g_nb_layout;
    // Layout 1 keeps the values' 128-B alignment by chunks (vptr); the column
    // stream of a row is padded to a multiple of 32 int32 (128 B) unless the
    // columns are computed from lattice boxes, so every 64-block pass of the
    // SpMV reads whole 128-B column lines instead of straddling a neighbour's
    // (KLE_BCOL_PAD overrides; 1 = unpadded).
    int pad = lay == 1 ? (is_box ? 1 : 32) : std::max(1, g_nb_pad);
    if (lay == 1)
        if (const char *e = getenv("KLE_BCOL_PAD")) pad = std::max(1, atoi(e));
    std::vector<int> rp32(nrows + 1), cnt(nrows);
    int64_t nbp = 0;
    for (int64_t i = 0; i < nrows; ++i) {
        cnt[i] = info[i].cnt;
        rp32[i] = (int)nbp;
        nbp += (cnt[i] + pad - 1) / pad * pad;
    }
    rp32[nrows] = (int)nbp;
    if (nbp >= (1ll << 31)) return fail(KLE_ERR_SUP, "padded pattern too large for int32 block offsets");
    // interior rows (no ghost column): [int_lo, int_hi) between the last row
    // reading a lower ghost and the first row reading an upper ghost
    // (slab layouts); graph partitions order the ghost-reading rows last, so
    // there the range is [0, first row reading any ghost)
    const int64_t glo = m->node_begin - m->ext_begin;
    int64_t last_lo = -1, first_hi = nrows, first_any = nrows;
    for (int64_t i = 0; i < nrows; ++i) {
        if (!info[i].cnt) continue;
        const bool rl = info[i].cmin < glo, rh = info[i].cmax >= glo + nrows;
        if (rl) last_lo = i;
        if (rh && first_hi == nrows) first_hi = i;
        if ((rl || rh) && first_any == nrows) first_any = i;
    }
    if (first_hi - (last_lo + 1) < first_any) {
        last_lo = -1;
        first_hi = first_any;
    }
    std::vector<int> c32;
    if (!on_dev) {
        c32.assign(std::max<int64_t>(nbp, 1), 0);
        parallel_for(nrows, [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi; ++i)
                for (int64_t k = rp[i]; k < rp[i + 1]; ++k) c32[rp32[i] + (k - rp[i])] = (int)(cols[k] - m->ext_begin);
        });
        std::vector<int64_t>().swap(cols);
    }
    tm.lap("pattern: host row offsets / ranges");
    kle_mat *A = new kle_mat;
    A->ctx = ctx;
    A->kind = 0;
    A->R = R;
    A->C = C;
    A->nrows = nrows;
    A->nblocks = nbp;
    A->nblocks_real = nb;
    A->pad = pad;
    A->vlayout = lay;
    std::vector<int64_t> vptr(nrows + 1, 0);
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t mi = cnt[i];
        vptr[i + 1] = vptr[i] + (lay == 1 ? (mi * R * C + 15) / 16 * 16 : (int64_t)(rp32[i + 1] - rp32[i]) * R * C);
    }
    A->nvals = vptr[nrows];
    A->int_lo = last_lo + 1;
    A->int_hi = first_hi;
    A->box_lx = Lx;
    A->box_lxy = Lxy;
    A->box_max = is_box ? box_max : 0;
    if (const char *e = getenv("KLE_HALO_OVERLAP")) A->halo_overlap = atoi(e) != 0;
    A->node_begin = m->node_begin;
    A->ext_begin = m->ext_begin;
    A->ext_nodes = m->ext_end - m->ext_begin;
    A->m_local = nrows * R;
    A->n_local = nrows * C;
    A->m_global = m->N * R;
    A->n_global = m->N * C;
    A->row_lo = m->node_begin * R;
    A->col_lo = m->node_begin * C;
    if (m->kind == 0) {
        A->row_lat[0] = m->L[0];
        A->row_lat[1] = m->dim == 3 ? m->L[1] : (m->node_end - m->node_begin) / m->L[0];
        A->row_lat[2] = m->dim == 3 ? (m->node_end - m->node_begin) / (m->L[0] * m->L[1]) : 1;
    } else {
        A->row_lat[0] = nrows;
        A->row_lat[1] = A->row_lat[2] = 1;
    }
    A->lo_rank = m->halo_lo_rank;
    A->hi_rank = m->halo_hi_rank;
    A->ghost_lo = (m->node_begin - m->ext_begin) * C;
    A->ghost_hi = (m->ext_end - m->node_end) * C;
    A->send_lo = m->send_lo_nodes * C;
    A->send_hi = m->send_hi_nodes * C;
    A->plan = m->plan;
    A->ext_gid = m->ext_gid;
    A->diag_only_row.assign(nrows, 0);
    if (which <= 1)
        for (int64_t i = 0; i < nrows; ++i) A->diag_only_row[i] = m->dir[m->node_begin + i - m->ext_begin];
    if (hipMalloc(&A->d_rowptr, sizeof(int) * (nrows + 1)) != hipSuccess ||
        (pad > 1 && hipMalloc(&A->d_rowcnt, sizeof(int) * std::max<int64_t>(nrows, 1)) != hipSuccess) ||
        hipMalloc(&A->d_bcol, sizeof(int) * std::max<int64_t>(nbp, 1)) != hipSuccess ||
        hipMalloc(&A->d_vptr, sizeof(int64_t) * (nrows + 1)) != hipSuccess ||
        big_alloc(reinterpret_cast<void **>(&A->d_val), sizeof(double) * std::max<int64_t>(A->nvals, 1)) < 0) {
        kle_mat_destroy(A);
        return fail(KLE_ERR_MEM, "out of device memory for a %lld-block matrix", (long long)nb);
    }
    KLE_HIP(hipMemcpyAsync(A->d_rowptr, rp32.data(), sizeof(int) * (nrows + 1), hipMemcpyHostToDevice,
                           ctx->stream));
    if (on_dev) {
        KLE_HIP(hipMemsetAsync(A->d_bcol, 0, sizeof(int) * std::max<int64_t>(nbp, 1), ctx->stream));
        if (nrows && m->kind == 1)
            hipLaunchKernelGGL(k_upat, dim3((unsigned)nrows), dim3(64), sizeof(int) * P, ctx->stream, *U, nrows, which,
                               P, ddir, nullptr, A->d_rowptr, A->d_bcol);
        else if (nrows)
            hipLaunchKernelGGL(k_pat_fill, dim3((unsigned)((nrows * 64 + 255) / 256)), dim3(256), 0, ctx->stream,
                               mesh_dev(m), nrows, which, ddir, A->d_rowptr, A->d_bcol);
        KLE_HIP(hipGetLastError());
    } else {
        KLE_HIP(hipMemcpyAsync(A->d_bcol, c32.data(), sizeof(int) * std::max<int64_t>(nbp, 1),
                               hipMemcpyHostToDevice, ctx->stream));
    }
    if (A->d_rowcnt)
        KLE_HIP(hipMemcpyAsync(A->d_rowcnt, cnt.data(), sizeof(int) * std::max<int64_t>(nrows, 1), hipMemcpyHostToDevice,
                               ctx->stream));
    KLE_HIP(hipMemcpyAsync(A->d_vptr, vptr.data(), sizeof(int64_t) * (nrows + 1), hipMemcpyHostToDevice, ctx->stream));
    // (always zeroed: not every fill writes every slot -- pad blocks, chunk
    // tails, pattern entries no element touches -- and recycled device memory
    // is not zero)
    KLE_HIP(hipMemsetAsync(A->d_val, 0, sizeof(double) * std::max<int64_t>(A->nvals, 1), ctx->stream));
    if (is_box) {
        KLE_HIP(hipMalloc(&A->d_rowbox, sizeof(int) * 2 * nrows));
        KLE_HIP(hipMemcpyAsync(A->d_rowbox, box.data(), sizeof(int) * 2 * nrows, hipMemcpyHostToDevice, ctx->stream));
    }
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    tm.lap("matrix alloc + uploads + column fill");
    if (!is_box && R == 3 && C == 3 && lay == 1 && nrows >= g_tune.spmv_dict_min_rows) {
        const int rc = nb_build_dict(A);
        if (rc) {
            kle_mat_destroy(A);
            return rc;
        }
        tm.lap("column dictionaries");
    }
    *out = A;
    return 0;
}

struct DevTables {
    double *buf = nullptr;
    Tables1D F, R, O;
    ~DevTables() { hipFree(buf); }
};

static int upload_tables(kle_ctx *ctx, int ngl, DevTables &T)
{
    PointSet1D full, red, op;
    element_sets(ngl, full, red, op);
    std::vector<double> h;
    auto put = [&](const std::vector<double> &v) {
        size_t o = h.size();
        h.insert(h.end(), v.begin(), v.end());
        return o;
    };
    size_t fx = put(full.x), fw = put(full.w), fh = put(full.h), fd = put(full.dh);
    size_t rx = put(red.x), rw = put(red.w), rh = put(red.h), rd = put(red.dh);
    size_t ox = put(op.x), ow = put(op.w), oh = put(op.h), od = put(op.dh);
    KLE_HIP(hipMalloc(&T.buf, sizeof(double) * h.size()));
    KLE_HIP(hipMemcpyAsync(T.buf, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice, ctx->stream));
    T.F = {(int)full.x.size(), T.buf + fx, T.buf + fw, T.buf + fh, T.buf + fd};
    T.R = {(int)red.x.size(), T.buf + rx, T.buf + rw, T.buf + rh, T.buf + rd};
    T.O = {(int)op.x.size(), T.buf + ox, T.buf + ow, T.buf + oh, T.buf + od};
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

// Element-matrix pipeline: tables, corners and the Gauss-point geometry of
// every local element once (ElemSetup), then K_e / Rw_e (/ Rd_e) of any
// contiguous range of local elements (element_batch, outputs indexed e - e0).
struct ElemSetup {
    DevTables T;
    double *dX = nullptr, *gF = nullptr, *gR = nullptr;
    int nqF = 0, nqR = 0;
    int64_t nel = 0;
    bool valu = false;
    int minw = 3;  // k_element_mfma register budget: 3 (default) or 2 waves / SIMD (KLE_ELEMENT_WAVES)
    ~ElemSetup()
    {
        if (dX) (void)hipFree(dX);
        if (gF) (void)hipFree(gF);
        if (gR) (void)hipFree(gR);
    }
};

static int element_setup(kle_ctx *ctx, const kle_mesh *m, ElemSetup &S)
{
    const int dim = m->dim, nc = 1 << dim, G1 = 1 + dim * dim;
    const int64_t nel = m->elem_end - m->elem_begin;
    S.nel = nel;
    KLE_TRY(upload_tables(ctx, m->ngl, S.T));
    std::vector<double> corners(std::max<int64_t>(nel * nc * dim, 1));
    KLE_TRY(kle_mesh_get_corners(m, corners.data()));
    S.nqF = dim == 2 ? S.T.F.np1 * S.T.F.np1 : S.T.F.np1 * S.T.F.np1 * S.T.F.np1;
    S.nqR = dim == 2 ? S.T.R.np1 * S.T.R.np1 : S.T.R.np1 * S.T.R.np1 * S.T.R.np1;
    KLE_HIP(hipMalloc(&S.dX, sizeof(double) * corners.size()));
    KLE_HIP(hipMalloc(&S.gF, sizeof(double) * std::max<int64_t>(nel * S.nqF * G1, 1)));
    KLE_HIP(hipMalloc(&S.gR, sizeof(double) * std::max<int64_t>(nel * S.nqR * G1, 1)));
    KLE_HIP(hipMemcpyAsync(S.dX, corners.data(), sizeof(double) * corners.size(), hipMemcpyHostToDevice,
                           ctx->stream));
    const int64_t nF = nel * S.nqF, nR = nel * S.nqR;
    if (nel > 0) {
        if (dim == 2) {
            hipLaunchKernelGGL(k_geometry<2>, dim3((nF + 255) / 256), dim3(256), 0, ctx->stream, nel, m->ngl, S.T.F, S.dX, S.gF);
            hipLaunchKernelGGL(k_geometry<2>, dim3((nR + 255) / 256), dim3(256), 0, ctx->stream, nel, m->ngl, S.T.R, S.dX, S.gR);
        } else {
            hipLaunchKernelGGL(k_geometry<3>, dim3((nF + 255) / 256), dim3(256), 0, ctx->stream, nel, m->ngl, S.T.F, S.dX, S.gF);
            hipLaunchKernelGGL(k_geometry<3>, dim3((nR + 255) / 256), dim3(256), 0, ctx->stream, nel, m->ngl, S.T.R, S.dX, S.gR);
        }
        KLE_HIP(hipGetLastError());
    }
    // KLE_ELEMENT_VALU=1: the FP64-VALU element kernel instead of the MFMA one
    const char *ev = getenv("KLE_ELEMENT_VALU");
    S.valu = ev && atoi(ev) != 0;
    if (const char *w = getenv("KLE_ELEMENT_WAVES")) S.minw = atoi(w) == 2 ? 2 : 3;
    return 0;
}

static int element_batch(kle_ctx *ctx, const kle_mesh *m, const ElemSetup &S, int64_t e0, int64_t cnt, double *Ke,
                         double *Rwe, double *Rde)
{
    if (cnt <= 0) return 0;
    const int dim = m->dim, ne = m->nn(), G1 = 1 + dim * dim;
    const double *gF = S.gF + e0 * S.nqF * G1, *gR = S.gR + e0 * S.nqR * G1;
    dim3 eg((ne + TL - 1) / TL, (ne + TL - 1) / TL, (unsigned)cnt);
#define KLE_ELEM_LAUNCH(KERN) \
    hipLaunchKernelGGL(KERN, eg, dim3(256), 0, ctx->stream, m->ngl, S.T.F, S.T.R, gF, gR, Ke, Rwe, Rde)
    if (dim == 2) {
        if (S.valu) KLE_ELEM_LAUNCH(k_element<2>);
        else if (S.minw == 3) KLE_ELEM_LAUNCH((k_element_mfma<2, 3>));
        else KLE_ELEM_LAUNCH((k_element_mfma<2, 2>));
    } else {
        if (S.valu) KLE_ELEM_LAUNCH(k_element<3>);
        else if (S.minw == 3) KLE_ELEM_LAUNCH((k_element_mfma<3, 3>));
        else KLE_ELEM_LAUNCH((k_element_mfma<3, 2>));
    }
#undef KLE_ELEM_LAUNCH
    KLE_HIP(hipGetLastError());
    return 0;
}

// K_e and Rw_e (and Rd_e) of all local elements into new device buffers.
static int element_matrices(kle_ctx *ctx, const kle_mesh *m, double **dKe, double **dRwe, double **dRde = nullptr)
{
    const int dim = m->dim, ne = m->nn(), dw = dim == 2 ? 1 : 3;
    PhaseTimer tm(ctx);
    ElemSetup S;
    KLE_TRY(element_setup(ctx, m, S));
    const int64_t nel = S.nel;
    const size_t keN = (size_t)nel * ne * ne * dim * dim, rwN = (size_t)nel * ne * ne * dim * dw;
    *dKe = *dRwe = nullptr;
    if (hipMalloc(dKe, sizeof(double) * std::max<size_t>(keN, 1)) != hipSuccess ||
        hipMalloc(dRwe, sizeof(double) * std::max<size_t>(rwN, 1)) != hipSuccess) {
        if (*dKe) hipFree(*dKe);
        return fail(KLE_ERR_MEM, "element matrix workspace (%.2f GB) does not fit", (keN + rwN) * 8.0 / 1e9);
    }
    if (dRde && hipMalloc(dRde, sizeof(double) * std::max<size_t>((size_t)nel * ne * ne * dim, 1)) != hipSuccess) {
        hipFree(*dKe);
        hipFree(*dRwe);
        return fail(KLE_ERR_MEM, "element Rd workspace does not fit");
    }
    KLE_TRY(element_batch(ctx, m, S, 0, nel, *dKe, *dRwe, dRde ? *dRde : nullptr));
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    tm.lap(S.valu ? "element: geometry + k_element (VALU)" : "element: geometry + k_element_mfma");
    return 0;
}


// ---------------------------------------------------------------- operators
// Operators (mat_fs.py:194-271, spectral.py:162-228) are collocation operators
// on the GLL nodes: at op point l of cell e only node l's basis is nonzero
// (H = delta), so the element block of (row node n = local l, col node m) is
//   c_{e,l} * B_{e,l}[a][(m, b)],  c = w_l det J,  Hxy = inv(J) dN_m/dxi at l,
// with B_curl / B_srt / B_div the sparse maps of spectral.py:205-228.
// dN_m/dxi_k at node l is D[l_k][m_k] when m and l agree on the other axes,
// else exactly 0.  The global entry is the ascending-cell sum of those blocks
// times 1/W_n, W_n = sum_e c_{e,l(n)} (Vec.reciprocal + diagonalScale(L)).
struct OpsOut {
    double *curl, *srt, *div;
    const int *rp_c, *rp_s, *rp_d;        // block row offsets (padded) of each matrix
    const int64_t *vp_c, *vp_s, *vp_d;    // value row offsets
    int lay;
};

template <int DIM>
__global__ __launch_bounds__(256) void k_ops_weights(MeshDev M, int64_t nrows, const double *__restrict__ geo,
                                                     double *__restrict__ winv)
{
    const int64_t row = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    constexpr int G1 = 1 + DIM * DIM;
    const int64_t gi = M.node_begin + row;
    const int64_t ci[3] = {gi % M.L[0], (gi / M.L[0]) % M.L[1], DIM == 3 ? gi / (M.L[0] * M.L[1]) : 0};
    int64_t elo[3] = {0, 0, 0}, ehi[3] = {0, 0, 0};
    for (int d = 0; d < DIM; ++d) {
        elo[d] = (ci[d] % M.p == 0) ? max((int64_t)0, ci[d] / M.p - 1) : ci[d] / M.p;
        ehi[d] = min(M.nel[d] - 1, ci[d] / M.p);
    }
    double W = 0.0;
    for (int64_t ez = elo[2]; ez <= ehi[2]; ++ez)
        for (int64_t ey = elo[1]; ey <= ehi[1]; ++ey)
            for (int64_t ex = elo[0]; ex <= ehi[0]; ++ex) {
                const int64_t eo[3] = {ex * M.p, ey * M.p, ez * M.p};
                int l = 0;
                for (int d = DIM - 1; d >= 0; --d) l = l * M.ngl + (int)(ci[d] - eo[d]);
                const int64_t e = ex + M.nel[0] * (ey + M.nel[1] * ez) - M.elem_begin;
                W += geo[(e * M.ne + l) * G1];
            }
    winv[row] = 1.0 / W;
}

template <int DIM>
__global__ __launch_bounds__(256) void k_ops_gather(MeshDev M, int64_t nrows, const int *__restrict__ rowcnt,
                                                    const int *__restrict__ bcol, const double *__restrict__ geo,
                                                    const double *__restrict__ dh, const double *__restrict__ winv,
                                                    OpsOut out)
{
    constexpr int DW = DIM == 2 ? 1 : 3, DS = DIM == 2 ? 3 : 6, G1 = 1 + DIM * DIM;
    const int lane = threadIdx.x & 63;
    const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (row >= nrows) return;
    const int64_t gi = M.node_begin + row;
    const int m = rowcnt[row];
    const int bc0 = out.rp_c[row];  // block offset in the (shared) column list
    const int64_t ci[3] = {gi % M.L[0], (gi / M.L[0]) % M.L[1], DIM == 3 ? gi / (M.L[0] * M.L[1]) : 0};
    int64_t elo[3] = {0, 0, 0}, ehi[3] = {0, 0, 0};
    for (int d = 0; d < DIM; ++d) {
        elo[d] = (ci[d] % M.p == 0) ? max((int64_t)0, ci[d] / M.p - 1) : ci[d] / M.p;
        ehi[d] = min(M.nel[d] - 1, ci[d] / M.p);
    }
    const double wi = winv[row];
    const int mpc = out.rp_c[row + 1] - out.rp_c[row], mps = out.rp_s[row + 1] - out.rp_s[row],
              mpd = out.rp_d[row + 1] - out.rp_d[row];
    double *vc = out.curl + out.vp_c[row];
    double *vs = out.srt + out.vp_s[row];
    double *vd = out.div + out.vp_d[row];
    for (int k = lane; k < m; k += 64) {
        const int64_t gj = M.ext_begin + bcol[bc0 + k];
        const int64_t cj[3] = {gj % M.L[0], (gj / M.L[0]) % M.L[1], DIM == 3 ? gj / (M.L[0] * M.L[1]) : 0};
        double C[DW * DIM], S[DS * DIM], D[DIM * DS];
        for (int t = 0; t < DW * DIM; ++t) C[t] = 0.0;
        for (int t = 0; t < DS * DIM; ++t) S[t] = D[t] = 0.0;
        for (int64_t ez = elo[2]; ez <= ehi[2]; ++ez)
            for (int64_t ey = elo[1]; ey <= ehi[1]; ++ey)
                for (int64_t ex = elo[0]; ex <= ehi[0]; ++ex) {
                    const int64_t eo[3] = {ex * M.p, ey * M.p, ez * M.p};
                    int oi[3] = {0, 0, 0}, oj[3] = {0, 0, 0};
                    bool in = true;
                    for (int d = 0; d < DIM; ++d) {
                        const int64_t o = cj[d] - eo[d];
                        in = in && o >= 0 && o <= M.p;
                        oj[d] = (int)o;
                        oi[d] = (int)(ci[d] - eo[d]);
                    }
                    if (!in) continue;
                    int l = 0;
                    for (int d = DIM - 1; d >= 0; --d) l = l * M.ngl + oi[d];
                    const int64_t e = ex + M.nel[0] * (ey + M.nel[1] * ez) - M.elem_begin;
                    const double *g = geo + (e * M.ne + l) * G1;
                    const double c = g[0];
                    double Hrs[DIM];
                    for (int kk = 0; kk < DIM; ++kk) {
                        bool line = true;
                        for (int j = 0; j < DIM; ++j)
                            if (j != kk) line = line && oj[j] == oi[j];
                        Hrs[kk] = line ? dh[oi[kk] * M.ngl + oj[kk]] : 0.0;
                    }
                    double H[DIM];
                    for (int d = 0; d < DIM; ++d) {
                        double acc = 0.0;
                        for (int kk = 0; kk < DIM; ++kk) acc += g[1 + d * DIM + kk] * Hrs[kk];
                        H[d] = acc;
                    }
                    if constexpr (DIM == 3) {
                        // curl: indCurl (spectral.py:31), signs (-1)^i
                        C[0 * 3 + 2] += c * H[1];
                        C[0 * 3 + 1] += c * -H[2];
                        C[1 * 3 + 0] += c * H[2];
                        C[1 * 3 + 2] += c * -H[0];
                        C[2 * 3 + 1] += c * H[0];
                        C[2 * 3 + 0] += c * -H[1];
                        // strain rate xx,xy,yy,yz,zz,zx (B_srt *= 0.5, spectral.py:209-220)
                        S[0 * 3 + 0] += c * H[0];
                        S[1 * 3 + 1] += c * (0.5 * H[0]);
                        S[5 * 3 + 2] += c * (0.5 * H[0]);
                        S[2 * 3 + 1] += c * H[1];
                        S[1 * 3 + 0] += c * (0.5 * H[1]);
                        S[3 * 3 + 2] += c * (0.5 * H[1]);
                        S[4 * 3 + 2] += c * H[2];
                        S[5 * 3 + 0] += c * (0.5 * H[2]);
                        S[3 * 3 + 1] += c * (0.5 * H[2]);
                        // divergence of the symmetric tensor: indBdiv (spectral.py:33)
                        D[0 * 6 + 0] += c * H[0];
                        D[0 * 6 + 1] += c * H[1];
                        D[0 * 6 + 5] += c * H[2];
                        D[1 * 6 + 1] += c * H[0];
                        D[1 * 6 + 2] += c * H[1];
                        D[1 * 6 + 3] += c * H[2];
                        D[2 * 6 + 5] += c * H[0];
                        D[2 * 6 + 3] += c * H[1];
                        D[2 * 6 + 4] += c * H[2];
                    } else {
                        C[1] += c * H[0];  // indCurl 2-D (spectral.py:27)
                        C[0] += c * -H[1];
                        S[0 * 2 + 0] += c * H[0];
                        S[1 * 2 + 1] += c * (0.5 * H[0]);
                        S[2 * 2 + 1] += c * H[1];
                        S[1 * 2 + 0] += c * (0.5 * H[1]);
                        D[0 * 3 + 0] += c * H[0];
                        D[0 * 3 + 1] += c * H[1];
                        D[1 * 3 + 1] += c * H[0];
                        D[1 * 3 + 2] += c * H[1];
                    }
                }
        for (int t = 0; t < DW * DIM; ++t) vc[vofs(out.lay, DW * DIM, t, k, m, mpc)] = C[t] * wi;
        for (int t = 0; t < DS * DIM; ++t) vs[vofs(out.lay, DS * DIM, t, k, m, mps)] = S[t] * wi;
        for (int t = 0; t < DIM * DS; ++t) vd[vofs(out.lay, DIM * DS, t, k, m, mpd)] = D[t] * wi;
    }
}


// ---------------------------------------------------------------- no-slip
// MatNS.buildNS (mat_ns.py:47-145) on the device.  DoF classes F (free),
// T (tangential), N (normal) per velocity DoF (ext range, cls[]).  Per entry
// (row DoF r, col DoF c) the ascending-cell sum S of the element blocks:
//   MODE 3 Kfs    : S on (T,F),(F,T),(T,T); T diagonal S + (-1)   (:104-116,124-125)
//   MODE 4 Krhsfs : -S on (F|T, N); N diagonal 1 (INSERT)        (:118-122,130-131)
//   MODE 5 Rwfs   : S of Rw_e on T rows                          (:110-111)
//   MODE 6 K+Kfs  : S on (F|T, F|T); T diagonal 1 + (S + (-1)); N diagonal 1
//                   (the matrix KleSolver.setUp hands to solverFS, kle_solver.py:25)
// Entries outside those sets are stored as exact zeros (node blocks) and
// left out of the exported CSR (kle_mat.mask_rule).
// Write the accumulated block (row node il, column node jl, ext-local) with
// the MODE's DoF-class rule.
template <int R, int C, int MODE>
__device__ __forceinline__ void store_ns(double *v, int lay, int k, int m, int mp, const double *acc, int64_t il,
                                         int64_t jl, const uint8_t *__restrict__ cls)
{
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < C; ++b) {
            const int rc = cls[il * R + a];
            const int cc = MODE == 5 ? DOF_FREE : cls[jl * C + b];
            const bool diag = jl == il && a == b;
            const int rule = MODE == 3 ? MASK_KFS : MODE == 4 ? MASK_KRHSFS : MODE == 5 ? MASK_TANG_ROWS : MASK_KSUM;
            double out = mask_entry(rule, rc, cc, diag) ? acc[a * C + b] : 0.0;
            if (diag) {
                if (MODE == 3 && rc == DOF_TANG) out = acc[a * C + b] + (-1.0);
                if (MODE == 4 && rc == DOF_NORMAL) out = 1.0;
                if (MODE == 6 && rc == DOF_TANG) out = 1.0 + (acc[a * C + b] + (-1.0));
                if (MODE == 6 && rc == DOF_NORMAL) out = 1.0;
            }
            v[vofs(lay, R * C, a * C + b, k, m, mp)] = out;
        }
}

template <int R, int C, int MODE>
__global__ __launch_bounds__(256) void k_gather_ns(MeshDev M, int64_t nrows, const int *__restrict__ rowptr,
                                                   const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr,
                                                   int lay, const int *__restrict__ bcol,
                                                   const uint8_t *__restrict__ cls, const double *__restrict__ Eblk,
                                                   double *__restrict__ val)
{
    const int lane = threadIdx.x & 63;
    const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (row >= nrows) return;
    const int64_t gi = M.node_begin + row, il = gi - M.ext_begin;
    const int b0 = rowptr[row], mp = rowptr[row + 1] - b0, m = rowcnt ? rowcnt[row] : mp;
    double *v = val + vptr[row];
    int64_t ci[3] = {gi % M.L[0], (gi / M.L[0]) % M.L[1], M.dim == 3 ? gi / (M.L[0] * M.L[1]) : 0};
    int64_t elo[3], ehi[3];
    for (int d = 0; d < 3; ++d) {
        if (d >= M.dim) {
            elo[d] = ehi[d] = 0;
            continue;
        }
        const int64_t c = ci[d];
        elo[d] = (c % M.p == 0) ? max((int64_t)0, c / M.p - 1) : c / M.p;
        ehi[d] = min(M.nel[d] - 1, c / M.p);
    }
    const int ngl = M.ngl, ne = M.ne;
    for (int k = lane; k < m; k += 64) {
        const int64_t jl = bcol[b0 + k], gj = M.ext_begin + jl;
        int64_t cj[3] = {gj % M.L[0], (gj / M.L[0]) % M.L[1], M.dim == 3 ? gj / (M.L[0] * M.L[1]) : 0};
        double acc[R * C];
#pragma unroll
        for (int t = 0; t < R * C; ++t) acc[t] = 0.0;
        for (int64_t ez = elo[2]; ez <= ehi[2]; ++ez)
            for (int64_t ey = elo[1]; ey <= ehi[1]; ++ey)
                for (int64_t ex = elo[0]; ex <= ehi[0]; ++ex) {
                    const int64_t eo[3] = {ex * M.p, ey * M.p, ez * M.p};
                    bool in = true;
                    int oj[3] = {0, 0, 0}, oi[3] = {0, 0, 0};
                    for (int d = 0; d < M.dim; ++d) {
                        const int64_t o = cj[d] - eo[d];
                        in = in && o >= 0 && o <= M.p;
                        oj[d] = (int)o;
                        oi[d] = (int)(ci[d] - eo[d]);
                    }
                    if (!in) continue;
                    const int64_t e = ex + M.nel[0] * (ey + M.nel[1] * ez) - M.elem_begin;
                    const int li = oi[0] + ngl * (oi[1] + ngl * oi[2]);
                    const int lj = oj[0] + ngl * (oj[1] + ngl * oj[2]);
                    const double *blk = Eblk + ((e * ne + li) * (int64_t)ne + lj) * (R * C);
#pragma unroll
                    for (int t = 0; t < R * C; ++t) acc[t] += (MODE == 4) ? -blk[t] : blk[t];
                }
        store_ns<R, C, MODE>(v, lay, k, m, mp, acc, il, jl, cls);
    }
}

template <int R, int C, int MODE>
static void launch_gather_ns(kle_ctx *ctx, const MeshDev &M, kle_mat *A, const uint8_t *cls, const double *E)
{
    const int64_t threads = A->nrows * 64;
    hipLaunchKernelGGL((k_gather_ns<R, C, MODE>), dim3((threads + 255) / 256), dim3(256), 0, ctx->stream, M,
                       A->nrows, A->d_rowptr, A->d_rowcnt, A->d_vptr, A->vlayout, A->d_bcol, cls, E, A->d_val);
}

template <int R, int C, int MODE>
static void launch_gather(kle_ctx *ctx, const MeshDev &M, kle_mat *A, const uint8_t *dir, const double *E,
                          int64_t eb0 = 0, int64_t eb1 = INT64_MAX, int accum = 0)
{
    const int64_t threads = A->nrows * 64;
    hipLaunchKernelGGL((k_gather<R, C, MODE>), dim3((threads + 255) / 256), dim3(256), 0, ctx->stream, M,
                       A->nrows, A->d_rowptr, A->d_rowcnt, A->d_vptr, A->vlayout, A->d_bcol, dir, E, A->d_val,
                       eb0, eb1, accum);
}

// ------------------------------------------------------- unstructured
// Unstructured meshes (kle_umesh.cpp) have no lattice to enumerate a row's
// cells, so the gather walks the row's incidence list instead: one 64-lane
// workgroup per node row, the row's incident (cell, local node) pairs in
// ascending cell order, lanes over the cell's nodes.  Each lane finds its
// column in the row's sorted column list (binary search; columns outside the
// pattern -- e.g. Dirichlet columns of K -- are skipped, which is the
// pattern's own filter) and adds the element block into an LDS window of
// UW block accumulators.  Within one cell the lanes hit distinct columns;
// cells are separated by a barrier, so every entry is the ascending-cell sum
// starting from 0, exactly as the lattice kernels and PETSc's ADD order.

constexpr int UW = 256;

__device__ __forceinline__ int find_col(const int *__restrict__ cols, int lo, int hi, int j)
{
    // cols[lo, hi) ascending; -1 if absent
    --hi;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const int c = cols[mid];
        if (c == j) return mid;
        if (c < j) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

// MODE as k_gather (0 K, 1 Krhs, 2 Rw) and k_gather_ns (3 Kfs, 4 Krhsfs, 5 Rwfs / Rdfs, 6 K+Kfs)
template <int R, int C, int MODE>
__global__ __launch_bounds__(64) void k_gather_u(UMeshDev U, int64_t nrows, const int *__restrict__ rowptr,
                                                 const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr,
                                                 int lay, const int *__restrict__ bcol,
                                                 const uint8_t *__restrict__ dir, const uint8_t *__restrict__ cls,
                                                 const double *__restrict__ Eblk, double *__restrict__ val,
                                                 int64_t eb0, int64_t eb1, int accum)
{
    constexpr int RC = R * C;
    __shared__ double acc[UW * RC];
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    if (row >= nrows) return;
    const int64_t il = row + U.glo;
    const int b0 = rowptr[row], mp = rowptr[row + 1] - b0, m = rowcnt ? rowcnt[row] : mp;
    double *v = val + vptr[row];
    const int *cols = bcol + b0;
    if (MODE <= 2 && dir[il]) {
        // K[dir,dir] = 0 + ... + 0 + 1 and Krhs[dir,dir] = 1 (mat_fs.py:115-120,182-183)
        if (MODE != 2 && lane == 0 && m == 1 && eb0 == 0)
            for (int a = 0; a < R; ++a)
                for (int b = 0; b < C; ++b) v[vofs(lay, RC, a * C + b, 0, m, mp)] = (a == b) ? 1.0 : 0.0;
        return;
    }
    const int ne = U.ne;
    const int64_t q0 = U.incp[row], q1 = U.incp[row + 1];
    // element batch [eb0, eb1): the incidence list ascends in e
    if (q0 == q1 || U.inc[q1 - 1] / ne < eb0 || U.inc[q0] / ne >= eb1) return;
    for (int w0 = 0; w0 < m; w0 += UW) {
        const int wn = min(UW, m - w0);
        for (int t = lane; t < wn * RC; t += 64) acc[t] = accum ? v[vofs(lay, RC, t % RC, w0 + t / RC, m, mp)] : 0.0;
        __syncthreads();
        for (int64_t q = q0; q < q1; ++q) {
            const int ei = U.inc[q];
            const int e = ei / ne, li = ei - e * ne;
            if (e < eb0 || e >= eb1) continue;  // uniform over the workgroup
            const int *ce = U.conn + (int64_t)e * ne;
            for (int lj = lane; lj < ne; lj += 64) {
                const int pos = find_col(cols, w0, w0 + wn, ce[lj]);
                if (pos < 0) continue;
                const double *blk = Eblk + (((int64_t)(e - eb0) * ne + li) * ne + lj) * RC;
                double *a = acc + (pos - w0) * RC;
#pragma unroll
                for (int t = 0; t < RC; ++t) a[t] += (MODE == 1 || MODE == 4) ? -blk[t] : blk[t];
            }
            __syncthreads();
        }
        for (int k = lane; k < wn; k += 64) {
            const double *a = acc + k * RC;
            if constexpr (MODE <= 2) {
#pragma unroll
                for (int t = 0; t < RC; ++t) v[vofs(lay, RC, t, w0 + k, m, mp)] = a[t];
            } else {
                double blk[RC];
#pragma unroll
                for (int t = 0; t < RC; ++t) blk[t] = a[t];
                store_ns<R, C, MODE>(v, lay, w0 + k, m, mp, blk, il, cols[w0 + k], cls);
            }
        }
        __syncthreads();
    }
}

template <int DIM>
__global__ __launch_bounds__(256) void k_ops_weights_u(UMeshDev U, int64_t nrows, const double *__restrict__ geo,
                                                       double *__restrict__ winv)
{
    const int64_t row = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    constexpr int G1 = 1 + DIM * DIM;
    double W = 0.0;
    for (int64_t q = U.incp[row]; q < U.incp[row + 1]; ++q) W += geo[(int64_t)U.inc[q] * G1];
    winv[row] = 1.0 / W;
}

// Collocation operators on an unstructured mesh: per incident (cell, li) only
// the nodes on the DIM tensor lines through li carry a nonzero block (the
// other entries of the element block are exact zeros, which do not change an
// ascending sum), so lanes take the DIM*ngl line candidates.  Block values as
// k_ops_gather.
constexpr int UWO = 128;
template <int DIM>
__global__ __launch_bounds__(64) void k_ops_gather_u(UMeshDev U, int ngl, int64_t nrows, const int *__restrict__ rowcnt,
                                                     const int *__restrict__ bcol, const double *__restrict__ geo,
                                                     const double *__restrict__ dh, const double *__restrict__ winv,
                                                     OpsOut out)
{
    constexpr int DW = DIM == 2 ? 1 : 3, DS = DIM == 2 ? 3 : 6, G1 = 1 + DIM * DIM;
    constexpr int NC = DW * DIM, NS = DS * DIM, ND = DIM * DS, NB = NC + NS + ND;
    __shared__ double acc[UWO * NB];
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    if (row >= nrows) return;
    const int m = rowcnt[row];
    const int *cols = bcol + out.rp_c[row];
    const double wi = winv[row];
    const int mpc = out.rp_c[row + 1] - out.rp_c[row], mps = out.rp_s[row + 1] - out.rp_s[row],
              mpd = out.rp_d[row + 1] - out.rp_d[row];
    double *vc = out.curl + out.vp_c[row];
    double *vs = out.srt + out.vp_s[row];
    double *vd = out.div + out.vp_d[row];
    const int ne = U.ne;
    const int64_t q0 = U.incp[row], q1 = U.incp[row + 1];
    for (int w0 = 0; w0 < m; w0 += UWO) {
        const int wn = min(UWO, m - w0);
        for (int t = lane; t < wn * NB; t += 64) acc[t] = 0.0;
        __syncthreads();
        for (int64_t q = q0; q < q1; ++q) {
            const int ei = U.inc[q];
            const int e = ei / ne, li = ei - e * ne;
            int oi[3] = {li % ngl, (li / ngl) % ngl, DIM == 3 ? li / (ngl * ngl) : 0};
            for (int cand = lane; cand < DIM * ngl; cand += 64) {
                const int ax = cand / ngl, t = cand - ax * ngl;
                if (ax > 0 && t == oi[ax]) continue;  // the row node itself: taken once, on axis 0
                int oj[3] = {oi[0], oi[1], oi[2]};
                oj[ax] = t;
                const int lj = oj[0] + ngl * (oj[1] + ngl * oj[2]);
                const int pos = find_col(cols, w0, w0 + wn, U.conn[(int64_t)e * ne + lj]);
                if (pos < 0) continue;
                const double *g = geo + ((int64_t)e * ne + li) * G1;
                const double c = g[0];
                double Hrs[DIM];
                for (int kk = 0; kk < DIM; ++kk) {
                    bool line = true;
                    for (int j = 0; j < DIM; ++j)
                        if (j != kk) line = line && oj[j] == oi[j];
                    Hrs[kk] = line ? dh[oi[kk] * ngl + oj[kk]] : 0.0;
                }
                double H[DIM];
                for (int d = 0; d < DIM; ++d) {
                    double s = 0.0;
                    for (int kk = 0; kk < DIM; ++kk) s += g[1 + d * DIM + kk] * Hrs[kk];
                    H[d] = s;
                }
                double *Cc = acc + (pos - w0) * NB, *S = Cc + NC, *D = S + NS;
                if constexpr (DIM == 3) {
                    Cc[0 * 3 + 2] += c * H[1];
                    Cc[0 * 3 + 1] += c * -H[2];
                    Cc[1 * 3 + 0] += c * H[2];
                    Cc[1 * 3 + 2] += c * -H[0];
                    Cc[2 * 3 + 1] += c * H[0];
                    Cc[2 * 3 + 0] += c * -H[1];
                    S[0 * 3 + 0] += c * H[0];
                    S[1 * 3 + 1] += c * (0.5 * H[0]);
                    S[5 * 3 + 2] += c * (0.5 * H[0]);
                    S[2 * 3 + 1] += c * H[1];
                    S[1 * 3 + 0] += c * (0.5 * H[1]);
                    S[3 * 3 + 2] += c * (0.5 * H[1]);
                    S[4 * 3 + 2] += c * H[2];
                    S[5 * 3 + 0] += c * (0.5 * H[2]);
                    S[3 * 3 + 1] += c * (0.5 * H[2]);
                    D[0 * 6 + 0] += c * H[0];
                    D[0 * 6 + 1] += c * H[1];
                    D[0 * 6 + 5] += c * H[2];
                    D[1 * 6 + 1] += c * H[0];
                    D[1 * 6 + 2] += c * H[1];
                    D[1 * 6 + 3] += c * H[2];
                    D[2 * 6 + 5] += c * H[0];
                    D[2 * 6 + 3] += c * H[1];
                    D[2 * 6 + 4] += c * H[2];
                } else {
                    Cc[1] += c * H[0];
                    Cc[0] += c * -H[1];
                    S[0 * 2 + 0] += c * H[0];
                    S[1 * 2 + 1] += c * (0.5 * H[0]);
                    S[2 * 2 + 1] += c * H[1];
                    S[1 * 2 + 0] += c * (0.5 * H[1]);
                    D[0 * 3 + 0] += c * H[0];
                    D[0 * 3 + 1] += c * H[1];
                    D[1 * 3 + 1] += c * H[0];
                    D[1 * 3 + 2] += c * H[1];
                }
            }
            __syncthreads();
        }
        for (int k = lane; k < wn; k += 64) {
            const double *Cc = acc + k * NB, *S = Cc + NC, *D = S + NS;
            for (int t = 0; t < NC; ++t) vc[vofs(out.lay, NC, t, w0 + k, m, mpc)] = Cc[t] * wi;
            for (int t = 0; t < NS; ++t) vs[vofs(out.lay, NS, t, w0 + k, m, mps)] = S[t] * wi;
            for (int t = 0; t < ND; ++t) vd[vofs(out.lay, ND, t, w0 + k, m, mpd)] = D[t] * wi;
        }
        __syncthreads();
    }
}


template <int R, int C, int MODE>
static void launch_gather_u(kle_ctx *ctx, const UMeshDev &U, kle_mat *A, const uint8_t *dir, const uint8_t *cls,
                            const double *E, int64_t eb0 = 0, int64_t eb1 = INT64_MAX, int accum = 0)
{
    if (A->nrows == 0) return;
    hipLaunchKernelGGL((k_gather_u<R, C, MODE>), dim3((unsigned)A->nrows), dim3(64), 0, ctx->stream, U, A->nrows,
                       A->d_rowptr, A->d_rowcnt, A->d_vptr, A->vlayout, A->d_bcol, dir, cls, E, A->d_val, eb0, eb1,
                       accum);
}

}  // namespace kle

using namespace kle;

extern "C" {

int kle_assemble_kle(kle_ctx *ctx, kle_mesh *m, kle_mat **K, kle_mat **Krhs, kle_mat **Rw)
{
    KLE_ARG(ctx && m && K && Krhs && Rw, "null arg");
    KLE_ARG(m->rank == ctx->rank && m->nranks == ctx->nranks, "mesh partition does not match ctx");
    KLE_ARG(m->dir_set, "Dirichlet nodes not set (kle_mesh_set_dirichlet_*)");
    const int dim = m->dim, dw = dim == 2 ? 1 : 3, ne = m->nn();
    KLE_HIP(hipSetDevice(ctx->device));
    kle_mat *mK = nullptr, *mKr = nullptr, *mRw = nullptr;
    // on any error below the partially built matrices are released
    struct Owned {
        kle_mat **p[3];
        bool keep = false;
        ~Owned()
        {
            if (!keep)
                for (auto q : p) kle_mat_destroy(*q);
        }
    } owned{{&mK, &mKr, &mRw}};
    PhaseTimer tm(ctx);
    UMeshBuf U;
    if (m->kind == 1) KLE_TRY(upload_umesh(ctx, m, U));
    const UMeshDev *Ud = m->kind == 1 ? &U.dev : nullptr;
    KLE_TRY(nb_create(ctx, m, 0, dim, dim, &mK, Ud));
    KLE_TRY(nb_create(ctx, m, 1, dim, dim, &mKr, Ud));
    KLE_TRY(nb_create(ctx, m, 2, dim, dw, &mRw, Ud));
    tm.lap("assemble_kle: three patterns");
    ElemSetup S;
    KLE_TRY(element_setup(ctx, m, S));
    const int64_t nel = S.nel;
    // Element scratch is bounded (KLE_ASM_SCRATCH_GB, default 8 GB): the
    // local elements are processed in ascending batches and every gather
    // continues each entry's ascending-cell sum from the stored partial, so
    // the result is bitwise the single-pass one (same additions, same order)
    // while config 4 needs 8 GB of scratch instead of 99 GB.
    const double per_el = (double)ne * ne * (dim * dim + dim * dw) * sizeof(double);
    double budget = 8e9;
    if (const char *e = getenv("KLE_ASM_SCRATCH_GB")) budget = atof(e) * 1e9;
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(nel, 1), (int64_t)(budget / per_el)));
    const int64_t nbatch = (nel + nb - 1) / nb;
    const int accum = nbatch > 1;
    struct Scratch {
        double *ke = nullptr, *rw = nullptr;
        uint8_t *dir = nullptr;
        ~Scratch()
        {
            if (ke) (void)hipFree(ke);
            if (rw) (void)hipFree(rw);
            if (dir) (void)hipFree(dir);
        }
    } sc;
    if (hipMalloc(&sc.ke, sizeof(double) * (size_t)std::max<int64_t>(nb * ne * ne * dim * dim, 1)) != hipSuccess ||
        hipMalloc(&sc.rw, sizeof(double) * (size_t)std::max<int64_t>(nb * ne * ne * dim * dw, 1)) != hipSuccess)
        return fail(KLE_ERR_MEM, "element matrix workspace (%.2f GB) does not fit", nb * per_el / 1e9);
    KLE_HIP(hipMalloc(&sc.dir, std::max<size_t>(m->dir.size(), 1)));
    KLE_HIP(hipMemcpyAsync(sc.dir, m->dir.data(), m->dir.size(), hipMemcpyHostToDevice, ctx->stream));
    if (accum)
        for (kle_mat *A : {mK, mKr, mRw})
            KLE_HIP(hipMemsetAsync(A->d_val, 0, sizeof(double) * std::max<int64_t>(A->nvals, 1), ctx->stream));
    MeshDev M = mesh_dev(m);
    const uint8_t *ddir = sc.dir;
    tm.lap("assemble_kle: geometry + scratch");
    for (int64_t e0 = 0; e0 < std::max<int64_t>(nel, 1); e0 += nb) {
        const int64_t cnt = std::min(nb, nel - e0), e1 = e0 + std::max<int64_t>(cnt, 0);
        KLE_TRY(element_batch(ctx, m, S, e0, cnt, sc.ke, sc.rw, nullptr));
        if (m->kind == 1) {
            if (dim == 3) {
                launch_gather_u<3, 3, 0>(ctx, U.dev, mK, ddir, nullptr, sc.ke, e0, e1, accum);
                launch_gather_u<3, 3, 1>(ctx, U.dev, mKr, ddir, nullptr, sc.ke, e0, e1, accum);
                launch_gather_u<3, 3, 2>(ctx, U.dev, mRw, ddir, nullptr, sc.rw, e0, e1, accum);
            } else {
                launch_gather_u<2, 2, 0>(ctx, U.dev, mK, ddir, nullptr, sc.ke, e0, e1, accum);
                launch_gather_u<2, 2, 1>(ctx, U.dev, mKr, ddir, nullptr, sc.ke, e0, e1, accum);
                launch_gather_u<2, 1, 2>(ctx, U.dev, mRw, ddir, nullptr, sc.rw, e0, e1, accum);
            }
        } else if (dim == 3) {
            launch_gather<3, 3, 0>(ctx, M, mK, ddir, sc.ke, e0, e1, accum);
            launch_gather<3, 3, 1>(ctx, M, mKr, ddir, sc.ke, e0, e1, accum);
            launch_gather<3, 3, 2>(ctx, M, mRw, ddir, sc.rw, e0, e1, accum);
        } else {
            launch_gather<2, 2, 0>(ctx, M, mK, ddir, sc.ke, e0, e1, accum);
            launch_gather<2, 2, 1>(ctx, M, mKr, ddir, sc.ke, e0, e1, accum);
            launch_gather<2, 1, 2>(ctx, M, mRw, ddir, sc.rw, e0, e1, accum);
        }
        KLE_HIP(hipGetLastError());
    }
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    tm.lap(nbatch > 1 ? "assemble_kle: element batches + gathers" : "assemble_kle: elements + gathers");
    owned.keep = true;
    // K is SPD (MatFS.buildFS: free-free blocks + unit Dirichlet diagonal):
    // a structured K (one rank or z slabs) of >= spmv_sym_min_rows node rows
    // per rank keeps its upper triangle only for the SpMV
    // (kle_mat_set_symmetric; collective, the same decision on every rank --
    // the count is the global one over the ranks); a K the symmetric path
    // cannot take keeps the full-storage kernels.  Per rank, because the
    // symmetric SpMV carries ~25 us of tile prologues, partial stores and
    // the gather that the full-storage SpMV does not: config 2's 1/4 slab
    // (85k rows) 133.6 vs 165 us, its 1/8 slab (43k rows) 77.6 vs 72.1 us
    // (profiles/r03/xl/slab_probes.jsonl)
    if (g_tune.spmv_sym && mK->m_global / 3 / ctx->nranks >= g_tune.spmv_sym_min_rows && mK->R == 3 &&
        mK->C == 3) {
        if (sym_build(mK)) (void)kle_last_error();
        tm.lap("assemble_kle: symmetric storage");
    }
    *K = mK;
    *Krhs = mKr;
    *Rw = mRw;
    return 0;
}

int kle_assemble_operators(kle_ctx *ctx, kle_mesh *m, kle_mat **Curl, kle_mat **SrT, kle_mat **DivSrT)
{
    KLE_ARG(ctx && m && Curl && SrT && DivSrT, "null arg");
    KLE_ARG(m->rank == ctx->rank && m->nranks == ctx->nranks, "mesh partition does not match ctx");
    const int dim = m->dim, dw = dim == 2 ? 1 : 3, ds = dim == 2 ? 3 : 6, nc = 1 << dim, G1 = 1 + dim * dim;
    KLE_HIP(hipSetDevice(ctx->device));
    kle_mat *mc = nullptr, *ms = nullptr, *md = nullptr;
    UMeshBuf U;
    if (m->kind == 1) KLE_TRY(upload_umesh(ctx, m, U));
    const UMeshDev *Ud = m->kind == 1 ? &U.dev : nullptr;
    KLE_TRY(nb_create(ctx, m, 3, dw, dim, &mc, Ud));
    KLE_TRY(nb_create(ctx, m, 3, ds, dim, &ms, Ud));
    KLE_TRY(nb_create(ctx, m, 3, dim, ds, &md, Ud));
    const int64_t nel = m->elem_end - m->elem_begin, nrows = mc->nrows;
    DevTables T;
    KLE_TRY(upload_tables(ctx, m->ngl, T));
    std::vector<double> corners(nel * nc * dim);
    KLE_TRY(kle_mesh_get_corners(m, corners.data()));
    std::vector<int> cnt(nrows);
    {
        std::vector<int> rp(nrows + 1);
        KLE_HIP(hipMemcpy(rp.data(), mc->d_rowptr, sizeof(int) * (nrows + 1), hipMemcpyDeviceToHost));
        if (mc->d_rowcnt) KLE_HIP(hipMemcpy(cnt.data(), mc->d_rowcnt, sizeof(int) * nrows, hipMemcpyDeviceToHost));
        else
            for (int64_t i = 0; i < nrows; ++i) cnt[i] = rp[i + 1] - rp[i];
    }
    double *dX = nullptr, *geo = nullptr, *winv = nullptr;
    int *dcnt = nullptr;
    const int64_t nq = nel * m->nn();
    KLE_HIP(hipMalloc(&dX, sizeof(double) * std::max<size_t>(corners.size(), 1)));
    KLE_HIP(hipMalloc(&geo, sizeof(double) * std::max<int64_t>(nq * G1, 1)));
    KLE_HIP(hipMalloc(&winv, sizeof(double) * std::max<int64_t>(nrows, 1)));
    KLE_HIP(hipMalloc(&dcnt, sizeof(int) * std::max<int64_t>(nrows, 1)));
    KLE_HIP(hipMemcpyAsync(dX, corners.data(), sizeof(double) * corners.size(), hipMemcpyHostToDevice, ctx->stream));
    KLE_HIP(hipMemcpyAsync(dcnt, cnt.data(), sizeof(int) * nrows, hipMemcpyHostToDevice, ctx->stream));
    MeshDev M = mesh_dev(m);
    OpsOut o{mc->d_val,   ms->d_val,   md->d_val,   mc->d_rowptr, ms->d_rowptr,
             md->d_rowptr, mc->d_vptr, ms->d_vptr, md->d_vptr, mc->vlayout};
    const unsigned gq = (unsigned)((nq + 255) / 256), gr = (unsigned)((nrows + 255) / 256),
                   gw = (unsigned)((nrows * 64 + 255) / 256);
    if (m->kind == 1 && nq > 0 && nrows > 0) {
        if (dim == 3) {
            hipLaunchKernelGGL(k_geometry<3>, dim3(gq), dim3(256), 0, ctx->stream, nel, m->ngl, T.O, dX, geo);
            hipLaunchKernelGGL(k_ops_weights_u<3>, dim3(gr), dim3(256), 0, ctx->stream, U.dev, nrows, geo, winv);
            hipLaunchKernelGGL(k_ops_gather_u<3>, dim3((unsigned)nrows), dim3(64), 0, ctx->stream, U.dev, m->ngl,
                               nrows, dcnt, mc->d_bcol, geo, T.O.dh, winv, o);
        } else {
            hipLaunchKernelGGL(k_geometry<2>, dim3(gq), dim3(256), 0, ctx->stream, nel, m->ngl, T.O, dX, geo);
            hipLaunchKernelGGL(k_ops_weights_u<2>, dim3(gr), dim3(256), 0, ctx->stream, U.dev, nrows, geo, winv);
            hipLaunchKernelGGL(k_ops_gather_u<2>, dim3((unsigned)nrows), dim3(64), 0, ctx->stream, U.dev, m->ngl,
                               nrows, dcnt, mc->d_bcol, geo, T.O.dh, winv, o);
        }
    } else if (m->kind == 1) {
    } else if (dim == 3) {
        hipLaunchKernelGGL(k_geometry<3>, dim3(gq), dim3(256), 0, ctx->stream, nel, m->ngl, T.O, dX, geo);
        hipLaunchKernelGGL(k_ops_weights<3>, dim3(gr), dim3(256), 0, ctx->stream, M, nrows, geo, winv);
        hipLaunchKernelGGL(k_ops_gather<3>, dim3(gw), dim3(256), 0, ctx->stream, M, nrows, dcnt, mc->d_bcol, geo,
                           T.O.dh, winv, o);
    } else {
        hipLaunchKernelGGL(k_geometry<2>, dim3(gq), dim3(256), 0, ctx->stream, nel, m->ngl, T.O, dX, geo);
        hipLaunchKernelGGL(k_ops_weights<2>, dim3(gr), dim3(256), 0, ctx->stream, M, nrows, geo, winv);
        hipLaunchKernelGGL(k_ops_gather<2>, dim3(gw), dim3(256), 0, ctx->stream, M, nrows, dcnt, mc->d_bcol, geo,
                           T.O.dh, winv, o);
    }
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    hipFree(dX);
    hipFree(geo);
    hipFree(winv);
    hipFree(dcnt);
    *Curl = mc;
    *SrT = ms;
    *DivSrT = md;
    return 0;
}

int kle_assemble_ns(kle_ctx *ctx, kle_mesh *m, kle_mat **K, kle_mat **Krhs, kle_mat **Rw, kle_mat **Rd,
                    kle_mat **Kfs, kle_mat **Krhsfs, kle_mat **Rwfs, kle_mat **Rdfs, kle_mat **Ksum)
{
    KLE_ARG(ctx && m && K && Krhs && Rw && Rd && Kfs && Krhsfs && Rwfs && Rdfs && Ksum, "null arg");
    KLE_ARG(m->rank == ctx->rank && m->nranks == ctx->nranks, "mesh partition does not match ctx");
    KLE_ARG(!m->dof_cls.empty(), "no-slip DoFs not set (kle_mesh_set_noslip_dofs)");
    // K, Krhs, Rw of MatNS are the free-slip ones with the no-slip nodes fixed
    // (mat_ns.py:124-141 + setIndices2One)
    KLE_TRY(kle_assemble_kle(ctx, m, K, Krhs, Rw));
    const int dim = m->dim, dw = dim == 2 ? 1 : 3;
    kle_mat *mf = nullptr, *mr = nullptr, *mw = nullptr, *ms = nullptr, *md = nullptr, *mdf = nullptr;
    UMeshBuf U;
    if (m->kind == 1) KLE_TRY(upload_umesh(ctx, m, U));
    const UMeshDev *Ud = m->kind == 1 ? &U.dev : nullptr;
    KLE_TRY(nb_create(ctx, m, 4, dim, dim, &mf, Ud));
    KLE_TRY(nb_create(ctx, m, 5, dim, dim, &mr, Ud));
    KLE_TRY(nb_create(ctx, m, 6, dim, dw, &mw, Ud));
    KLE_TRY(nb_create(ctx, m, 3, dim, dim, &ms, Ud));
    KLE_TRY(nb_create(ctx, m, 2, dim, 1, &md, Ud));   // Rd: free rows x cell nodes (mat_ns.py:139-141)
    KLE_TRY(nb_create(ctx, m, 6, dim, 1, &mdf, Ud));  // Rdfs: tangential rows x cell nodes (:113-114)
    const int rules[5] = {MASK_KFS, MASK_KRHSFS, MASK_TANG_ROWS, MASK_KSUM, MASK_TANG_ROWS};
    kle_mat *all[5] = {mf, mr, mw, ms, mdf};
    for (int t = 0; t < 5; ++t) {
        all[t]->mask_rule = rules[t];
        all[t]->dof_cls = m->dof_cls;
        all[t]->diag_only_row.assign(all[t]->nrows, 0);
    }
    double *dKe = nullptr, *dRwe = nullptr, *dRde = nullptr;
    KLE_TRY(element_matrices(ctx, m, &dKe, &dRwe, &dRde));
    uint8_t *ddir = nullptr;
    KLE_HIP(hipMalloc(&ddir, m->dir.size()));
    KLE_HIP(hipMemcpyAsync(ddir, m->dir.data(), m->dir.size(), hipMemcpyHostToDevice, ctx->stream));
    uint8_t *dcls = nullptr;
    KLE_HIP(hipMalloc(&dcls, m->dof_cls.size()));
    KLE_HIP(hipMemcpyAsync(dcls, m->dof_cls.data(), m->dof_cls.size(), hipMemcpyHostToDevice, ctx->stream));
    MeshDev M = mesh_dev(m);
    if (m->kind == 1) {
        if (dim == 3) {
            launch_gather_u<3, 3, 3>(ctx, U.dev, mf, ddir, dcls, dKe);
            launch_gather_u<3, 3, 4>(ctx, U.dev, mr, ddir, dcls, dKe);
            launch_gather_u<3, 3, 5>(ctx, U.dev, mw, ddir, dcls, dRwe);
            launch_gather_u<3, 3, 6>(ctx, U.dev, ms, ddir, dcls, dKe);
            launch_gather_u<3, 1, 2>(ctx, U.dev, md, ddir, dcls, dRde);
            launch_gather_u<3, 1, 5>(ctx, U.dev, mdf, ddir, dcls, dRde);
        } else {
            launch_gather_u<2, 2, 3>(ctx, U.dev, mf, ddir, dcls, dKe);
            launch_gather_u<2, 2, 4>(ctx, U.dev, mr, ddir, dcls, dKe);
            launch_gather_u<2, 1, 5>(ctx, U.dev, mw, ddir, dcls, dRwe);
            launch_gather_u<2, 2, 6>(ctx, U.dev, ms, ddir, dcls, dKe);
            launch_gather_u<2, 1, 2>(ctx, U.dev, md, ddir, dcls, dRde);
            launch_gather_u<2, 1, 5>(ctx, U.dev, mdf, ddir, dcls, dRde);
        }
    } else if (dim == 3) {
        launch_gather_ns<3, 3, 3>(ctx, M, mf, dcls, dKe);
        launch_gather_ns<3, 3, 4>(ctx, M, mr, dcls, dKe);
        launch_gather_ns<3, 3, 5>(ctx, M, mw, dcls, dRwe);
        launch_gather_ns<3, 3, 6>(ctx, M, ms, dcls, dKe);
        launch_gather<3, 1, 2>(ctx, M, md, ddir, dRde);
        launch_gather_ns<3, 1, 5>(ctx, M, mdf, dcls, dRde);
    } else {
        launch_gather_ns<2, 2, 3>(ctx, M, mf, dcls, dKe);
        launch_gather_ns<2, 2, 4>(ctx, M, mr, dcls, dKe);
        launch_gather_ns<2, 1, 5>(ctx, M, mw, dcls, dRwe);
        launch_gather_ns<2, 2, 6>(ctx, M, ms, dcls, dKe);
        launch_gather<2, 1, 2>(ctx, M, md, ddir, dRde);
        launch_gather_ns<2, 1, 5>(ctx, M, mdf, dcls, dRde);
    }
    KLE_HIP(hipGetLastError());
    KLE_HIP(hipStreamSynchronize(ctx->stream));
    hipFree(dKe);
    hipFree(dRwe);
    hipFree(dRde);
    hipFree(dcls);
    hipFree(ddir);
    *Rd = md;
    *Rdfs = mdf;
    *Kfs = mf;
    *Krhsfs = mr;
    *Rwfs = mw;
    *Ksum = ms;
    return 0;
}

int kle_element_kle(kle_ctx *ctx, kle_mesh *m, int64_t e, double *Ke, double *Rwe)
{
    KLE_ARG(ctx && m && Ke && Rwe, "null arg");
    const int64_t nel = m->elem_end - m->elem_begin;
    KLE_ARG(e >= 0 && e < nel, "element %lld out of local range", (long long)e);
    KLE_HIP(hipSetDevice(ctx->device));
    double *dKe = nullptr, *dRwe = nullptr;
    KLE_TRY(element_matrices(ctx, m, &dKe, &dRwe));
    const int dim = m->dim, ne = m->nn(), dw = dim == 2 ? 1 : 3;
    std::vector<double> kb((size_t)ne * ne * dim * dim), rb((size_t)ne * ne * dim * dw);
    KLE_HIP(hipMemcpy(kb.data(), dKe + (size_t)e * kb.size(), sizeof(double) * kb.size(), hipMemcpyDeviceToHost));
    KLE_HIP(hipMemcpy(rb.data(), dRwe + (size_t)e * rb.size(), sizeof(double) * rb.size(), hipMemcpyDeviceToHost));
    hipFree(dKe);
    hipFree(dRwe);
    // block layout [l][m][a][b] -> row-major [l a][m b]
    for (int l = 0; l < ne; ++l)
        for (int mm = 0; mm < ne; ++mm)
            for (int a = 0; a < dim; ++a) {
                for (int b = 0; b < dim; ++b)
                    Ke[(size_t)(l * dim + a) * ne * dim + mm * dim + b] = kb[(((size_t)l * ne + mm) * dim + a) * dim + b];
                for (int c = 0; c < dw; ++c)
                    Rwe[(size_t)(l * dim + a) * ne * dw + mm * dw + c] = rb[(((size_t)l * ne + mm) * dim + a) * dw + c];
            }
    return 0;
}

}  // extern "C"
