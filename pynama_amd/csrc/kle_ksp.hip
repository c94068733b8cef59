// kle_ksp.hip -- Krylov solvers on the device (KSP replacement).
//
// Replaces KspSolver / KSPSolve (solver/kle_solver.py:33-41,54-64).  The
// reference configures gmres + PC lu and the makefile forces preonly + lu
// (makefile:7); K is SPD (identity on Dirichlet rows, SPD free block), so the
// hot path is (Jacobi-)preconditioned CG:
//   * every scalar (alpha, beta, rho, norms) stays in device memory; kernels
//     read them directly -> no host round trip inside an iteration;
//   * convergence is decided on the device: the scalar kernel sets a reason
//     word and every later kernel of the solve turns into a no-op, so the
//     host only polls every few iterations and the iteration count is exact;
//   * single-reduction and pipelined CG: the vector update, its dot partials
//     and -- in its prologue -- the previous iteration's fixed-order final
//     sums and scalar stage are one kernel (k_sr_iter / k_pipe_iter); per
//     iteration: update, SpMV, and for single-reduction CG a (w, u) partial
//     launch; N ranks allreduce the partial arrays, not scalars;
//   * deterministic reductions (per-workgroup partials, fixed-order final
//     sum), RCCL allreduce of the 1-3 scalars across ranks.
// PC lu (and KSP preonly) are a dense rocSOLVER factorization for the
// small sequential systems the reference's own cases use (config 1).
// GMRES(m) (classical Gram-Schmidt, right Jacobi preconditioning) is the
// general fallback; its tiny Hessenberg least-squares update runs on the host.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "kle_internal.hpp"

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

namespace kle {

__device__ __forceinline__ double wsum2(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block sum of 1..3 values, lane 0 of wave 0 holds the result
template <int NQ>
__device__ __forceinline__ void block_sums(double (&v)[NQ], double *partials, int stride)
{
    __shared__ double lds[NQ][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] = wsum2(v[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NQ; ++q) lds[q][w] = v[q];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            double s = 0;
            for (int i = 0; i < nw; ++i) s += lds[q][i];
            partials[q * stride + blockIdx.x] = s;
        }
}

constexpr int KB = 256;

enum Stage { ST_START = 0, ST_ALPHA = 1, ST_BETA = 2, ST_SR_START = 3, ST_SR = 4 };
__device__ void cg_scalars(int stage, double *scal, int *ist, double rtol, double atol);

// Last-arriving workgroup of the grid, as seen by the calling thread (thread 0
// of each workgroup, after its partials are written through and drained):
// one ticket word, reset by the last arriver (the next launch that uses it is
// stream-ordered behind this one).  Eight per-slot words + a global word
// (fewer arrivals per word) were measured slower: 89.3 vs 88.5 us per CG
// iteration on the 1/8 slab, 784.9 vs 784.1 at config 2
// (profiles/r02/ticket_*.jsonl) -- at <= 256 workgroups the second atomic
// round trip costs more than the contention it removes.
__device__ __forceinline__ bool grid_last_arriver(int *tk)
{
    const int t = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t != (int)gridDim.x - 1) return false;
    __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// x = 0, r = b, p = 0 ; partials: [0] r.z, [1] r.r
template <bool JAC>
__global__ __launch_bounds__(KB) void k_cg_start(int64_t n, const double *__restrict__ b,
                                                 const double *__restrict__ dinv, double *__restrict__ x,
                                                 double *__restrict__ r, double *__restrict__ p,
                                                 double *__restrict__ partials)
{
    double s[2] = {0.0, 0.0};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double ri = b[i];
        x[i] = 0.0;
        r[i] = ri;
        p[i] = 0.0;
        const double zi = JAC ? dinv[i] * ri : ri;
        s[0] += ri * zi;
        s[1] += ri * ri;
    }
    block_sums<2>(s, partials, PART_STRIDE);
}

// p = z + beta p,  z = D^-1 r
template <bool JAC>
__global__ __launch_bounds__(KB) void k_cg_p(int64_t n, const double *__restrict__ r, const double *__restrict__ dinv,
                                             double *__restrict__ p, const double *__restrict__ scal,
                                             const int *__restrict__ ist)
{
    if (ist[I_REASON] != 0) return;
    const double beta = scal[S_BETA];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double zi = JAC ? dinv[i] * r[i] : r[i];
        p[i] = zi + beta * p[i];
    }
}

// x += alpha p ; r -= alpha q ; partials: [0] r.z, [1] r.r
template <bool JAC>
__global__ __launch_bounds__(KB) void k_cg_update(int64_t n, const double *__restrict__ p, const double *__restrict__ q,
                                                  const double *__restrict__ dinv, double *__restrict__ x,
                                                  double *__restrict__ r, double *__restrict__ partials,
                                                  const double *__restrict__ scal, const int *__restrict__ ist)
{
    if (ist[I_REASON] != 0) return;
    const double alpha = scal[S_ALPHA];
    double s[2] = {0.0, 0.0};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] += alpha * p[i];
        const double ri = r[i] - alpha * q[i];
        r[i] = ri;
        const double zi = JAC ? dinv[i] * ri : ri;
        s[0] += ri * zi;
        s[1] += ri * ri;
    }
    block_sums<2>(s, partials, PART_STRIDE);
}

// x = 0, r = b, u = M r, p = s = 0 ; partials: [0] r.u, [1] r.r
template <bool JAC>
__global__ __launch_bounds__(KB) void k_sr_start(int64_t n, const double *__restrict__ b,
                                                 const double *__restrict__ dinv, double *__restrict__ x,
                                                 double *__restrict__ r, double *__restrict__ u, double *__restrict__ p,
                                                 double *__restrict__ sv, double *__restrict__ partials)
{
    double acc[2] = {0.0, 0.0};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double ri = b[i];
        const double ui = JAC ? dinv[i] * ri : ri;
        x[i] = 0.0;
        r[i] = ri;
        u[i] = ui;
        p[i] = 0.0;
        sv[i] = 0.0;
        acc[0] += ri * ui;
        acc[1] += ri * ri;
    }
    block_sums<2>(acc, partials, PART_STRIDE);
}

// m = M w ; z = q = 0 (start of pipelined CG)
template <bool JAC>
__global__ __launch_bounds__(KB) void k_pipe_init(int64_t n, const double *__restrict__ dinv,
                                                  const double *__restrict__ w, double *__restrict__ m,
                                                  double *__restrict__ z, double *__restrict__ q)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        m[i] = JAC ? dinv[i] * w[i] : w[i];
        z[i] = 0.0;
        q[i] = 0.0;
    }
}

// One Chronopoulos-Gear scalar stage from the three sums g = (r,u),
// rn = ||r||, d = (w,u) and the previous rho / alpha / iteration count: the
// iteration count, a reason (0: go on) and, when the recurrence continues
// (upd), the new beta, alpha, rho.  Shared by cg_scalars (ST_SR) and the
// pipelined update's prologue, so both apply the same arithmetic.
struct SrStep {
    double alpha, beta, rho;
    int its, reason;
    bool upd;
};
__device__ __forceinline__ SrStep sr_step(double g, double rn, double d, double rho_prev, double alpha_prev,
                                          int its_prev, double tol, int fixed, int maxit, double atol)
{
    SrStep s{alpha_prev, 0.0, rho_prev, its_prev + 1, 0, false};
    if (fixed) {
        // fixed iterations: the host launches exactly I_FIXED of them, so no
        // kernel has to stop; the recurrence stays complete for kle_ksp_continue
        if (!isfinite(rn)) s.reason = KLE_DIVERGED_NANORINF;
    } else if (!isfinite(rn)) {
        s.reason = KLE_DIVERGED_NANORINF;
        return s;
    } else if (rn <= tol) {
        s.reason = rn <= atol ? KLE_CONVERGED_ATOL : KLE_CONVERGED_RTOL;
        return s;
    } else if (s.its >= maxit) {
        s.reason = KLE_DIVERGED_ITS;
        return s;
    }
    const double beta = g / rho_prev;
    const double den = d - beta * g / alpha_prev;
    if (den <= 0.0 && !fixed) {
        s.reason = -8;
        return s;
    }
    s.beta = beta;
    s.alpha = g / den;
    s.rho = g;
    s.upd = true;
    return s;
}

__device__ void cg_scalars(int stage, double *scal, int *ist, double rtol, double atol)
{
    if (stage == ST_SR_START || stage == ST_SR) {
        // Chronopoulos-Gear single-reduction CG: sums = (r,u), (r,r), (w,u)
        const double g = scal[S_SUM0], rr = scal[S_SUM1], d = scal[S_SUM2];
        const double rn = sqrt(rr);
        scal[S_RR] = rr;
        if (stage == ST_SR_START) {
            scal[S_BNORM] = rn;
            scal[S_TOL] = fmax(rtol * rn, atol);
            ist[I_ITS] = 0;
            ist[I_REASON] = 0;
            scal[S_BETA] = 0.0;
            scal[S_RHO] = g;
            scal[S_ALPHA] = g / d;
            if (!ist[I_FIXED] && rn <= scal[S_TOL]) ist[I_REASON] = rn <= atol ? KLE_CONVERGED_ATOL : KLE_CONVERGED_RTOL;
            else if (!isfinite(rn)) ist[I_REASON] = KLE_DIVERGED_NANORINF;
            else if (d <= 0.0 && !ist[I_FIXED]) ist[I_REASON] = -8;
            return;
        }
        if (ist[I_REASON] != 0) return;
        const SrStep st = sr_step(g, rn, d, scal[S_RHO], scal[S_ALPHA], ist[I_ITS], scal[S_TOL], ist[I_FIXED],
                                  ist[I_MAXIT], atol);
        ist[I_ITS] = st.its;
        if (st.reason) ist[I_REASON] = st.reason;
        if (st.upd) {
            scal[S_BETA] = st.beta;
            scal[S_ALPHA] = st.alpha;
            scal[S_RHO] = st.rho;
        }
        return;
    }
    if (stage == ST_START) {
        const double rz = scal[S_SUM0], rr = scal[S_SUM1];
        const double bn = sqrt(rr);
        scal[S_BNORM] = bn;
        scal[S_TOL] = fmax(rtol * bn, atol);
        scal[S_RHO] = rz;
        scal[S_RR] = rr;
        scal[S_BETA] = 0.0;
        ist[I_ITS] = 0;
        ist[I_REASON] = 0;
        if (!ist[I_FIXED] && bn <= scal[S_TOL]) ist[I_REASON] = bn <= atol ? KLE_CONVERGED_ATOL : KLE_CONVERGED_RTOL;
        if (!isfinite(bn)) ist[I_REASON] = KLE_DIVERGED_NANORINF;
        return;
    }
    if (ist[I_REASON] != 0) return;
    if (stage == ST_ALPHA) {
        const double pq = scal[S_SUM0];
        scal[S_PQ] = pq;
        if (!isfinite(pq)) {
            ist[I_REASON] = KLE_DIVERGED_NANORINF;
            return;
        }
        if (pq <= 0.0 && !ist[I_FIXED]) {
            ist[I_REASON] = -8;  // KSP_DIVERGED_INDEFINITE_MAT
            return;
        }
        scal[S_ALPHA] = scal[S_RHO] / pq;
        return;
    }
    // ST_BETA
    const double rz = scal[S_SUM0], rr = scal[S_SUM1];
    scal[S_RHO_OLD] = scal[S_RHO];
    scal[S_RHO] = rz;
    scal[S_BETA] = rz / scal[S_RHO_OLD];
    scal[S_RR] = rr;
    const int its = ++ist[I_ITS];
    const double rn = sqrt(rr);
    if (ist[I_FIXED]) {
        if (!isfinite(rn)) ist[I_REASON] = KLE_DIVERGED_NANORINF;
        return;
    }
    if (!isfinite(rn)) ist[I_REASON] = KLE_DIVERGED_NANORINF;
    else if (rn <= scal[S_TOL]) ist[I_REASON] = rn <= atol ? KLE_CONVERGED_ATOL : KLE_CONVERGED_RTOL;
    else if (its >= ist[I_MAXIT]) ist[I_REASON] = KLE_DIVERGED_ITS;
}

// Sum nq partial arrays (fixed order) into scal[S_SUM0..]; optionally apply
// the stage's scalar update in the same launch (single rank).
struct NParts {
    int n[4];
};

__global__ __launch_bounds__(1024) void k_reduce_stage(const double *__restrict__ partials, NParts np, int nq,
                                                       double *__restrict__ scal, int *__restrict__ ist, int stage,
                                                       int fuse, double rtol, double atol)
{
    if (stage != ST_START && stage != ST_SR_START && ist[I_REASON] != 0) return;
    __shared__ double lds[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int q = 0; q < nq; ++q) {
        double s = 0;
        const int nparts = np.n[q];
        for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += partials[q * PART_STRIDE + i];
        s = wsum2(s);
        __syncthreads();
        if (lane == 0) lds[w] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0;
            for (int i = 0; i < nw; ++i) t += lds[i];
            scal[S_SUM0 + q] = t;
        }
    }
    if (fuse && threadIdx.x == 0) cg_scalars(stage, scal, ist, rtol, atol);
}

__global__ void k_scalars(double *scal, int *ist, int stage, double rtol, double atol)
{
    cg_scalars(stage, scal, ist, rtol, atol);
}

// Three sums of per-workgroup partials in a fixed order (every caller gets
// bitwise the same values): t0 = sum a0[0..Ga), t1 = sum a1[0..Ga),
// t2 = sum a2[0..G2).
__device__ __forceinline__ void sums3(const double *__restrict__ a0, const double *__restrict__ a1, int Ga,
                                      const double *__restrict__ a2, int G2, double (&t)[3])
{
    __shared__ double red[3][KB / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[3] = {0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < Ga; i += KB) {
        a[0] += a0[i];
        a[1] += a1[i];
    }
    for (int i = threadIdx.x; i < G2; i += KB) a[2] += a2[i];
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] = wsum2(a[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < 3; ++q) red[q][w] = a[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < KB / 64; ++i) s += red[q][i];
        t[q] = s;
    }
}

// The prologue shared by the pipelined and the single-reduction CG update
// kernels: with pro, the previous iteration's scalar stage from the sums t
// (every workgroup runs the same sr_step; workgroup 0 writes the next
// parity's stage inputs and the reporting slots); without, alpha / beta from
// the scalar slots (workgroup 0 seeds the next parity's inputs from them).
// Returns, in every thread, whether the stage ended the solve; alpha / beta
// for the update.
// The scalar inputs of the stage, read by thread 0 at kernel entry so their
// latency overlaps the partial sums.
struct StageIn {
    double prho, palpha, tol, alpha, beta, rho;
    int pits, fixed, maxit, its;
};
__device__ __forceinline__ StageIn stage_inputs(const double *__restrict__ scal, const int *__restrict__ ist, int par)
{
    StageIn in;
    in.prho = scal[S_PRHO0 + par];
    in.palpha = scal[S_PALPHA0 + par];
    in.tol = scal[S_TOL];
    in.alpha = scal[S_ALPHA];
    in.beta = scal[S_BETA];
    in.rho = scal[S_RHO];
    in.pits = ist[I_PITS0 + par];
    in.fixed = ist[I_FIXED];
    in.maxit = ist[I_MAXIT];
    in.its = ist[I_ITS];
    return in;
}

__device__ __forceinline__ bool stage_prologue(int pro, const double (&t)[3], double *__restrict__ scal,
                                               int *__restrict__ ist, int par, double atol, double &alpha,
                                               double &beta, const StageIn *pre = nullptr)
{
    __shared__ double ab[2];
    __shared__ int stop;
    const bool w0 = blockIdx.x == 0 && threadIdx.x == 0;
    const int nxt = par ^ 1;
    if (threadIdx.x == 0) {
        const StageIn in = pre ? *pre : stage_inputs(scal, ist, par);
        if (pro) {
            const SrStep st = sr_step(t[0], sqrt(t[1]), t[2], in.prho, in.palpha, in.pits, in.tol, in.fixed,
                                      in.maxit, atol);
            ab[0] = st.alpha;
            ab[1] = st.beta;
            stop = st.reason != 0;
            if (w0) {
                scal[S_RR] = t[1];
                ist[I_ITS] = st.its;
                if (st.upd) {
                    scal[S_ALPHA] = st.alpha;
                    scal[S_BETA] = st.beta;
                    scal[S_RHO] = st.rho;
                }
                scal[S_PRHO0 + nxt] = st.rho;
                scal[S_PALPHA0 + nxt] = st.alpha;
                ist[I_PITS0 + nxt] = st.its;
                if (st.reason) ist[I_REASON] = st.reason;
            }
        } else {
            ab[0] = in.alpha;
            ab[1] = in.beta;
            stop = 0;
            if (w0) {
                scal[S_PRHO0 + nxt] = in.rho;
                scal[S_PALPHA0 + nxt] = in.alpha;
                ist[I_PITS0 + nxt] = in.its;
            }
        }
    }
    __syncthreads();
    alpha = ab[0];
    beta = ab[1];
    return stop != 0;
}

constexpr int PRO_UPD_BLOCKS = 1024;  // update kernels whose partials a prologue re-sums
constexpr int PRO_DOT_BLOCKS = 512;

// One pipelined CG iteration (PETSc KSPPIPECG; Ghysels & Vanroose 2014):
// with w = A u, u = M r kept by recurrence, one fused pass
//   z = n + b z, q = m + b q, s = w + b s, p = u + b p,
//   x += a p, r -= a s, u -= a q, w -= a z, m = M w
// writing its per-workgroup sums (r,u), (r,r), (w,u) to pp_out [3][G].
// pro = 1: the prologue first applies the PREVIOUS iteration's scalar stage --
// every workgroup sums pp_in (the previous launch's partials, allreduced over
// the ranks) in the same fixed order and runs sr_step, so no reduction or
// scalar launch sits between two iterations (one rank: update + SpMV per
// iteration).  The stage's inputs (rho, alpha, iteration count) are
// double-buffered by launch parity: this launch reads set `par`, workgroup 0
// writes set par^1 and the reporting slots.  pro = 0 (first launch after a
// start or a flush): alpha, beta from the scalar slots.  A stage that ends the
// solve (converged, diverged, NaN) skips the update in every workgroup, as the
// reason word makes every later launch a no-op.
// (SGPRs capped at 64: the HIP runtime admits waves per SIMD as 512 / SGPRs
// rounded up to 16, so 71-83 SGPRs held these streaming updates at 5-6 waves
// per SIMD instead of 8; kle_sym.hip SYM_XL_SGPRS)
template <bool JAC, bool PRE>
__global__ __launch_bounds__(KB) __attribute__((amdgpu_num_sgpr(64))) void k_pipe_iter(int64_t n, const double *__restrict__ dinv,
                                                  const double *__restrict__ nv, double *__restrict__ z,
                                                  double *__restrict__ q, double *__restrict__ sv,
                                                  double *__restrict__ p, double *__restrict__ x,
                                                  double *__restrict__ r, double *__restrict__ u,
                                                  double *__restrict__ w, double *__restrict__ m,
                                                  const double *__restrict__ pp_in, double *__restrict__ pp_out,
                                                  double *__restrict__ scal, int *__restrict__ ist, int pro, int par,
                                                  double atol)
{
    const int G = (int)gridDim.x;
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    // PRE: this thread's first element and the stage's scalar inputs are
    // loaded before the reason check and the partial sums, so their latency
    // overlaps the prologue instead of following it (same arithmetic)
    double e[11];
    StageIn in;
    if constexpr (PRE) {
        if (i0 < n) {
            e[0] = nv[i0], e[1] = z[i0], e[2] = m[i0], e[3] = q[i0], e[4] = w[i0], e[5] = sv[i0];
            e[6] = u[i0], e[7] = p[i0], e[8] = x[i0], e[9] = r[i0], e[10] = JAC ? dinv[i0] : 1.0;
        }
        if (threadIdx.x == 0) in = stage_inputs(scal, ist, par);
    }
    if (ist[I_REASON] != 0) return;
    double t[3] = {0.0, 0.0, 0.0};
    if (pro) sums3(pp_in, pp_in + G, G, pp_in + 2 * G, G, t);
    double alpha, beta;
    if (stage_prologue(pro, t, scal, ist, par, atol, alpha, beta, PRE ? &in : nullptr)) return;
    double acc[3] = {0.0, 0.0, 0.0};
    for (int64_t i = i0; i < n; i += stride) {
        if (!PRE || i != i0) {
            e[0] = nv[i], e[1] = z[i], e[2] = m[i], e[3] = q[i], e[4] = w[i], e[5] = sv[i];
            e[6] = u[i], e[7] = p[i], e[8] = x[i], e[9] = r[i], e[10] = JAC ? dinv[i] : 1.0;
        }
        const double zi = e[0] + beta * e[1];
        const double qi = e[2] + beta * e[3];
        const double si = e[4] + beta * e[5];
        const double pi = e[6] + beta * e[7];
        z[i] = zi;
        q[i] = qi;
        sv[i] = si;
        p[i] = pi;
        x[i] = e[8] + alpha * pi;
        const double ri = e[9] - alpha * si;
        const double ui = e[6] - alpha * qi;
        const double wi = e[4] - alpha * zi;
        r[i] = ri;
        u[i] = ui;
        w[i] = wi;
        m[i] = JAC ? e[10] * wi : wi;
        acc[0] += ri * ui;
        acc[1] += ri * ri;
        acc[2] += wi * ui;
    }
    block_sums<3>(acc, pp_out, G);
}

// k_pipe_iter with the gather of a split box-brick product n = A m folded in
// (kle_brick.hip brick_spmv split): the product left
// its bricks' region sums in ws and the rows' direct sums in n, and a wave of
// this update takes one 64-row slice -- it sums the slice's runs (the
// run-mask gather's order: runs, then the direct sum or a one-block row's
// B_ii x_i, then the lower neighbour's reverse-halo sum) into LDS and updates
// the slice's 192 entries from there.  So n's gather costs no launch of its
// own, and n is neither written nor read back (it is not used after the
// update).  The slices past ng (the rows the split product gathered with the
// upper ghost rows) read n.  One-block rows read m before this wave updates
// it (the same slice).
template <bool JAC>
__global__ __launch_bounds__(KB) __attribute__((amdgpu_num_sgpr(64))) void k_pipe_iter_g(BrickGather gs, int64_t n,
                                                  const double *__restrict__ dinv,
                                                  const double *__restrict__ nv, double *__restrict__ z,
                                                  double *__restrict__ q, double *__restrict__ sv,
                                                  double *__restrict__ p, double *__restrict__ x,
                                                  double *__restrict__ r, double *__restrict__ u,
                                                  double *__restrict__ w, double *__restrict__ m,
                                                  const double *__restrict__ pp_in, double *__restrict__ pp_out,
                                                  double *__restrict__ scal, int *__restrict__ ist, int pro, int par,
                                                  double atol)
{
    constexpr int WPB = KB / 64;
    __shared__ double nl[WPB][192];
    const int G = (int)gridDim.x;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nsl = (gs.nrows + 63) / 64, sst = (int64_t)G * WPB;
    const unsigned long long below = (1ull << lane) - 1ull;
    // n of one slice into nl[wv] (entries 3 j .. 3 j + 2 of its row j)
    auto gather = [&](int64_t sl) {
        const int64_t j = sl * 64 + lane;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        if (sl * 64 < gs.ng) {
            const int rb = gs.runptr[sl], re = gs.runptr[sl + 1];
            const bool one = j < gs.nrows && gs.single && ((gs.single[sl] >> lane) & 1ull);
            double d0 = 0.0, d1 = 0.0, d2 = 0.0;
            if (j < gs.nrows) {
                if (one) {
                    const double *v = gs.sval + gs.svptr[j];
                    const double x0 = gs.xs[3 * j], x1 = gs.xs[3 * j + 1], x2 = gs.xs[3 * j + 2];
                    d0 = v[0] * x0 + v[1] * x1 + v[2] * x2;
                    d1 = v[3] * x0 + v[4] * x1 + v[5] * x2;
                    d2 = v[6] * x0 + v[7] * x1 + v[8] * x2;
                } else {
                    d0 = nv[3 * j];
                    d1 = nv[3 * j + 1];
                    d2 = nv[3 * j + 2];
                }
            }
#pragma unroll 8
            for (int rr = rb; rr < re; ++rr) {
                const unsigned long long mk = gs.rmask[rr];
                const bool in = (mk >> lane) & 1ull;
                const double *pw = gs.ws + (int64_t)gs.rstart[rr] + (in ? 3 * __popcll(mk & below) : 0);
                const double a0 = pw[0], a1 = pw[1], a2 = pw[2];
                s0 += in ? a0 : 0.0;
                s1 += in ? a1 : 0.0;
                s2 += in ? a2 : 0.0;
            }
            s0 += d0;
            s1 += d1;
            s2 += d2;
        } else if (j < gs.nrows) {
            s0 = nv[3 * j];
            s1 = nv[3 * j + 1];
            s2 = nv[3 * j + 2];
        }
        if (3 * j < gs.nrecv) {  // (the reverse halo's sums, last)
            s0 += gs.recv[3 * j];
            s1 += gs.recv[3 * j + 1];
            s2 += gs.recv[3 * j + 2];
        }
        nl[wv][3 * lane] = s0;
        nl[wv][3 * lane + 1] = s1;
        nl[wv][3 * lane + 2] = s2;
        __builtin_amdgcn_wave_barrier();
    };
    int64_t sl = (int64_t)blockIdx.x * WPB + wv;
    // the first slice's gather before the prologue (it needs no scalar)
    StageIn in;
    if (threadIdx.x == 0) in = stage_inputs(scal, ist, par);
    if (sl < nsl) gather(sl);
    if (ist[I_REASON] != 0) return;
    double t[3] = {0.0, 0.0, 0.0};
    if (pro) sums3(pp_in, pp_in + G, G, pp_in + 2 * G, G, t);
    double alpha, beta;
    if (stage_prologue(pro, t, scal, ist, par, atol, alpha, beta, &in)) return;
    double acc[3] = {0.0, 0.0, 0.0};
    for (; sl < nsl; sl += sst) {
        if (sl != (int64_t)blockIdx.x * WPB + wv) gather(sl);
#pragma unroll
        for (int ps = 0; ps < 3; ++ps) {
            const int el = ps * 64 + lane;
            const int64_t i = sl * 192 + el;
            if (i >= n) break;
            const double e0 = nl[wv][el];
            const double zi = e0 + beta * z[i];
            const double qi = m[i] + beta * q[i];
            const double wo = w[i];
            const double si = wo + beta * sv[i];
            const double uo = u[i];
            const double pi = uo + beta * p[i];
            z[i] = zi;
            q[i] = qi;
            sv[i] = si;
            p[i] = pi;
            x[i] = x[i] + alpha * pi;
            const double ri = r[i] - alpha * si;
            const double ui = uo - alpha * qi;
            const double wi = wo - alpha * zi;
            r[i] = ri;
            u[i] = ui;
            w[i] = wi;
            m[i] = JAC ? dinv[i] * wi : wi;
            acc[0] += ri * ui;
            acc[1] += ri * ri;
            acc[2] += wi * ui;
        }
        __builtin_amdgcn_wave_barrier();  // (nl[wv] read before the next slice's gather writes it)
    }
    block_sums<3>(acc, pp_out, G);
}

// The scalar stage of the last update of a solve call whose partials would
// otherwise wait for the next launch's prologue (pipelined / single-reduction
// CG): leaves the reporting slots (iterations, residual, reason, alpha / beta
// / rho) consistent.
__global__ __launch_bounds__(KB) void k_cg_flush(const double *__restrict__ a0, const double *__restrict__ a1,
                                                 int Ga, const double *__restrict__ a2, int G2,
                                                 double *__restrict__ scal, int *__restrict__ ist, int par,
                                                 double atol)
{
    if (ist[I_REASON] != 0) return;  // the last launch stopped: nothing pending
    double t[3];
    sums3(a0, a1, Ga, a2, G2, t);
    if (threadIdx.x != 0) return;
    const SrStep st = sr_step(t[0], sqrt(t[1]), t[2], scal[S_PRHO0 + par], scal[S_PALPHA0 + par], ist[I_PITS0 + par],
                              scal[S_TOL], ist[I_FIXED], ist[I_MAXIT], atol);
    scal[S_RR] = t[1];
    ist[I_ITS] = st.its;
    if (st.upd) {
        scal[S_ALPHA] = st.alpha;
        scal[S_BETA] = st.beta;
        scal[S_RHO] = st.rho;
    }
    if (st.reason) ist[I_REASON] = st.reason;
}

// Single-reduction CG iteration with the previous stage in its prologue (one
// rank): sums (r,u), (r,r) of the previous update [2][G] and (w,u) of the
// dot launch [Gd], then  p = u + b p ; s = w + b s ; x += a p ; r -= a s ;
// u = M r  with the new (r,u), (r,r) partials to pu_out [2][G].
// NT (tuning upd_nt): every vector but u is loaded and stored nontemporal, so
// that u -- the next SpMV's x -- is what the Infinity Cache keeps of this
// launch (vectors of 64 MB at 8M DoF: the update's other 704 MB evict it)
template <bool NT>
__device__ __forceinline__ double ld_upd(const double *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st_upd(double *p, double v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool JAC, bool PRE, bool NT = false, int SR_UNR = 1>
__global__ __launch_bounds__(KB) __attribute__((amdgpu_num_sgpr(64))) void k_sr_iter(int64_t n, const double *__restrict__ dinv,
                                                const double *__restrict__ w, double *__restrict__ u,
                                                double *__restrict__ p, double *__restrict__ sv,
                                                double *__restrict__ x, double *__restrict__ r,
                                                const double *__restrict__ pu_in, const double *__restrict__ pd,
                                                int Gd, double *__restrict__ pu_out, double *__restrict__ scal,
                                                int *__restrict__ ist, int pro, int par, double atol)
{
    const int G = (int)gridDim.x;
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    // SR_UNR elements of the grid-stride sequence per pass, all their loads
    // in flight before the first update (upd_unroll; 2: 97 VGPRs, all 4096
    // waves of config 2 still resident); the elements are summed in the same
    // order as one at a time (bitwise equal)
    double e[SR_UNR][7];  // PRE: the first element before the prologue (as k_pipe_iter)
    auto load = [&](int64_t i, double *f) {
        f[0] = u[i], f[1] = ld_upd<NT>(p + i), f[2] = ld_upd<NT>(w + i), f[3] = ld_upd<NT>(sv + i);
        f[4] = ld_upd<NT>(x + i), f[5] = ld_upd<NT>(r + i);
        f[6] = JAC ? ld_upd<NT>(dinv + i) : 1.0;
    };
    StageIn in;
    if constexpr (PRE) {
        if (i0 < n) load(i0, e[0]);
        if (threadIdx.x == 0) in = stage_inputs(scal, ist, par);
    }
    if (ist[I_REASON] != 0) return;
    double t[3] = {0.0, 0.0, 0.0};
    if (pro) sums3(pu_in, pu_in + G, G, pd, Gd, t);
    double alpha, beta;
    if (stage_prologue(pro, t, scal, ist, par, atol, alpha, beta, PRE ? &in : nullptr)) return;
    double acc[2] = {0.0, 0.0};
    for (int64_t ib = i0; ib < n; ib += SR_UNR * stride) {
#pragma unroll
        for (int q = 0; q < SR_UNR; ++q) {
            const int64_t i = ib + q * stride;
            if (i < n && (!PRE || i != i0)) load(i, e[q]);
        }
#pragma unroll
        for (int q = 0; q < SR_UNR; ++q) {
            const int64_t i = ib + q * stride;
            if (i >= n) break;
            const double pi = e[q][0] + beta * e[q][1];
            const double si = e[q][2] + beta * e[q][3];
            st_upd<NT>(p + i, pi);
            st_upd<NT>(sv + i, si);
            st_upd<NT>(x + i, e[q][4] + alpha * pi);
            const double ri = e[q][5] - alpha * si;
            st_upd<NT>(r + i, ri);
            const double ui = JAC ? e[q][6] * ri : ri;
            u[i] = ui;
            acc[0] += ri * ui;
            acc[1] += ri * ri;
        }
    }
    block_sums<2>(acc, pu_out, G);
}

// k_sr_iter with the gather of a split box-brick product w = A u folded in
// (one rank; VERDICT r05 item 1a, as k_pipe_iter_g): the product left its
// bricks' region sums in ws, the rows' direct sums in w and the bricks'
// shares of (w, u) in the partials after this launch's (k_nb_spmv_sym_brick
// DOT), so the prologue has the whole (w, u) before any row is gathered.  A
// wave takes one 64-row slice: it sums the slice's runs (the run-mask
// gather's order: runs, then the direct sum or a one-block row's B_ii u_i)
// into LDS and updates the slice's 192 entries from there; w is neither
// written nor read back.  The one-block rows' share of the NEXT product's
// (w, u), (B_ii u_i, u_i), is formed here from the new u (those rows are no
// brick's): partials [3][G] = (r,u) | (r,r) | that share, the bricks' after
// them (G2 = G + bricks in all).  Without pro (the first update of a call)
// w is complete and read as it is.
// PRE (upd_preload): the first slice's vectors are loaded before the
// prologue too, so their latency overlaps the partial sums (same arithmetic)
template <bool JAC, bool PRE>
__global__ __launch_bounds__(KB) __attribute__((amdgpu_num_sgpr(64))) void k_sr_iter_g(BrickGather gs, int64_t n,
                                                  const double *__restrict__ dinv, const double *__restrict__ w,
                                                  double *__restrict__ u, double *__restrict__ p,
                                                  double *__restrict__ sv, double *__restrict__ x,
                                                  double *__restrict__ r, const double *__restrict__ pu_in, int G2,
                                                  double *__restrict__ pu_out, double *__restrict__ scal,
                                                  int *__restrict__ ist, int pro, int par, double atol)
{
    constexpr int WPB = KB / 64;
    __shared__ double nl[WPB][192];
    const int G = (int)gridDim.x;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nsl = (gs.nrows + 63) / 64, sst = (int64_t)G * WPB;
    const unsigned long long below = (1ull << lane) - 1ull;
    // w of one slice into nl[wv] (entries 3 j .. 3 j + 2 of its row j)
    auto gather = [&](int64_t sl) {
        const int64_t j = sl * 64 + lane;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        if (sl * 64 < gs.ng) {
            const int rb = gs.runptr[sl], re = gs.runptr[sl + 1];
            const bool one = j < gs.nrows && gs.single && ((gs.single[sl] >> lane) & 1ull);
            double d0 = 0.0, d1 = 0.0, d2 = 0.0;
            if (j < gs.nrows) {
                if (one) {
                    const double *v = gs.sval + gs.svptr[j];
                    const double x0 = gs.xs[3 * j], x1 = gs.xs[3 * j + 1], x2 = gs.xs[3 * j + 2];
                    d0 = v[0] * x0 + v[1] * x1 + v[2] * x2;
                    d1 = v[3] * x0 + v[4] * x1 + v[5] * x2;
                    d2 = v[6] * x0 + v[7] * x1 + v[8] * x2;
                } else {
                    d0 = w[3 * j];
                    d1 = w[3 * j + 1];
                    d2 = w[3 * j + 2];
                }
            }
#pragma unroll 8
            for (int rr = rb; rr < re; ++rr) {
                const unsigned long long mk = gs.rmask[rr];
                const bool in = (mk >> lane) & 1ull;
                const double *pw = gs.ws + (int64_t)gs.rstart[rr] + (in ? 3 * __popcll(mk & below) : 0);
                const double a0 = pw[0], a1 = pw[1], a2 = pw[2];
                s0 += in ? a0 : 0.0;
                s1 += in ? a1 : 0.0;
                s2 += in ? a2 : 0.0;
            }
            s0 += d0;
            s1 += d1;
            s2 += d2;
        } else if (j < gs.nrows) {
            s0 = w[3 * j];
            s1 = w[3 * j + 1];
            s2 = w[3 * j + 2];
        }
        nl[wv][3 * lane] = s0;
        nl[wv][3 * lane + 1] = s1;
        nl[wv][3 * lane + 2] = s2;
        __builtin_amdgcn_wave_barrier();
    };
    const int64_t sl0 = (int64_t)blockIdx.x * WPB + wv;
    int64_t sl = sl0;
    // the first slice's gather (and, PRE, its vectors) before the prologue
    // (they need no scalar)
    StageIn in;
    if (threadIdx.x == 0) in = stage_inputs(scal, ist, par);
    double e[3][6];  // u, p, s, x, r, M of the slice's entries
    auto load = [&](int64_t s0) {
#pragma unroll
        for (int ps = 0; ps < 3; ++ps) {
            const int64_t i = s0 * 192 + ps * 64 + lane;
            if (i < n) {
                e[ps][0] = u[i], e[ps][1] = p[i], e[ps][2] = sv[i], e[ps][3] = x[i], e[ps][4] = r[i];
                e[ps][5] = JAC ? dinv[i] : 1.0;
            }
        }
    };
    if (sl < nsl) {
        if constexpr (PRE) load(sl);
        gather(sl);
    }
    if (ist[I_REASON] != 0) return;
    double t[3] = {0.0, 0.0, 0.0};
    if (pro) sums3(pu_in, pu_in + G, G, pu_in + 2 * G, G2, t);
    double alpha, beta;
    if (stage_prologue(pro, t, scal, ist, par, atol, alpha, beta, &in)) return;
    double acc[3] = {0.0, 0.0, 0.0};
    for (; sl < nsl; sl += sst) {
        if (sl != sl0) {
            load(sl);
            gather(sl);
        } else if (!PRE) {
            load(sl);
        }
#pragma unroll
        for (int ps = 0; ps < 3; ++ps) {
            const int el = ps * 64 + lane;
            const int64_t i = sl * 192 + el;
            if (i >= n) break;
            const double wi = nl[wv][el];
            const double pi = e[ps][0] + beta * e[ps][1];
            const double si = wi + beta * e[ps][2];
            p[i] = pi;
            sv[i] = si;
            x[i] = e[ps][3] + alpha * pi;
            const double ri = e[ps][4] - alpha * si;
            r[i] = ri;
            const double ui = JAC ? e[ps][5] * ri : ri;
            u[i] = ui;
            nl[wv][el] = ui;  // (this lane's own entry: read above, by this lane only)
            acc[0] += ri * ui;
            acc[1] += ri * ri;
        }
        __builtin_amdgcn_wave_barrier();
        const int64_t j = sl * 64 + lane;
        if (gs.single && j < gs.nrows && ((gs.single[sl] >> lane) & 1ull)) {
            const double *v = gs.sval + gs.svptr[j];
            const double x0 = nl[wv][3 * lane], x1 = nl[wv][3 * lane + 1], x2 = nl[wv][3 * lane + 2];
            const double d0 = v[0] * x0 + v[1] * x1 + v[2] * x2;
            const double d1 = v[3] * x0 + v[4] * x1 + v[5] * x2;
            const double d2 = v[6] * x0 + v[7] * x1 + v[8] * x2;
            acc[2] += (d0 * x0 + d1 * x1) + d2 * x2;
        }
        __builtin_amdgcn_wave_barrier();  // (nl[wv] read before the next slice's gather writes it)
    }
    block_sums<3>(acc, pu_out, G);
}

// (w, u) per workgroup after the SpMV (no last-arriver: the next update's
// prologue sums the partials); FIN_UNR independent load pairs per thread.
__global__ __launch_bounds__(KB) void k_dot_part(int64_t n, const double *__restrict__ vx,
                                                 const double *__restrict__ vy, double *__restrict__ pd,
                                                 const int *__restrict__ ist)
{
    if (ist[I_REASON] != 0) return;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * KB;
    for (int64_t i0 = blockIdx.x * (int64_t)KB + threadIdx.x; i0 < n; i0 += stride * 4) {
        double v[4];
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) v[uu] = i0 + uu * stride < n ? vx[i0 + uu * stride] * vy[i0 + uu * stride] : 0.0;
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) acc += v[uu];
    }
    double a[1] = {acc};
    block_sums<1>(a, pd, 0);
}

// Dot + reduction + scalar update in one launch: each workgroup forms its
// slice of (x, y) (FIN_UNR independent loads in flight per thread) and of the
// preceding update kernel's NQ0 partial arrays; the last-arriving workgroup
// sums the per-workgroup partials in a fixed order and (one rank) applies the
// stage's scalar update.  Replaces a dot pass + two reduction launches.
// Measured against forming per-row shares of (x, A x) in the SpMV epilogue
// (8 B per row instead of the 16-B-per-entry pass here): the epilogue slowed
// the SpMV by 1.3 % at config 2 and tied on the 1/8 slab (tools/cg_ab.py,
// profiles/r02/cg_ab_rowdot_*.jsonl); 64x1024 / 128x512 shapes were no faster,
// nor 64 / 128 / 512 / 1024 workgroups of 256 (config 2: 801.8 us per
// iteration at 256 vs 803.5-812.4; 1/8 slab 88.9-89.6 for all;
// profiles/r02/fin_blocks_*.jsonl): the launch is a latency chain (loads,
// ticket, last-arriver sum), not bandwidth.
// Hand-off (cdna_hip_programming.md §6 G16, counter form): partials stored
// write-through (agent-scope atomic store = sc1), the storing wave drains
// vmcnt, relaxed agent fetch_add on the ticket; the last arriver takes one
// agent acquire and reads this launch's partials with sc1 loads.  The sum
// order depends only on the sizes, never on which workgroup arrives last:
// bitwise deterministic.
constexpr int FIN_BLOCKS = 256;   // workgroups
constexpr int FIN_THREADS = 256;  // threads per workgroup
constexpr int FIN_UNR = 4;
constexpr int FIN_OFF = PART_STRIDE / 2;  // this launch's per-workgroup partials, slot q
template <int NQ0, int NT>
__global__ __launch_bounds__(NT) void k_dot_finish(int64_t n, const double *__restrict__ vx,
                                                   const double *__restrict__ vy,
                                                   double *__restrict__ partials, int np0, double *__restrict__ scal,
                                                   int *__restrict__ ist, int stage, int fuse, double rtol,
                                                   double atol)
{
    if (stage != ST_SR_START && stage != ST_START && ist[I_REASON] != 0) return;
    constexpr int NQ = NQ0 + 1;
    __shared__ double lds[NQ][NT / 64];
    __shared__ int last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double s[NQ];
    // this workgroup's slice of (x, y): FIN_UNR independent load pairs in
    // flight per thread (a grid-stride loop of single loads is latency bound)
    {
        double acc = 0.0;
        const int64_t stride = (int64_t)gridDim.x * NT;
        for (int64_t i0 = blockIdx.x * (int64_t)NT + threadIdx.x; i0 < n; i0 += stride * FIN_UNR) {
            double v[FIN_UNR];
#pragma unroll
            for (int u = 0; u < FIN_UNR; ++u)
                v[u] = i0 + u * stride < n ? vx[i0 + u * stride] * vy[i0 + u * stride] : 0.0;
#pragma unroll
            for (int u = 0; u < FIN_UNR; ++u) acc += v[u];
        }
        s[NQ0] = acc;
    }
    // and its slice of the update kernel's partials (visible across the launch boundary)
    const int chunk = (np0 + (int)gridDim.x - 1) / (int)gridDim.x;
#pragma unroll
    for (int q = 0; q < NQ0; ++q) {
        double acc = 0.0;
        for (int i = threadIdx.x; i < chunk; i += NT) {
            const int j = blockIdx.x * chunk + i;
            if (j < np0) acc += partials[q * PART_STRIDE + j];
        }
        s[q] = acc;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) s[q] = wsum2(s[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NQ; ++q) lds[q][w] = s[q];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            double t = 0.0;
#pragma unroll
            for (int i = 0; i < NT / 64; ++i) t += lds[q][i];
            __hip_atomic_store(partials + q * PART_STRIDE + FIN_OFF + blockIdx.x, t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = grid_last_arriver(ist + I_TICKET);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;
    // last arriver: the per-workgroup partials of this launch (sc1 loads), fixed order
    const int G = (int)gridDim.x;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        double t = 0.0;
        for (int i = threadIdx.x; i < G; i += NT)
            t += __hip_atomic_load(partials + q * PART_STRIDE + FIN_OFF + i, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        s[q] = wsum2(t);
    }
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NQ; ++q) lds[q][w] = s[q];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            double u = 0.0;
#pragma unroll
            for (int i = 0; i < NT / 64; ++i) u += lds[q][i];
            scal[S_SUM0 + q] = u;
        }
        if (fuse) cg_scalars(stage, scal, ist, rtol, atol);
    }
}

__global__ void k_invert_diag(int64_t n, const double *__restrict__ d, double *__restrict__ dinv)
{
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) dinv[i] = d[i] != 0.0 ? 1.0 / d[i] : 1.0;
}

// y = b - y (true residual)
__global__ void k_bmy(int64_t n, const double *__restrict__ b, double *__restrict__ y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = b[i] - y[i];
}

// ------------------------------------------------------------- GMRES kernels
// h[j] partials of V[:,j] . w for j < k (classical Gram-Schmidt, one pass)
__global__ __launch_bounds__(KB) void k_mdot(int64_t n, int k, const double *const *__restrict__ V,
                                             const double *__restrict__ w, double *__restrict__ partials)
{
    __shared__ double lds[16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int j = 0; j < k; ++j) {
        double s = 0;
        const double *v = V[j];
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
            s += v[i] * w[i];
        s = wsum2(s);
        __syncthreads();
        if (lane == 0) lds[wv] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0;
            for (int i = 0; i < nw; ++i) t += lds[i];
            partials[j * RED_BLOCKS + blockIdx.x] = t;
        }
    }
}

// w -= sum_j h[j] V[:,j]
__global__ __launch_bounds__(KB) void k_maxpy(int64_t n, int k, const double *const *__restrict__ V,
                                              const double *__restrict__ h, double *__restrict__ w)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double s = w[i];
        for (int j = 0; j < k; ++j) s -= h[j] * V[j][i];
        w[i] = s;
    }
}

__global__ void k_reduce_many(const double *__restrict__ partials, int nparts, int nq, double *__restrict__ out)
{
    __shared__ double lds[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int q = 0; q < nq; ++q) {
        double s = 0;
        for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += partials[q * RED_BLOCKS + i];
        s = wsum2(s);
        __syncthreads();
        if (lane == 0) lds[w] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0;
            for (int i = 0; i < nw; ++i) t += lds[i];
            out[q] = t;
        }
    }
}

}  // namespace kle

using namespace kle;

struct kle_ksp {
    kle_ctx *ctx = nullptr;
    std::string type = "cg", pc = "jacobi";
    double rtol = 1e-5, atol = 1e-50, dtol = 1e5;
    int maxit = 10000, restart = 30, fixed = 0, check_every = 8;
    int pipe_par = 0;  // pipelined CG: parity of the next update launch (k_pipe_iter)
    std::string prod_kernel;  // the kernel(s) of the last call's products (kle_ksp_get_product_kernel)
    double prod_bytes = 0.0;  // and the algorithmic bytes each moves (kle_ksp_get_product_bytes)
    kle_mat *A = nullptr;
    kle_vec *r = nullptr, *p = nullptr, *q = nullptr, *dinv = nullptr;
    kle_vec *u = nullptr, *w = nullptr, *s = nullptr;  // single-reduction CG
    kle_vec *m = nullptr, *nv = nullptr, *z = nullptr;  // pipelined CG
    int single_reduction = 0;
    const kle_vec *last_b = nullptr, *last_x = nullptr;  // last fixed-iteration solve (kle_ksp_continue)
    std::vector<kle_vec *> V;  // GMRES basis
    double **d_Vptr = nullptr;
    double *d_h = nullptr;
    double *d_gpart = nullptr;  // GMRES dot partials [restart+2][RED_BLOCKS]
    // PC lu: dense LU factors on the device (rocSOLVER getrf, column major)
    double *d_lu = nullptr;
    rocblas_int *d_ipiv = nullptr, *d_info = nullptr;
    rocblas_handle blas = nullptr;
    bool setup = false;
    int its = 0, reason = 0;
    double rnorm = 0, true_rel = -1;
    int max_corr = g_tune.ksp_refine;  // correction solves on a missed true residual (refine)
    int corr_its = 0;                  // iterations of the last solve's corrections
    int corr_reason = 0;               // converged reason of the last correction (0: none ran)
};

static void free_work(kle_ksp *k)
{
    kle_vec_destroy(k->r);
    kle_vec_destroy(k->p);
    kle_vec_destroy(k->q);
    kle_vec_destroy(k->dinv);
    kle_vec_destroy(k->u);
    kle_vec_destroy(k->w);
    kle_vec_destroy(k->s);
    kle_vec_destroy(k->m);
    kle_vec_destroy(k->nv);
    kle_vec_destroy(k->z);
    k->u = k->w = k->s = k->m = k->nv = k->z = nullptr;
    for (auto v : k->V) kle_vec_destroy(v);
    k->V.clear();
    hipFree(k->d_Vptr);
    hipFree(k->d_h);
    hipFree(k->d_gpart);
    k->d_gpart = nullptr;
    hipFree(k->d_lu);
    hipFree(k->d_ipiv);
    hipFree(k->d_info);
    k->d_lu = nullptr;
    k->d_ipiv = k->d_info = nullptr;
    if (k->blas) rocblas_destroy_handle(k->blas);
    k->blas = nullptr;
    k->r = k->p = k->q = k->dinv = nullptr;
    k->d_Vptr = nullptr;
    k->d_h = nullptr;
    k->setup = false;
}

static int make_vec_like_cols(kle_ksp *k, kle_vec **out)
{
    // a vector in the column space of A (ghosted for nb matrices)
    kle_mat *A = k->A;
    KLE_TRY(vec_alloc(k->ctx, A->n_local, A->n_global, A->col_lo, A->kind == 0 ? A->ghost_lo : 0,
                      A->kind == 0 ? A->ghost_hi : 0, out));
    (*out)->bs = A->C;
    (*out)->lo_rank = A->lo_rank;
    (*out)->hi_rank = A->hi_rank;
    (*out)->send_lo = A->send_lo;
    (*out)->send_hi = A->send_hi;
    (*out)->plan = A->plan;
    return 0;
}

// First level of a two-level reduction: 64 workgroups each sum a contiguous
// chunk of the partials (fixed order) into partials[q*PART_STRIDE + PART2 + g].
constexpr int PART2_OFF = PART_STRIDE - 128;
constexpr int PART2_N = 64;
__global__ __launch_bounds__(1024) void k_reduce_l1(double *__restrict__ partials, NParts np, int nq,
                                                    const int *__restrict__ ist, int stage)
{
    if (stage != ST_START && stage != ST_SR_START && ist[I_REASON] != 0) return;
    __shared__ double lds[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int q = 0; q < nq; ++q) {
        const int nparts = np.n[q];
        const int chunk = (nparts + PART2_N - 1) / PART2_N;
        const int lo = blockIdx.x * chunk, hi = min(nparts, lo + chunk);
        double s = 0;
        for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) s += partials[q * PART_STRIDE + i];
        s = wsum2(s);
        __syncthreads();
        if (lane == 0) lds[w] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0;
            for (int i = 0; i < nw; ++i) t += lds[i];
            partials[q * PART_STRIDE + PART2_OFF + blockIdx.x] = t;
        }
    }
}

static int reduce_stage(kle_ksp *k, NParts np, int nq, int stage, hipStream_t st = nullptr)
{
    kle_ctx *c = k->ctx;
    if (!st) st = c->stream;
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(c->tic("reduce", &ev, st));
    const double *parts = c->d_partials;
    int big = 0;
    for (int q = 0; q < nq; ++q) big |= np.n[q] > 4096;
    if (big) {
        // first level per quantity (small quantities just copy through)
        hipLaunchKernelGGL(k_reduce_l1, dim3(PART2_N), dim3(1024), 0, st, c->d_partials, np, nq,
                           c->d_istate, stage);
        parts = c->d_partials + PART2_OFF;
        for (int q = 0; q < nq; ++q) np.n[q] = PART2_N;
    }
    const int fuse = c->nranks == 1 && !c->comm;
    hipLaunchKernelGGL(k_reduce_stage, dim3(1), dim3(1024), 0, st, parts, np, nq, c->d_scal,
                       c->d_istate, stage, fuse, k->rtol, k->atol);
    KLE_HIP(hipGetLastError());
    KLE_TRY(c->toc("reduce", &ev, st));
    if (!fuse) {
        KLE_TRY(allreduce_sum(c, c->d_scal + S_SUM0, nq, st));
        hipLaunchKernelGGL(k_scalars, dim3(1), dim3(1), 0, st, c->d_scal, c->d_istate, stage, k->rtol, k->atol);
        KLE_HIP(hipGetLastError());
    }
    return 0;
}

// y = A x, then k_dot_finish: (x, y) + the NQ0 update-kernel sums + the
// scalar stage.  On N ranks (or a one-rank RCCL communicator) the raw sums
// are allreduced and the scalar stage runs behind them.
static int spmv_finish(kle_ksp *k, kle_vec *x, kle_vec *y, int nq0, int np0, int stage, const int *istate)
{
    kle_ctx *c = k->ctx;
    KLE_TRY(spmv(k->A, x, y, istate));
    std::pair<hipEvent_t, hipEvent_t> ev;
    KLE_TRY(c->tic("reduce", &ev));
    const int fuse = c->nranks == 1 && !c->comm;
    const int g = grid_for(x->n_local, FIN_THREADS * FIN_UNR, FIN_BLOCKS);
    if (nq0 == 2)
        hipLaunchKernelGGL((k_dot_finish<2, FIN_THREADS>), dim3(g), dim3(FIN_THREADS), 0, c->stream, x->n_local, x->d,
                           y->d, c->d_partials, np0, c->d_scal, c->d_istate, stage, fuse, k->rtol, k->atol);
    else
        hipLaunchKernelGGL((k_dot_finish<0, FIN_THREADS>), dim3(g), dim3(FIN_THREADS), 0, c->stream, x->n_local, x->d,
                           y->d, c->d_partials, np0, c->d_scal, c->d_istate, stage, fuse, k->rtol, k->atol);
    KLE_HIP(hipGetLastError());
    KLE_TRY(c->toc("reduce", &ev));
    if (!fuse) {
        KLE_TRY(allreduce_sum(c, c->d_scal + S_SUM0, nq0 + 1));
        hipLaunchKernelGGL(k_scalars, dim3(1), dim3(1), 0, c->stream, c->d_scal, c->d_istate, stage, k->rtol, k->atol);
        KLE_HIP(hipGetLastError());
    }
    return 0;
}

static int poll_state(kle_ksp *k)
{
    kle_ctx *c = k->ctx;
    KLE_HIP(hipMemcpyAsync(c->h_istate, c->d_istate, sizeof(int) * I_COUNT, hipMemcpyDeviceToHost, c->stream));
    KLE_HIP(hipMemcpyAsync(c->h_scal, c->d_scal, sizeof(double) * NSCAL, hipMemcpyDeviceToHost, c->stream));
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

static int true_residual(kle_ksp *k, kle_vec *b, kle_vec *x)
{
    kle_ctx *c = k->ctx;
    // q = A x ; q = b - q ; ||q|| / ||b||
    KLE_HIP(hipMemcpyAsync(k->p->d, x->d, sizeof(double) * x->n_local, hipMemcpyDeviceToDevice, c->stream));
    KLE_TRY(spmv(k->A, k->p, k->q, nullptr));
    hipLaunchKernelGGL(k_bmy, dim3(grid_for(b->n_local, KB, RED_BLOCKS)), dim3(KB), 0, c->stream, b->n_local, b->d,
                       k->q->d);
    KLE_HIP(hipGetLastError());
    double rn, bn;
    KLE_TRY(kle_vec_norm2(k->q, &rn));
    KLE_TRY(kle_vec_norm2(b, &bn));
    k->true_rel = bn > 0 ? rn / bn : rn;
    return 0;
}

static int solve_cg(kle_ksp *k, kle_vec *b, kle_vec *x)
{
    kle_ctx *c = k->ctx;
    const int64_t n = b->n_local;
    const bool jac = k->pc == "jacobi";
    const double *dinv = jac ? k->dinv->d : nullptr;
    const int g = grid_for(n, KB, RED_BLOCKS);
    int host_fixed[I_COUNT] = {0, 0, k->fixed, k->fixed ? k->fixed : k->maxit, 0, 0, 0, 0};
    KLE_HIP(hipMemcpyAsync(c->d_istate, host_fixed, sizeof(int) * I_COUNT, hipMemcpyHostToDevice, c->stream));
    if (jac)
        hipLaunchKernelGGL(k_cg_start<true>, dim3(g), dim3(KB), 0, c->stream, n, b->d, dinv, x->d, k->r->d, k->p->d,
                           c->d_partials);
    else
        hipLaunchKernelGGL(k_cg_start<false>, dim3(g), dim3(KB), 0, c->stream, n, b->d, dinv, x->d, k->r->d, k->p->d,
                           c->d_partials);
    KLE_HIP(hipGetLastError());
    KLE_TRY(reduce_stage(k, NParts{{g, g, 0, 0}}, 2, ST_START));
    const int limit = k->fixed ? k->fixed : k->maxit;
    std::pair<hipEvent_t, hipEvent_t> ev;
    for (int it = 0; it < limit; ++it) {
        KLE_TRY(c->tic("p_update", &ev));
        if (jac)
            hipLaunchKernelGGL(k_cg_p<true>, dim3(g), dim3(KB), 0, c->stream, n, k->r->d, dinv, k->p->d, c->d_scal,
                               c->d_istate);
        else
            hipLaunchKernelGGL(k_cg_p<false>, dim3(g), dim3(KB), 0, c->stream, n, k->r->d, dinv, k->p->d, c->d_scal,
                               c->d_istate);
        KLE_HIP(hipGetLastError());
        KLE_TRY(c->toc("p_update", &ev));
        KLE_TRY(spmv_finish(k, k->p, k->q, 0, 0, ST_ALPHA, c->d_istate));
        KLE_TRY(c->tic("cg_update", &ev));
        if (jac)
            hipLaunchKernelGGL(k_cg_update<true>, dim3(g), dim3(KB), 0, c->stream, n, k->p->d, k->q->d, dinv, x->d,
                               k->r->d, c->d_partials, c->d_scal, c->d_istate);
        else
            hipLaunchKernelGGL(k_cg_update<false>, dim3(g), dim3(KB), 0, c->stream, n, k->p->d, k->q->d, dinv, x->d,
                               k->r->d, c->d_partials, c->d_scal, c->d_istate);
        KLE_HIP(hipGetLastError());
        KLE_TRY(c->toc("cg_update", &ev));
        KLE_TRY(reduce_stage(k, NParts{{g, g, 0, 0}}, 2, ST_BETA));
        if (!k->fixed && ((it + 1) % k->check_every == 0)) {
            KLE_TRY(poll_state(k));
            if (c->h_istate[I_REASON] != 0) break;
        }
    }
    KLE_TRY(poll_state(k));
    k->its = c->h_istate[I_ITS];
    k->reason = c->h_istate[I_REASON];
    if (k->reason == 0) k->reason = k->fixed ? KLE_CONVERGED_ITS : KLE_DIVERGED_ITS;
    k->rnorm = std::sqrt(c->h_scal[S_RR]);
    return 0;
}

// The kernel names a solve's products launch, as rocprof lists them: the
// matrix's own (kle_mat_spmv_kernel), or a split product's -- the bricks
// (with their (y, x) shares: dot) and, on a slab partition, the ghost
// slices' gather
static std::string mat_kernel_name(const kle_mat *A)
{
    char buf[160];
    if (kle_mat_spmv_kernel(A, buf, sizeof buf)) return "?";
    return buf;
}
static double mat_bytes(const kle_mat *A)
{
    double b = 0.0;
    return kle_mat_spmv_bytes(A, &b) ? 0.0 : b;
}
static std::string split_kernel_name(const kle_mat *A, bool dot)
{
    const std::string m = mat_kernel_name(A);
    const bool dist = A->ctx->nranks > 1 && (A->lo_rank >= 0 || A->hi_rank >= 0);
    if (dist) return m;
    const size_t plus = m.find('+');
    std::string b = plus == std::string::npos ? m : m.substr(0, plus);
    if (dot) b.replace(b.rfind("false>"), 6, "true>");
    return b;
}

// Chronopoulos-Gear CG (PETSc -ksp_cg_single_reduction): one fused update
// kernel + one SpMV (with fused (w,u)) + one reduction (three sums) per
// iteration -> one allreduce per iteration across ranks.
// cont: continue the previous fixed-iteration solve's recurrence (no start)
static int solve_cg_single(kle_ksp *k, kle_vec *b, kle_vec *x, bool cont)
{
    kle_ctx *c = k->ctx;
    const int64_t n = b->n_local;
    const bool jac = k->pc == "jacobi";
    const double *dinv = jac ? k->dinv->d : nullptr;
    const int g = grid_for(n, KB, RED_BLOCKS);
    int host_fixed[I_COUNT] = {0, 0, k->fixed, k->fixed ? k->fixed : k->maxit, 0, 0, 0, 0};
    KLE_HIP(hipMemcpyAsync(c->d_istate, host_fixed, sizeof(int) * I_COUNT, hipMemcpyHostToDevice, c->stream));
    if (!cont) {
        if (jac)
            hipLaunchKernelGGL(k_sr_start<true>, dim3(g), dim3(KB), 0, c->stream, n, b->d, dinv, x->d, k->r->d,
                               k->u->d, k->p->d, k->s->d, c->d_partials);
        else
            hipLaunchKernelGGL(k_sr_start<false>, dim3(g), dim3(KB), 0, c->stream, n, b->d, dinv, x->d, k->r->d,
                               k->u->d, k->p->d, k->s->d, c->d_partials);
        KLE_HIP(hipGetLastError());
        KLE_TRY(spmv_finish(k, k->u, k->w, 2, g, ST_SR_START, nullptr));
    }
    const int limit = k->fixed ? k->fixed : k->maxit;
    std::pair<hipEvent_t, hipEvent_t> ev;
    // pro_mode (default): the scalar stage runs in the next update's prologue
    // (k_sr_iter) and the (w, u) dot is a plain partial launch -- no
    // last-arriver ticket, no scalar kernel (as the pipelined CG, §3).  Per
    // parity one buffer [2][G] update partials | [Gd] dot partials; on N ranks
    // (or a one-rank RCCL communicator) it is allreduced as one array after
    // the dot (G, Gd equal on every rank), then the next prologue reads it.  A
    // flush closes the call.  Against update + SpMV + k_dot_finish (last-
    // arriver sum + stage): config 2 782.3 vs 782.3 us per iteration, 1/8
    // slab 85.65 vs 88.29 (profiles/r02/sr_prologue_*.jsonl).
    const bool pro_mode = true;
    const bool fuse = c->nranks == 1 && !c->comm;
    // grids capped at 1024 update / 512 dot workgroups: every prologue reads
    // all 2 Gu + Gd partials (config 2: 788.5 vs 792.4 us per iteration with
    // 2048 / 1024; the 1/8 slab is below both caps; profiles/r02/grids_*.jsonl)
    int Gu = grid_for(n, KB, PRO_UPD_BLOCKS), Gd = grid_for(n, KB * 4, PRO_DOT_BLOCKS);
    // one rank with the symmetric SpMV: its gather forms the (w, u) partials
    // (spmv_dot), one launch less per iteration
    const int Gf = c->nranks == 1 && !c->comm ? spmv_dot_parts(k->A) : 0;
    if (Gf > 0 && 2 * Gu + Gf <= PART_STRIDE / 2) Gd = Gf;
    // one rank on box bricks: the product's gather folded into the next
    // update (k_sr_iter_g), whose prologue sums (w, u) from the one-block
    // rows' share (the previous update's) and the bricks' (the product's);
    // npend: w awaits that gather
    // From 2^17 node rows (1, default): config 2 (342k rows) 425.3 -> 422.2 us
    // per iteration, the 1/8 slab (47k rows, a third of the update's waves
    // with a slice) 59.7 -> 61.2 (profiles/r06/cg_ab_sr_fused_gather_*.jsonl)
    const bool gfuse = (g_tune.ksp_sr_gather == 2 || (g_tune.ksp_sr_gather == 1 && k->A->nrows >= (1 << 17))) &&
                       c->nranks == 1 && !c->comm && spmv_can_split(k->A) &&
                       3 * Gu + k->A->nbricks <= PART_STRIDE / 2;
    if (gfuse) Gd = Gu + k->A->nbricks;
    bool npend = false;
    k->prod_kernel = gfuse ? split_kernel_name(k->A, true) : mat_kernel_name(k->A);
    k->prod_bytes = gfuse ? brick_split_bytes(k->A) : mat_bytes(k->A);
    if (pro_mode && c->nranks > 1) {
        std::vector<int64_t> all;
        KLE_TRY(allgather_i64(c, ((int64_t)Gu << 20) | Gd, all));
        for (int64_t v : all) {
            Gu = std::max<int>(Gu, (int)(v >> 20));
            Gd = std::max<int>(Gd, (int)(v & ((1 << 20) - 1)));
        }
    }
    double *const pu[2] = {c->d_partials + 3 * (int64_t)PART_STRIDE,
                           c->d_partials + 3 * (int64_t)PART_STRIDE + PART_STRIDE / 2};
    if (!cont) k->pipe_par = 0;
    int par = k->pipe_par;
    bool pending = false;  // an update's partials await the next launch's prologue
    auto iteration = [&]() -> int {
        KLE_TRY(c->tic("cg_update", &ev));
        {
            auto go = [&](auto kern) {
                hipLaunchKernelGGL(kern, dim3(Gu), dim3(KB), 0, c->stream, n, dinv, k->w->d, k->u->d, k->p->d,
                                   k->s->d, x->d, k->r->d, pu[par], pu[par] + 2 * Gu, Gd, pu[par ^ 1], c->d_scal,
                                   c->d_istate, (int)pending, par, k->atol);
            };
            auto gog = [&](auto kern) {
                BrickGather gs = brick_gather_src(k->A, k->u);
                if (!npend) gs.ng = 0;  // (w complete: read it)
                hipLaunchKernelGGL(kern, dim3(Gu), dim3(KB), 0, c->stream, gs, n, dinv, k->w->d, k->u->d, k->p->d,
                                   k->s->d, x->d, k->r->d, pu[par], Gd, pu[par ^ 1], c->d_scal, c->d_istate,
                                   (int)pending, par, k->atol);
            };
            const bool unr = g_tune.upd_unroll == 2 && g_tune.upd_preload;
            if (gfuse) {
                // (w complete -- the first update of a call -- the same
                // kernel reads it: W + n iterations equal one call, bitwise)
                if (jac) gog(g_tune.upd_preload ? k_sr_iter_g<true, true> : k_sr_iter_g<true, false>);
                else gog(g_tune.upd_preload ? k_sr_iter_g<false, true> : k_sr_iter_g<false, false>);
                npend = false;
            } else if (jac && (g_tune.upd_nt == 1 || (g_tune.upd_nt == 2 && n >= 2000000)))
                go(unr ? k_sr_iter<true, true, true, 2> : g_tune.upd_preload ? k_sr_iter<true, true, true> : k_sr_iter<true, false, true>);
            else if (jac) go(unr ? k_sr_iter<true, true, false, 2> : g_tune.upd_preload ? k_sr_iter<true, true> : k_sr_iter<true, false>);
            else go(g_tune.upd_preload ? k_sr_iter<false, true> : k_sr_iter<false, false>);
            KLE_HIP(hipGetLastError());
            KLE_TRY(c->toc("cg_update", &ev));
            par ^= 1;
            pending = true;
            int nd = 0;
            if (gfuse) {
                KLE_TRY(spmv_split(k->A, k->u, k->w, c->d_istate, pu[par] + 3 * Gu));
                npend = true;
                nd = Gd;  // (the update's one-block share + the bricks')
            } else if (Gd == Gf) KLE_TRY(spmv_dot(k->A, k->u, k->w, c->d_istate, pu[par] + 2 * Gu, &nd));
            else KLE_TRY(spmv(k->A, k->u, k->w, c->d_istate));
            if (nd != Gd) {
                KLE_TRY(c->tic("reduce", &ev));
                hipLaunchKernelGGL(k_dot_part, dim3(Gd), dim3(KB), 0, c->stream, n, k->u->d, k->w->d,
                                   pu[par] + 2 * Gu, c->d_istate);
                KLE_HIP(hipGetLastError());
                KLE_TRY(c->toc("reduce", &ev));
            }
            if (!fuse) KLE_TRY(allreduce_sum(c, pu[par], 2 * Gu + Gd));
            return 0;
        }
        return 0;
    };
    int it = 0;
    for (; it < limit; ++it) {
        KLE_TRY(iteration());
        if (!k->fixed && ((it + 1) % k->check_every == 0)) {
            KLE_TRY(poll_state(k));
            if (c->h_istate[I_REASON] != 0) break;
        }
    }
    if (pro_mode && pending) {
        hipLaunchKernelGGL(k_cg_flush, dim3(1), dim3(KB), 0, c->stream, pu[par], pu[par] + Gu, Gu, pu[par] + 2 * Gu,
                           Gd, c->d_scal, c->d_istate, par, k->atol);
        KLE_HIP(hipGetLastError());
    }
    // (w complete when the call returns: a continuation's first update reads it)
    if (npend) KLE_TRY(brick_gather_rest(k->A, k->u, k->w, c->d_istate, 1));
    k->pipe_par = par;
    KLE_TRY(poll_state(k));
    k->its = c->h_istate[I_ITS];
    k->reason = c->h_istate[I_REASON];
    if (k->reason == 0) k->reason = k->fixed ? KLE_CONVERGED_ITS : KLE_DIVERGED_ITS;
    k->rnorm = std::sqrt(c->h_scal[S_RR]);
    return 0;
}


// Pipelined CG (PETSc KSPPIPECG): the reduction of iteration i (and its
// allreduce across ranks) runs on the comm stream while the SpMV n = A m of
// the same iteration runs on the compute stream.  Same scalar recurrence as
// the single-reduction CG (stages ST_SR_START / ST_SR).
static int solve_pipecg(kle_ksp *k, kle_vec *b, kle_vec *x, bool cont)
{
    kle_ctx *c = k->ctx;
    const int64_t n = b->n_local;
    const bool jac = k->pc == "jacobi";
    const double *dinv = jac ? k->dinv->d : nullptr;
    const int g = grid_for(n, KB, RED_BLOCKS);
    int host_fixed[I_COUNT] = {0, 0, k->fixed, k->fixed ? k->fixed : k->maxit, 0, 0, 0, 0};
    KLE_HIP(hipMemcpyAsync(c->d_istate, host_fixed, sizeof(int) * I_COUNT, hipMemcpyHostToDevice, c->stream));
    if (!cont) {
        if (jac)
            hipLaunchKernelGGL(k_sr_start<true>, dim3(g), dim3(KB), 0, c->stream, n, b->d, dinv, x->d, k->r->d,
                               k->u->d, k->p->d, k->s->d, c->d_partials);
        else
            hipLaunchKernelGGL(k_sr_start<false>, dim3(g), dim3(KB), 0, c->stream, n, b->d, dinv, x->d, k->r->d,
                               k->u->d, k->p->d, k->s->d, c->d_partials);
        KLE_HIP(hipGetLastError());
        KLE_TRY(spmv_finish(k, k->u, k->w, 2, g, ST_SR_START, nullptr));  // w = A u, (w,u), scalars
        if (jac)
            hipLaunchKernelGGL(k_pipe_init<true>, dim3(g), dim3(KB), 0, c->stream, n, dinv, k->w->d, k->m->d,
                               k->z->d, k->q->d);
        else
            hipLaunchKernelGGL(k_pipe_init<false>, dim3(g), dim3(KB), 0, c->stream, n, dinv, k->w->d, k->m->d,
                               k->z->d, k->q->d);
        KLE_HIP(hipGetLastError());
    }
    // box bricks: each product n = A m leaves its owned rows' gather to the
    // next update (k_pipe_iter_g); npend: n awaits that gather
    const bool gfuse = g_tune.ksp_pipe_gather && spmv_can_split(k->A);
    const bool gdist = c->nranks > 1 && (k->A->lo_rank >= 0 || k->A->hi_rank >= 0);
    k->prod_kernel = gfuse ? split_kernel_name(k->A, false) : mat_kernel_name(k->A);
    k->prod_bytes = gfuse ? brick_split_bytes(k->A) : mat_bytes(k->A);  // (N > 1: the ghost slices' gather not counted)
    bool npend = false;
    auto product = [&](const int *ist) -> int {
        if (!gfuse) return spmv(k->A, k->m, k->nv, ist);
        KLE_TRY(spmv_split(k->A, k->m, k->nv, ist));
        npend = true;
        return 0;
    };
    if (!cont) KLE_TRY(product(nullptr));  // n = A m
    // the allreduce may run beside the SpMV only where the SpMV's own halo uses
    // the comm stream too (one RCCL stream: halo, then allreduce)
    const bool side = spmv_uses_comm_stream(k->A, k->m);
    const int fuse = c->nranks == 1 && !c->comm;
    // every rank launches the update with the same grid, so the [3][G]
    // partials allreduce element-wise; capped like the single-reduction update
    int G = grid_for(n, KB, PRO_UPD_BLOCKS);
    if (c->nranks > 1) {
        std::vector<int64_t> all;
        KLE_TRY(allgather_i64(c, G, all));
        for (int64_t v : all) G = std::max<int>(G, (int)v);
    }
    double *const pp[2] = {c->d_partials + 3 * (int64_t)PART_STRIDE, c->d_partials + 3 * (int64_t)PART_STRIDE +
                                                                          PART_STRIDE / 2};
    if (!cont) k->pipe_par = 0;
    int par = k->pipe_par;
    bool pending = false;  // a launch's partials await the next launch's prologue
    hipEvent_t ev_red = nullptr;
    KLE_HIP(hipEventCreateWithFlags(&ev_red, sync_event_flags()));
    const int limit = k->fixed ? k->fixed : k->maxit;
    std::pair<hipEvent_t, hipEvent_t> ev;
    int rc = 0;
    for (int it = 0; it < limit && !rc; ++it) {
        rc = c->tic("cg_update", &ev);
        if (rc) break;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(G), dim3(KB), 0, c->stream, n, dinv, k->nv->d, k->z->d, k->q->d, k->s->d,
                               k->p->d, x->d, k->r->d, k->u->d, k->w->d, k->m->d, pp[par], pp[par ^ 1], c->d_scal,
                               c->d_istate, (int)pending, par, k->atol);
        };
        auto gog = [&](auto kern) {
            BrickGather gs = brick_gather_src(k->A, k->m);
            if (!npend) gs.ng = gs.nrecv = 0;  // (n complete: read it)
            hipLaunchKernelGGL(kern, dim3(G), dim3(KB), 0, c->stream, gs, n, dinv,
                               k->nv->d, k->z->d, k->q->d, k->s->d, k->p->d, x->d, k->r->d, k->u->d, k->w->d,
                               k->m->d, pp[par], pp[par ^ 1], c->d_scal, c->d_istate, (int)pending, par, k->atol);
        };
        if (gfuse) {
            // (n complete -- the first update of a continued call -- the
            // same kernel reads it: the same arithmetic in the same order as
            // one uninterrupted solve, bitwise)
            if (jac) gog(k_pipe_iter_g<true>);
            else gog(k_pipe_iter_g<false>);
            npend = false;
        } else if (jac) {
            go(g_tune.upd_preload ? k_pipe_iter<true, true> : k_pipe_iter<true, false>);
        } else {
            go(g_tune.upd_preload ? k_pipe_iter<false, true> : k_pipe_iter<false, false>);
        }
        if (hipGetLastError() != hipSuccess) { rc = fail(KLE_ERR_DEVICE, "k_pipe_iter launch failed"); break; }
        if ((rc = c->toc("cg_update", &ev))) break;
        par ^= 1;
        pending = true;
        if (fuse) {
            // one rank: the next launch's prologue reduces these partials
            if ((rc = product(c->d_istate))) break;
        } else if (side && c->nranks > 1) {
            // the partials' allreduce on the comm stream behind the halo, beside
            // the SpMV; the overlapped SpMV already makes the comm stream wait
            // for the update (ev_x_ready), so no event of its own: each event
            // record / cross-stream wait costs ~2.5 us on the critical path
            // (profiles/r02/sync_cost_eighth.jsonl)
            // (a split product's reverse halo went first on the comm stream:
            // the wait for the allreduce covers the received sums too)
            if ((rc = product(c->d_istate))) break;
            if ((rc = allreduce_sum(c, pp[par], 3 * G, c->comm_stream))) break;
            if (hipEventRecord(ev_red, c->comm_stream) != hipSuccess ||
                hipStreamWaitEvent(c->stream, ev_red, 0) != hipSuccess) {
                rc = fail(KLE_ERR_DEVICE, "event record/wait failed");
                break;
            }
        } else {
            // no overlap possible on this rank (or a one-rank RCCL
            // communicator): same collective order as the overlapping ranks
            // (halo, then allreduce), all on one stream
            if ((rc = product(c->d_istate))) break;
            if (gfuse && gdist && k->A->halo_overlap &&
                hipStreamWaitEvent(c->stream, c->ev_halo_done, 0) != hipSuccess) {  // (the received sums)
                rc = fail(KLE_ERR_DEVICE, "event wait failed");
                break;
            }
            if ((rc = allreduce_sum(c, pp[par], 3 * G, c->stream))) break;
        }
        if (!k->fixed && ((it + 1) % k->check_every == 0)) {
            if ((rc = poll_state(k))) break;
            if (c->h_istate[I_REASON] != 0) break;
        }
    }
    if (!rc && pending) {
        hipLaunchKernelGGL(k_cg_flush, dim3(1), dim3(KB), 0, c->stream, pp[par], pp[par] + G, G, pp[par] + 2 * G, G,
                           c->d_scal, c->d_istate, par, k->atol);
        if (hipGetLastError() != hipSuccess) rc = fail(KLE_ERR_DEVICE, "k_cg_flush launch failed");
    }
    // (n complete when the call returns: a continuation starts with the plain
    // update, and nothing may clobber the bricks' sums in between)
    if (!rc && npend) rc = brick_gather_rest(k->A, k->m, k->nv, c->d_istate, 1);
    k->pipe_par = par;
    hipEventDestroy(ev_red);
    if (rc) return rc;
    KLE_TRY(poll_state(k));
    k->its = c->h_istate[I_ITS];
    k->reason = c->h_istate[I_REASON];
    if (k->reason == 0) k->reason = k->fixed ? KLE_CONVERGED_ITS : KLE_DIVERGED_ITS;
    k->rnorm = std::sqrt(c->h_scal[S_RR]);
    return 0;
}

// ------------------------------------------------------------------ GMRES
static int gmres_dots(kle_ksp *k, int kk, const kle_vec *w, double *h)
{
    kle_ctx *c = k->ctx;
    const int64_t n = w->n_local;
    const int g = grid_for(n, KB, RED_BLOCKS);
    hipLaunchKernelGGL(k_mdot, dim3(g), dim3(KB), 0, c->stream, n, kk, (const double *const *)k->d_Vptr, w->d,
                       k->d_gpart);
    hipLaunchKernelGGL(k_reduce_many, dim3(1), dim3(1024), 0, c->stream, k->d_gpart, g, kk, k->d_h);
    KLE_HIP(hipGetLastError());
    KLE_TRY(allreduce_sum(c, k->d_h, kk));
    KLE_HIP(hipMemcpyAsync(h, k->d_h, sizeof(double) * kk, hipMemcpyDeviceToHost, c->stream));
    KLE_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

static int solve_gmres(kle_ksp *k, kle_vec *b, kle_vec *x)
{
    // right-preconditioned GMRES(m): A M^-1 u = b, x = M^-1 u; the residual
    // norm is the true (unpreconditioned) one, as for CG.
    kle_ctx *c = k->ctx;
    const int m = k->restart;
    const bool jac = k->pc == "jacobi";
    const int64_t n = b->n_local;
    KLE_TRY(kle_vec_set(x, 0.0));
    double bn;
    KLE_TRY(kle_vec_norm2(b, &bn));
    const double tol = std::max(k->rtol * bn, k->atol);
    std::vector<double> H((m + 1) * m), cs(m), sn(m), gvec(m + 1), hcol(m + 1);
    k->its = 0;
    k->reason = 0;
    double rn = bn;
    if (rn <= tol) {
        k->reason = rn <= k->atol ? KLE_CONVERGED_ATOL : KLE_CONVERGED_RTOL;
        k->rnorm = rn;
        return 0;
    }
    kle_vec *z = k->q;  // scratch for M^-1 v
    while (true) {
        // r = b - A x  -> V0
        KLE_HIP(hipMemcpyAsync(k->p->d, x->d, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
        KLE_TRY(spmv(k->A, k->p, k->V[0], nullptr));
        hipLaunchKernelGGL(k_bmy, dim3(grid_for(n, KB, RED_BLOCKS)), dim3(KB), 0, c->stream, n, b->d, k->V[0]->d);
        KLE_TRY(kle_vec_norm2(k->V[0], &rn));
        if (rn <= tol) break;
        KLE_TRY(kle_vec_scale(k->V[0], 1.0 / rn));
        std::fill(gvec.begin(), gvec.end(), 0.0);
        gvec[0] = rn;
        int j = 0;
        for (; j < m && k->its < k->maxit; ++j) {
            // w = A M^-1 v_j
            if (jac) KLE_TRY(kle_vec_pointwise_mult(z, k->dinv, k->V[j]));
            else KLE_TRY(kle_vec_copy(k->V[j], z));
            KLE_TRY(spmv(k->A, z, k->V[j + 1], nullptr));
            // two passes of classical Gram-Schmidt (CGS2)
            std::fill(hcol.begin(), hcol.end(), 0.0);
            for (int pass = 0; pass < 2; ++pass) {
                std::vector<double> h(j + 1);
                KLE_TRY(gmres_dots(k, j + 1, k->V[j + 1], h.data()));
                KLE_HIP(hipMemcpyAsync(k->d_h, h.data(), sizeof(double) * (j + 1), hipMemcpyHostToDevice, c->stream));
                hipLaunchKernelGGL(k_maxpy, dim3(grid_for(n, KB, RED_BLOCKS)), dim3(KB), 0, c->stream, n, j + 1,
                                   (const double *const *)k->d_Vptr, k->d_h, k->V[j + 1]->d);
                KLE_HIP(hipGetLastError());
                for (int i = 0; i <= j; ++i) hcol[i] += h[i];
            }
            double hn;
            KLE_TRY(kle_vec_norm2(k->V[j + 1], &hn));
            hcol[j + 1] = hn;
            if (hn > 0) KLE_TRY(kle_vec_scale(k->V[j + 1], 1.0 / hn));
            for (int i = 0; i < j; ++i) {  // apply previous rotations
                double t = cs[i] * hcol[i] + sn[i] * hcol[i + 1];
                hcol[i + 1] = -sn[i] * hcol[i] + cs[i] * hcol[i + 1];
                hcol[i] = t;
            }
            double den = std::hypot(hcol[j], hcol[j + 1]);
            cs[j] = den > 0 ? hcol[j] / den : 1.0;
            sn[j] = den > 0 ? hcol[j + 1] / den : 0.0;
            hcol[j] = den;
            hcol[j + 1] = 0;
            gvec[j + 1] = -sn[j] * gvec[j];
            gvec[j] = cs[j] * gvec[j];
            for (int i = 0; i <= j; ++i) H[i * m + j] = hcol[i];
            ++k->its;
            rn = std::fabs(gvec[j + 1]);
            if (rn <= tol || hn == 0) {
                ++j;
                break;
            }
        }
        // solve H y = g, x += M^-1 V y
        std::vector<double> y(j);
        for (int i = j - 1; i >= 0; --i) {
            double s = gvec[i];
            for (int l = i + 1; l < j; ++l) s -= H[i * m + l] * y[l];
            y[i] = s / H[i * m + i];
        }
        KLE_HIP(hipMemcpyAsync(k->d_h, y.data(), sizeof(double) * j, hipMemcpyHostToDevice, c->stream));
        // z = - sum y_i v_i  (k_maxpy subtracts), then x += M^-1 (-z)
        KLE_TRY(kle_vec_set(z, 0.0));
        hipLaunchKernelGGL(k_maxpy, dim3(grid_for(n, KB, RED_BLOCKS)), dim3(KB), 0, c->stream, n, j,
                           (const double *const *)k->d_Vptr, k->d_h, z->d);
        KLE_HIP(hipGetLastError());
        if (jac) KLE_TRY(kle_vec_pointwise_mult(z, k->dinv, z));
        KLE_TRY(kle_vec_axpy(x, -1.0, z));
        if (rn <= tol) break;
        if (k->its >= k->maxit) {
            k->reason = KLE_DIVERGED_ITS;
            break;
        }
    }
    if (!k->reason) k->reason = rn <= k->atol ? KLE_CONVERGED_ATOL : KLE_CONVERGED_RTOL;
    k->rnorm = rn;
    return 0;
}

// ---------------------------------------------------------------- PC lu
// The reference's solver is KSPPREONLY + PCLU (makefile:7; kle_solver.py:54-64
// configures gmres + lu).  On the device: the operator densified column-major
// and factored once by rocSOLVER (getrf, partial pivoting); every solve is one
// getrs.  Sequential only -- like PETSc's own LU, which needs an external
// package (MUMPS, SuperLU_dist) for a parallel matrix -- and dense, so sizes
// stay below LU_MAX_N (config 1, unit tests); the large systems use CG.
constexpr int64_t LU_MAX_N = 40000;

__global__ void k_densify_nb(int64_t nrows, int R, int C, int lay, const int *__restrict__ rowptr,
                             const int *__restrict__ rowcnt, const int64_t *__restrict__ vptr,
                             const int *__restrict__ bcol, const double *__restrict__ val, double *__restrict__ D,
                             int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    const int b0 = rowptr[i], mp = rowptr[i + 1] - b0, m = rowcnt ? rowcnt[i] : mp;
    const double *v = val + vptr[i];
    for (int k = 0; k < m; ++k) {
        const int64_t j = bcol[b0 + k];
        for (int a = 0; a < R; ++a)
            for (int b = 0; b < C; ++b) D[(j * C + b) * n + i * R + a] += v[vofs(lay, R * C, a * C + b, k, m, mp)];
    }
}

__global__ void k_densify_aij(int64_t m, const int64_t *__restrict__ ptr, const int *__restrict__ col,
                              const double *__restrict__ val, double *__restrict__ D, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) D[(int64_t)col[k] * n + i] += val[k];
}

static int lu_factor(kle_ksp *k)
{
    kle_ctx *c = k->ctx;
    kle_mat *A = k->A;
    if (c->nranks > 1)
        return fail(KLE_ERR_SUP, "PC lu on %d ranks needs a parallel direct solver (PETSc: MUMPS / SuperLU_dist); "
                                 "use -ksp_type cg -pc_type jacobi (K is SPD)", c->nranks);
    const int64_t n = A->m_local;
    if (n > LU_MAX_N)
        return fail(KLE_ERR_SUP, "PC lu is a dense device factorization: n = %lld exceeds %lld; use -ksp_type cg "
                                 "-pc_type jacobi (K is SPD)", (long long)n, (long long)LU_MAX_N);
    KLE_HIP(hipMalloc(&k->d_lu, sizeof(double) * std::max<int64_t>(n * n, 1)));
    KLE_HIP(hipMalloc(&k->d_ipiv, sizeof(rocblas_int) * std::max<int64_t>(n, 1)));
    KLE_HIP(hipMalloc(&k->d_info, sizeof(rocblas_int)));
    KLE_HIP(hipMemsetAsync(k->d_lu, 0, sizeof(double) * n * n, c->stream));
    if (A->kind == 0) {
        KLE_ARG(A->R == A->C, "PC lu needs square blocks");
        hipLaunchKernelGGL(k_densify_nb, dim3((A->nrows + 127) / 128), dim3(128), 0, c->stream, A->nrows, A->R, A->C,
                           A->vlayout, A->d_rowptr, A->d_rowcnt, A->d_vptr, A->d_bcol, A->d_val, k->d_lu, n);
    } else {
        hipLaunchKernelGGL(k_densify_aij, dim3((A->m_local + 127) / 128), dim3(128), 0, c->stream, A->m_local,
                           A->d_aptr, A->d_acol, A->d_aval, k->d_lu, n);
    }
    KLE_HIP(hipGetLastError());
    if (rocblas_create_handle(&k->blas) != rocblas_status_success) return fail(KLE_ERR_DEVICE, "rocblas_create_handle failed");
    rocblas_set_stream(k->blas, c->stream);
    if (rocsolver_dgetrf(k->blas, (rocblas_int)n, (rocblas_int)n, k->d_lu, (rocblas_int)n, k->d_ipiv, k->d_info) !=
        rocblas_status_success)
        return fail(KLE_ERR_DEVICE, "rocsolver_dgetrf failed");
    rocblas_int info = 0;
    KLE_HIP(hipMemcpyAsync(&info, k->d_info, sizeof(info), hipMemcpyDeviceToHost, c->stream));
    KLE_HIP(hipStreamSynchronize(c->stream));
    if (info > 0) return fail(71, "zero pivot in LU factorization: row %d", (int)info);  // PETSC_ERR_MAT_LU_ZRPVT
    return 0;
}

// preonly / PC lu: one application of the preconditioner (x = M^-1 b)
static int solve_direct(kle_ksp *k, kle_vec *b, kle_vec *x)
{
    kle_ctx *c = k->ctx;
    const int64_t n = b->n_local;
    KLE_HIP(hipMemcpyAsync(x->d, b->d, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
    if (k->pc == "lu") {
        if (rocsolver_dgetrs(k->blas, rocblas_operation_none, (rocblas_int)n, 1, k->d_lu, (rocblas_int)n, k->d_ipiv,
                             x->d, (rocblas_int)n) != rocblas_status_success)
            return fail(KLE_ERR_DEVICE, "rocsolver_dgetrs failed");
    } else if (k->pc == "jacobi") {
        KLE_TRY(kle_vec_pointwise_mult(x, x, k->dinv));
    }
    KLE_HIP(hipStreamSynchronize(c->stream));
    k->its = 1;
    k->reason = 4;  // KSP_CONVERGED_ITS
    return 0;
}

extern "C" {

int kle_ksp_create(kle_ctx *ctx, kle_ksp **out)
{
    KLE_ARG(ctx && out, "null arg");
    kle_ksp *k = new kle_ksp;
    k->ctx = ctx;
    *out = k;
    return 0;
}

int kle_ksp_destroy(kle_ksp *k)
{
    if (!k) return 0;
    free_work(k);
    delete k;
    return 0;
}

int kle_ksp_set_type(kle_ksp *k, const char *t)
{
    KLE_ARG(k && t, "null arg");
    std::string s(t);
    KLE_ARG(s == "cg" || s == "pipecg" || s == "gmres" || s == "preonly", "unknown KSP type '%s' (cg|pipecg|gmres|preonly)",
            t);
    k->type = s;
    k->setup = false;
    return 0;
}

int kle_ksp_set_pc(kle_ksp *k, const char *t) { return kle_ksp_set_pc_type(k, t); }

int kle_ksp_set_pc_type(kle_ksp *k, const char *t)
{
    KLE_ARG(k && t, "null arg");
    std::string s(t);
    KLE_ARG(s == "none" || s == "jacobi" || s == "lu", "unknown PC type '%s' (none|jacobi|lu)", t);
    k->pc = s;
    k->setup = false;
    return 0;
}

int kle_ksp_set_tolerances(kle_ksp *k, double rtol, double atol, double dtol, int maxit)
{
    KLE_ARG(k, "null ksp");
    if (rtol >= 0) k->rtol = rtol;
    if (atol >= 0) k->atol = atol;
    if (dtol >= 0) k->dtol = dtol;
    if (maxit > 0) k->maxit = maxit;
    return 0;
}

int kle_ksp_set_gmres_restart(kle_ksp *k, int restart)
{
    KLE_ARG(k && restart >= 1 && restart <= 200, "bad restart");
    k->restart = restart;
    k->setup = false;
    return 0;
}

int kle_ksp_set_cg_single_reduction(kle_ksp *k, int flag)
{
    KLE_ARG(k, "null ksp");
    k->single_reduction = flag != 0;
    k->setup = false;
    return 0;
}

int kle_ksp_set_fixed_iterations(kle_ksp *k, int n)
{
    KLE_ARG(k && n >= 0, "bad arg");
    k->fixed = n;
    return 0;
}

int kle_ksp_set_operators(kle_ksp *k, kle_mat *A)
{
    KLE_ARG(k && A, "null arg");
    KLE_ARG(A->m_global == A->n_global, "KSP needs a square operator");
    k->A = A;
    k->setup = false;
    return 0;
}

int kle_ksp_set_up(kle_ksp *k)
{
    KLE_ARG(k && k->A, "operators not set");
    if (k->setup) return 0;
    free_work(k);
    if (k->pc == "lu") {
        KLE_TRY(make_vec_like_cols(k, &k->p));
        KLE_TRY(make_vec_like_cols(k, &k->q));
        KLE_TRY(lu_factor(k));
        k->setup = true;
        return 0;
    }
    KLE_TRY(make_vec_like_cols(k, &k->r));
    KLE_TRY(make_vec_like_cols(k, &k->p));
    KLE_TRY(make_vec_like_cols(k, &k->q));
    if ((k->type == "cg" && k->single_reduction) || k->type == "pipecg") {
        KLE_TRY(make_vec_like_cols(k, &k->u));
        KLE_TRY(make_vec_like_cols(k, &k->w));
        KLE_TRY(make_vec_like_cols(k, &k->s));
    }
    if (k->type == "pipecg") {
        KLE_TRY(make_vec_like_cols(k, &k->m));
        KLE_TRY(make_vec_like_cols(k, &k->nv));
        KLE_TRY(make_vec_like_cols(k, &k->z));
    }
    if (k->pc == "jacobi") {
        KLE_TRY(make_vec_like_cols(k, &k->dinv));
        KLE_TRY(kle_mat_get_diagonal(k->A, k->q));
        hipLaunchKernelGGL(k_invert_diag, dim3((k->A->m_local + 255) / 256), dim3(256), 0, k->ctx->stream,
                           k->A->m_local, k->q->d, k->dinv->d);
        KLE_HIP(hipGetLastError());
    }
    if (k->type == "gmres") {
        k->V.resize(k->restart + 1);
        for (auto &v : k->V) KLE_TRY(make_vec_like_cols(k, &v));
        std::vector<double *> ptrs(k->V.size());
        for (size_t i = 0; i < ptrs.size(); ++i) ptrs[i] = k->V[i]->d;
        KLE_HIP(hipMalloc(&k->d_Vptr, sizeof(double *) * ptrs.size()));
        KLE_HIP(hipMalloc(&k->d_h, sizeof(double) * (k->restart + 2)));
        KLE_HIP(hipMalloc(&k->d_gpart, sizeof(double) * (k->restart + 2) * RED_BLOCKS));
        KLE_TRY(h2d(k->d_Vptr, ptrs.data(), sizeof(double *) * ptrs.size()));
    }
    KLE_HIP(hipStreamSynchronize(k->ctx->stream));
    k->setup = true;
    return 0;
}

// CG and pipelined CG stop on their recursive residual, which drifts from
// the true one: the pipelined recurrence ends at 1.1-1.3e-10 true residual at
// rtol 1e-10 on 2-8 ranks.  When the true residual b - A x (in k->q after
// true_residual) misses rtol, a correction solve A e = r to 0.5 rtol ||b||
// (same method, zero start) and x += e bring it under; at most k->max_corr
// such passes (default 2: kle_set_tuning("ksp_refine") / KLE_KSP_REFINE for
// new KSPs, kle_ksp_set_corrections per KSP).  0 is PETSc's KSPCG/KSPPIPECG
// exactly: stop on the recursive residual whatever the true one.  The main
// solve's converged reason, iteration count and residual norm stand as PETSc
// reports them (a correction that runs out of iterations does not turn a
// converged solve into DIVERGED_ITS); the corrections are reported apart:
// kle_ksp_get_correction_iterations / _reason.  Each correction has the
// KSP's max_it of its own.
static int refine(kle_ksp *k, kle_vec *b, kle_vec *x)
{
    k->corr_its = 0;
    k->corr_reason = 0;
    if (k->max_corr <= 0 || (k->type != "pipecg" && k->type != "cg") || k->pc == "lu") return 0;
    kle_ctx *c = k->ctx;
    const int reason0 = k->reason, its_main = k->its;
    const double rnorm0 = k->rnorm;
    for (int pass = 0; pass < k->max_corr; ++pass) {
        if (reason0 <= 0 || k->corr_reason < 0 || (!(k->true_rel > k->rtol) && !g_tune.ksp_corr_fault)) return 0;
        kle_vec *rv = nullptr, *e = nullptr;
        int rc = vec_alloc(c, b->n_local, b->n_global, b->lo, 0, 0, &rv);
        if (!rc) rc = vec_alloc(c, x->n_local, x->n_global, x->lo, 0, 0, &e);
        const double rtol0 = k->rtol;
        if (!rc) rc = kle_vec_copy(k->q, rv);
        if (!rc) {
            k->rtol = 0.5 * rtol0 / k->true_rel;  // (relative to ||r|| = true_rel ||b||)
            rc = k->type == "pipecg" ? solve_pipecg(k, rv, e, false)
                 : k->single_reduction ? solve_cg_single(k, rv, e, false)
                                       : solve_cg(k, rv, e);
            k->rtol = rtol0;
            k->corr_its += k->its;
            k->corr_reason = k->reason;
            k->its = its_main;
            k->reason = reason0;
            k->rnorm = rnorm0;
        }
        if (!rc && g_tune.ksp_corr_fault) {  // (test hook: a correction that ends in NaN)
            rc = kle_vec_set(e, __builtin_nan(""));
            k->corr_reason = KLE_DIVERGED_NANORINF;
        }
        bool kept = false;  // (x left as it was: its true residual in k->q still holds)
        if (!rc && k->corr_reason > 0) {
            rc = kle_vec_axpy(x, 1.0, e);
        } else if (!rc) {
            // the correction broke down, met NaN/Inf or ran out of iterations:
            // x + e only if e is finite and the true residual drops, else x
            // stays as it was -- rv (the correction's right-hand
            // side, spent) keeps x meanwhile
            double en = 0.0;
            rc = kle_vec_norm2(e, &en);
            kept = true;
            if (!rc && std::isfinite(en) && en > 0.0) {
                const double rel0 = k->true_rel;
                rc = kle_vec_copy(x, rv);
                if (!rc) rc = kle_vec_axpy(x, 1.0, e);
                if (!rc) rc = true_residual(k, b, x);
                if (!rc && !(k->true_rel < rel0)) {
                    rc = kle_vec_copy(rv, x);
                    if (!rc) rc = true_residual(k, b, x);
                }
            }
        }
        for (kle_vec *v : {rv, e})
            if (v) {
                (void)hipStreamSynchronize(c->stream);
                (void)hipFree(v->base);
                delete v;
            }
        if (rc) return rc;
        if (!kept) KLE_TRY(true_residual(k, b, x));
    }
    return 0;
}

int kle_ksp_solve(kle_ksp *k, kle_vec *b, kle_vec *x)
{
    KLE_ARG(k && b && x, "null arg");
    KLE_TRY(kle_ksp_set_up(k));
    KLE_ARG(b->n_local == k->A->m_local && x->n_local == k->A->n_local, "b/x sizes do not match the operator");
    k->true_rel = -1;
    // an exact preconditioner makes any Krylov method converge in one step:
    // PC lu is applied directly whatever the KSP type (gmres + lu, kle_solver.py:57-61)
    k->last_b = k->last_x = nullptr;
    if (k->pc == "lu" || k->type == "preonly") KLE_TRY(solve_direct(k, b, x));
    else if (k->type == "pipecg") KLE_TRY(solve_pipecg(k, b, x, false));
    else if (k->type == "cg" && k->single_reduction) KLE_TRY(solve_cg_single(k, b, x, false));
    else if (k->type == "cg") KLE_TRY(solve_cg(k, b, x));
    else KLE_TRY(solve_gmres(k, b, x));
    if (!k->fixed) {
        KLE_TRY(true_residual(k, b, x));
        KLE_TRY(refine(k, b, x));
    } else {
        k->last_b = b;
        k->last_x = x;
    }
    return 0;
}

int kle_ksp_continue(kle_ksp *k, kle_vec *b, kle_vec *x, int n)
{
    KLE_ARG(k && b && x && n >= 1, "bad arg");
    KLE_ARG(k->setup && k->fixed && k->last_b == b && k->last_x == x,
            "continue needs a preceding fixed-iteration solve with the same b and x");
    KLE_ARG(k->pc != "lu" && (k->type == "pipecg" || (k->type == "cg" && k->single_reduction)),
            "continue: single-reduction or pipelined CG only");
    const int keep = k->fixed;
    k->fixed = n;
    const int rc = k->type == "pipecg" ? solve_pipecg(k, b, x, true) : solve_cg_single(k, b, x, true);
    k->fixed = keep;
    return rc;
}

int kle_ksp_get_product_kernel(const kle_ksp *k, char *buf, int buflen)
{
    KLE_ARG(k && buf && buflen > 0, "bad arg");
    snprintf(buf, buflen, "%s", k->prod_kernel.c_str());
    return 0;
}

int kle_ksp_get_product_bytes(const kle_ksp *k, double *bytes)
{
    KLE_ARG(k && bytes, "null arg");
    *bytes = k->prod_bytes;
    return 0;
}

int kle_ksp_get_iteration_number(const kle_ksp *k, int *its)
{
    KLE_ARG(k && its, "null arg");
    *its = k->its;
    return 0;
}

int kle_ksp_get_residual_norm(const kle_ksp *k, double *rn)
{
    KLE_ARG(k && rn, "null arg");
    *rn = k->rnorm;
    return 0;
}

int kle_ksp_get_converged_reason(const kle_ksp *k, int *reason)
{
    KLE_ARG(k && reason, "null arg");
    *reason = k->reason;
    return 0;
}

int kle_ksp_set_corrections(kle_ksp *k, int max_corrections)
{
    KLE_ARG(k && max_corrections >= 0 && max_corrections <= 8, "corrections: 0 .. 8");
    k->max_corr = max_corrections;
    return 0;
}

int kle_ksp_get_correction_iterations(const kle_ksp *k, int *its)
{
    KLE_ARG(k && its, "null arg");
    *its = k->corr_its;
    return 0;
}

int kle_ksp_get_correction_reason(const kle_ksp *k, int *reason)
{
    KLE_ARG(k && reason, "null arg");
    *reason = k->corr_reason;
    return 0;
}

int kle_ksp_get_true_relative_residual(const kle_ksp *k, double *rel)
{
    KLE_ARG(k && rel, "null arg");
    *rel = k->true_rel;
    return 0;
}

}  // extern "C"
