// kmpc_solve.hip — batched MPC solve on gfx950 (replaces solve_mpc_log_utility, mpc.py:27-117).
//
// One workgroup per window (problem), one asset per thread (blockDim = 64 * ceil(N / 64)); all
// arithmetic in float64 (the reference's own solver, SCS, runs in float64; the f32 predicted
// returns are widened on load exactly as cvxpy does).
//
// Algorithm: Mehrotra predictor-corrector primal-dual interior point on the epigraph form of the
// reference program (derivation and CPU restatement: oracle/kmpc_oracle.c):
//   min  -(1/sig) sum_t log(1 + m_t.w_t) + (c/sig) sum_t 1's_t        m = expm1(yhat)
//   s.t. w >= 0 (no short), s_t -+ (w_t - w_{t-1}) >= 0, tau - 1's_t >= 0, 1'w_t = 1.
// Each Newton system is reduced exactly to
//   (Q + Z_U Z_U^T) dw + A^T dnu = r,  A dw = r2,   Q = diag(W1) + D^T E D  (per-asset tridiagonal in t)
// with Z = [a_t | sqrt(rho_t) D^T e_t | 1_t] (K = 3H columns). Per asset (= per thread, registers):
// the LDL^T of Q (cancellation-free pivots), Q^{-1} applied by two O(H) sweeps, and the explicit
// H x H inverse Q^{-1} for the Schur (Woodbury) matrix G = I' + Z^T Q^{-1} Z, whose K(K+1)/2 entries
// are accumulated in register panels of PW and summed across the block by a butterfly
// reduce-scatter (__shfl_xor) + LDS. Wave 0 factors G (Cholesky, one row per lane) and solves.
//
// Per-problem status / fallback follow mpc.py:107-117: non-optimal -> W = tile(w_prev), obj = NaN.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kmpc_internal.h"

namespace kmpc {

constexpr int WAVE = 64;
constexpr int MAX_WAVES = KMPC_MAX_N / WAVE;   // 16
constexpr int RED_W = 64;                      // slots per wave in the reduction buffer
constexpr int PW = 32;                         // Schur entries per Gram panel
#ifdef KMPC_STATS
__device__ unsigned long long g_stats[2];   // dev builds only: refinement steps, Newton solves
#endif
#ifndef KMPC_REFINE_RTOL
#define KMPC_REFINE_RTOL 1e-7
#endif
constexpr double REFINE_RTOL = KMPC_REFINE_RTOL;           // refinement stops at ||r|| <= REFINE_RTOL ||b|| (oracle: same)

struct SolveArgs {
    int B, N, H;
    double c, tau;
    int allow_short, max_iter, return_full, n_refine;
    double tol;
    const float* yhat;
    const double* wp;
    double* wout;
    int* status;
    double* obj;
    int* iters;
    double* trace;   // debug: per-iteration (mu, rd, pr, step) of problem 0, or null
};

// ---- reductions ---------------------------------------------------------------------------------

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
    return v;
}

// Wave reduce-scatter of M = 2^k values (k <= 6): afterwards lane l holds in v[0] the wave total
// of slot `slot` (returned); the 64/M lanes that agree in their high bits share a slot. Each
// butterfly step sends the half it does not keep: ~M shuffles instead of 6M.
template <int M>
__device__ __forceinline__ int wave_reduce_scatter(double (&v)[M]) {
    const int lane = threadIdx.x & (WAVE - 1);
    int slot = 0;
    int n = M;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        if (n > 1) {
            const int h = n >> 1;
            const bool up = (lane & d) != 0;
#pragma unroll
            for (int j = 0; j < (M > 1 ? M / 2 : 1); ++j) {
                if (j < h) {
                    const double lo = v[j], hi = v[j + h];
                    const double send = up ? lo : hi;
                    const double keep = up ? hi : lo;
                    v[j] = keep + __shfl_xor(send, d, WAVE);
                }
            }
            slot += up ? h : 0;
            n = h;
        } else {
            v[0] += __shfl_xor(v[0], d, WAVE);
        }
    }
    return slot;
}

// Block sum of M (power of two, <= 64) values; every thread receives all totals.
template <int M>
__device__ __forceinline__ void block_sum(double (&v)[M], double* red, int nw) {
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    double tmp[M];
#pragma unroll
    for (int j = 0; j < M; ++j) tmp[j] = v[j];
    const int slot = wave_reduce_scatter<M>(tmp);
    if ((lane & ((WAVE / M) - 1)) == 0) red[wv * RED_W + slot] = tmp[0];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < M; ++j) {
        double s = 0.0;
        for (int q = 0; q < nw; ++q) s += red[q * RED_W + j];
        v[j] = s;
    }
    __syncthreads();
}

// Block sum of M (power of two, <= 64) values; thread q < M writes the total of slot q to out[q].
template <int M>
__device__ __forceinline__ void block_sum_lds(double (&v)[M], double* red, double* out, int nw,
                                              int nout = M) {
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    const int slot = wave_reduce_scatter<M>(v);
    if ((lane & ((WAVE / M) - 1)) == 0) red[wv * RED_W + slot] = v[0];
    __syncthreads();
    if ((int)threadIdx.x < nout) {
        double s = 0.0;
        for (int q = 0; q < nw; ++q) s += red[q * RED_W + threadIdx.x];
        out[threadIdx.x] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ double block_sum1(double v, double* red, int nw) {
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    v = wave_sum(v);
    if (lane == 0) red[wv * RED_W] = v;
    __syncthreads();
    double s = 0.0;
    for (int q = 0; q < nw; ++q) s += red[q * RED_W];
    __syncthreads();
    return s;
}
__device__ __forceinline__ double block_max1(double v, double* red, int nw) {
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    v = wave_max(v);
    if (lane == 0) red[wv * RED_W] = v;
    __syncthreads();
    double s = red[0];
    for (int q = 1; q < nw; ++q) s = fmax(s, red[q * RED_W]);
    __syncthreads();
    return s;
}
__device__ __forceinline__ double block_min1(double v, double* red, int nw) {
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    v = wave_min(v);
    if (lane == 0) red[wv * RED_W] = v;
    __syncthreads();
    double s = red[0];
    for (int q = 1; q < nw; ++q) s = fmin(s, red[q * RED_W]);
    __syncthreads();
    return s;
}

__device__ __forceinline__ double to_bound(double v, double dv, double a) {
    return (dv < 0.0) ? fmin(a, -v / dv) : a;
}

__host__ __device__ constexpr int pow2_at_least(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}
__host__ __device__ constexpr int min_i(int a, int b) { return a < b ? a : b; }

// ---- compile-time layout of the Schur system ----------------------------------------------------
// Column j of Z: type = j / HM (0: a_t utility, 1: v_t turnover cap, 2: 1_t budget), t = j % HM.
// Upper-triangle entries (j <= l) are ordered by c = max(t_j, t_l) (the later period), so a panel
// of PW consecutive entries touches only Q^{-1} columns c_lo-1 .. c_hi.
template <int HM>
struct Tri {
    static constexpr int KM = 3 * HM;
    static constexpr int NE = KM * (KM + 1) / 2;
    static constexpr int NP = (NE + PW - 1) / PW;
    int row[NP * PW];
    int col[NP * PW];
    int clo[NP];
    int chi[NP];
    constexpr Tri() : row(), col(), clo(), chi() {
        int q = 0;
        for (int c = 0; c < HM; ++c)
            for (int j = 0; j < KM; ++j)
                for (int l = j; l < KM; ++l) {
                    const int tj = j % HM, tl = l % HM;
                    if ((tj > tl ? tj : tl) == c) { row[q] = j; col[q] = l; ++q; }
                }
        for (; q < NP * PW; ++q) { row[q] = -1; col[q] = -1; }
        for (int p = 0; p < NP; ++p) {
            int lo = HM, hi = -1;
            for (int e = p * PW; e < p * PW + PW; ++e) {
                if (row[e] < 0) continue;
                const int tj = row[e] % HM, tl = col[e] % HM;
                const int c = tj > tl ? tj : tl;
                lo = c < lo ? c : lo;
                hi = c > hi ? c : hi;
            }
            clo[p] = lo;
            chi[p] = hi;
        }
    }
};

// ---- the solver ---------------------------------------------------------------------------------

template <int HM>
struct Shared {
    static constexpr int KM = 3 * HM;
    double G[KM * KM];          // Schur matrix, then its Cholesky factor (lower, row-major)
    double bs[KM];              // Schur right-hand side, then solution q
    double panel[PW];
    double red[MAX_WAVES * RED_W];
    double den[HM], rp[HM], rg4[HM], z4[HM], l4[HM], nu[HM];
    double rho[HM], sr[HM];
    double rc4[HM], b5[HM], b6[HM], dnu[HM], dz4[HM], dl4[HM];
    double sv_nu[HM], sv_b5[HM], sv_b6[HM];
    double t_adw[HM], t_sds[HM], t_sdw[HM];
    int flag;
};

template <int HM>
struct Thread {
    int H, N, i;
    bool act, hw, hs, ht;
    double c, tau, sig, rsig, wpi;
    // state
    double w[HM], s[HM], l1[HM], l2[HM], l3[HM], m[HM];
    // factorization of the current iterate
    double P[HM], bma[HM], Dd[HM], Lr[HM];
    // complementarity targets rc = z*l (- sigma mu + dz_aff dl_aff)
    double rc1[HM], rc2[HM], rc3[HM];
    // direction
    double dw[HM], ds[HM];

    __device__ __forceinline__ double wprev(int t) const { return t ? w[t - 1] : wpi; }
    __device__ __forceinline__ double alpha(int t, const Shared<HM>& sh) const {   // a_t (utility)
        return m[t] / (sh.den[t] * rsig);
    }
    __device__ __forceinline__ double eps(int t, const Shared<HM>& sh) const {     // sqrt(rho) e
        return sh.sr[t] * bma[t] * P[t];
    }

    // x = Q^{-1} r  (LDL^T: y_t = r_t + Lr_t y_{t-1};  x_t = y_t / Dd_t + Lr_{t+1} x_{t+1})
    __device__ __forceinline__ void qsolve(const double (&r)[HM], double (&x)[HM]) const {
        double y = 0.0;
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            if (t < H) { y = r[t] + Lr[t] * y; x[t] = y; } else { x[t] = 0.0; }
        }
        double nxt = 0.0;
#pragma unroll
        for (int t = HM - 1; t >= 0; --t) {
            if (t < H) {
                const double v = x[t] / Dd[t] + ((t + 1 < HM && t + 1 < H) ? Lr[t + 1] * nxt : 0.0);
                x[t] = v;
                nxt = v;
            }
        }
    }
};

// per-period block sums of an [HM] register array -> out (all threads)
template <int HM>
__device__ __forceinline__ void period_sums(const double (&x)[HM], double (&out)[HM], double* red,
                                            int nw) {
    constexpr int M = pow2_at_least(HM);
    double v[M];
#pragma unroll
    for (int t = 0; t < M; ++t) v[t] = t < HM ? x[t] : 0.0;
    block_sum<M>(v, red, nw);
#pragma unroll
    for (int t = 0; t < HM; ++t) out[t] = v[t];
}

// (diag(alpha+beta) + gamma 1 1')^{-1} x per period = P (x - rho 1'P x)
template <int HM>
__device__ __forceinline__ void sinv(Thread<HM>& T, Shared<HM>& sh, const double (&x)[HM],
                                     double (&out)[HM], int nw) {
    double px[HM], acc[HM];
#pragma unroll
    for (int t = 0; t < HM; ++t) px[t] = (T.act && t < T.H) ? T.P[t] * x[t] : 0.0;
    period_sums<HM>(px, acc, sh.red, nw);
#pragma unroll
    for (int t = 0; t < HM; ++t) out[t] = T.P[t] * (x[t] - sh.rho[t] * acc[t]);
}

// Solve the Newton system (oracle/kmpc_oracle.c:lsolve) for rhs (b0, b1, [bc = -rc], sh.b5, sh.b6)
//   -> T.dw, T.ds, sh.dnu.
template <int HM>
__device__ __forceinline__ void lsolve(Thread<HM>& T, Shared<HM>& sh, const double (&b0)[HM],
                                       const double (&b1)[HM], bool with_c, int nw) {
    constexpr int KM = 3 * HM;
    const int H = T.H;
    double rhsw[HM], rhss[HM];
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        double p1 = 0.0, p2 = 0.0, p3 = 0.0, pn = 0.0;
        rhsw[t] = rhss[t] = 0.0;
        if (T.act && t < H) {
            const double d = T.w[t] - T.wprev(t);
            if (with_c) {
                if (T.hw) p1 = -T.rc1[t] / T.w[t];
                if (T.hs) {
                    p2 = -T.rc2[t] / (T.s[t] - d);
                    p3 = -T.rc3[t] / (T.s[t] + d);
                    if (t + 1 < HM && t + 1 < H) {
                        const double dn = T.w[t + 1] - T.w[t];
                        pn = -T.rc3[t + 1] / (T.s[t + 1] + dn) + T.rc2[t + 1] / (T.s[t + 1] - dn);
                    }
                }
            }
            rhsw[t] = b0[t] + p1 + (p3 - p2) - pn;
            rhss[t] = T.hs ? b1[t] + p2 + p3 - (T.ht ? sh.b5[t] / sh.z4[t] : 0.0) : 0.0;
        }
    }
    if (T.hs) {
        double g[HM];
        sinv<HM>(T, sh, rhss, g, nw);
#pragma unroll
        for (int t = 0; t < HM; ++t) g[t] *= T.bma[t];
#pragma unroll
        for (int t = 0; t < HM; ++t) rhsw[t] -= g[t] - ((t + 1 < HM && t + 1 < H) ? g[t + 1] : 0.0);
    }
    // x = Q^{-1} rhsw ;  bs = Z^T x  (block-summed over assets, in chunks of M slots)
    double x[HM];
    T.qsolve(rhsw, x);
    {
        constexpr int M = min_i(pow2_at_least(KM), 32);
#pragma unroll
        for (int c0 = 0; c0 < KM; c0 += M) {
            double v[M];
#pragma unroll
            for (int q = 0; q < M; ++q) {
                const int j = c0 + q;
                double val = 0.0;
                if (j < KM && T.act) {
                    const int ty = j / HM, t = j % HM;
                    if (t < H) {
                        if (ty == 0) val = T.alpha(t, sh) * x[t];
                        else if (ty == 1) val = T.ht ? T.eps(t, sh) * (x[t] - (t ? x[t - 1] : 0.0)) : 0.0;
                        else val = x[t];
                    }
                }
                v[q] = val;
            }
            block_sum_lds<M>(v, sh.red, sh.bs + c0, nw, min_i(M, KM - c0));
        }
    }
    if (threadIdx.x < WAVE) {
        // wave 0: q = G^{-1} (bs - [0; 0; b6]) by forward / back substitution; lane r owns row r
        const int lane = threadIdx.x;
        double rhs = 0.0;
        if (lane < KM) {
            rhs = sh.bs[lane];
            const int t = lane - 2 * HM;
            if (t >= 0 && t < H) rhs -= sh.b6[t];
        }
        for (int j = 0; j < KM; ++j) {
            const double yj = __shfl(rhs, j, WAVE) / sh.G[j * KM + j];
            if (lane == j) rhs = yj;
            if (lane > j && lane < KM) rhs -= sh.G[lane * KM + j] * yj;
        }
        for (int j = KM - 1; j >= 0; --j) {
            const double qj = __shfl(rhs, j, WAVE) / sh.G[j * KM + j];
            if (lane == j) rhs = qj;
            if (lane < j) rhs -= sh.G[j * KM + lane] * qj;
        }
        const double qn = __shfl(rhs, (2 * HM + lane) & (WAVE - 1), WAVE);
        if (lane < KM) sh.bs[lane] = rhs;
        if (lane < HM) sh.dnu[lane] = (lane < H) ? qn : 0.0;
    }
    __syncthreads();
    // dw = x - Q^{-1} (Z q)
    {
        double zq[HM], y[HM];
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            zq[t] = 0.0;
            if (T.act && t < H) {
                double v = T.alpha(t, sh) * sh.bs[t] + sh.bs[2 * HM + t];
                if (T.ht) {
                    v += T.eps(t, sh) * sh.bs[HM + t];
                    if (t + 1 < HM && t + 1 < H) v -= T.eps(t + 1, sh) * sh.bs[HM + t + 1];
                }
                zq[t] = v;
            }
        }
        T.qsolve(zq, y);
#pragma unroll
        for (int t = 0; t < HM; ++t) T.dw[t] = (T.act && t < H) ? x[t] - y[t] : 0.0;
    }
    if (T.hs) {
        double tmp[HM];
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            const double dd = T.dw[t] - (t ? T.dw[t - 1] : 0.0);
            tmp[t] = (T.act && t < H) ? rhss[t] - T.bma[t] * dd : 0.0;
        }
        sinv<HM>(T, sh, tmp, T.ds, nw);
#pragma unroll
        for (int t = 0; t < HM; ++t) if (!T.act || t >= H) T.ds[t] = 0.0;
    } else {
#pragma unroll
        for (int t = 0; t < HM; ++t) T.ds[t] = 0.0;
    }
}

// Multipliers of the current direction (complementarity rows, bc = -rc).
template <int HM>
__device__ __forceinline__ void dual_dirs(const Thread<HM>& T, int t, double& dl1, double& dl2,
                                          double& dl3) {
    const double d = T.w[t] - T.wprev(t);
    const double dd = T.dw[t] - (t ? T.dw[t - 1] : 0.0);
    dl1 = T.hw ? (-T.rc1[t] - T.l1[t] * T.dw[t]) / T.w[t] : 0.0;
    if (T.hs) {
        dl2 = (-T.rc2[t] - T.l2[t] * (T.ds[t] - dd)) / (T.s[t] - d);
        dl3 = (-T.rc3[t] - T.l3[t] * (T.ds[t] + dd)) / (T.s[t] + d);
    } else {
        dl2 = dl3 = 0.0;
    }
}

// Dual residuals of the current iterate (rows 1-2) at period t.
template <int HM>
__device__ __forceinline__ void dual_residual(const Thread<HM>& T, const Shared<HM>& sh, int t,
                                              double& rdw, double& rds) {
    const double eta = T.l3[t] - T.l2[t];
    const double etan = (t + 1 < HM && t + 1 < T.H) ? T.l3[t + 1] - T.l2[t + 1] : 0.0;
    rdw = -T.m[t] / (T.sig * sh.den[t]) - (T.l1[t] + eta - etan) + sh.nu[t];
    rds = T.hs ? T.c - (T.l2[t] + T.l3[t] - sh.l4[t]) : 0.0;
}

// Full Newton direction for the current rc targets with n_refine steps of iterative refinement
// against the unreduced system. On exit: T.dw, T.ds, sh.dnu, sh.dz4, sh.dl4.
template <int HM>
__device__ __forceinline__ void newton(Thread<HM>& T, Shared<HM>& sh, int nw, int n_refine) {
    const int H = T.H;
    if (threadIdx.x < HM) {
        const int t = threadIdx.x;
        sh.b5[t] = (T.ht && t < H) ? -sh.rc4[t] - sh.l4[t] * sh.rg4[t] : 0.0;
        sh.b6[t] = (t < H) ? -sh.rp[t] : 0.0;
    }
    __syncthreads();
    double bn = 0.0;   // ||b||_inf of this thread's rows
    {
        double b0[HM], b1[HM];
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            b0[t] = b1[t] = 0.0;
            if (T.act && t < H) {
                double rdw, rds;
                dual_residual<HM>(T, sh, t, rdw, rds);
                b0[t] = -rdw;
                b1[t] = -rds;
                bn = fmax(bn, fmax(fmax(fabs(rdw), fabs(rds)),
                                   fmax(fabs(T.rc1[t]), fmax(fabs(T.rc2[t]), fabs(T.rc3[t])))));
            }
            if (threadIdx.x == 0 && t < H) bn = fmax(bn, fmax(fabs(sh.b5[t]), fabs(sh.b6[t])));
        }
        lsolve<HM>(T, sh, b0, b1, true, nw);
    }
    __syncthreads();
    if (n_refine > 0) bn = block_max1(bn, sh.red, nw);
    // adaptive refinement: stop once ||r||_inf <= REFINE_RTOL ||b||_inf (block-uniform decision)
    int r = 0;
    for (; r < n_refine; ++r) {
        // residual of rows (1), (2), (6), (7); rows (3)-(5) hold by construction
        {
            double adw[HM], sds[HM], sdw[HM];
#pragma unroll
            for (int t = 0; t < HM; ++t) {
                const bool on = T.act && t < H;
                adw[t] = on ? T.alpha(t, sh) * T.dw[t] : 0.0;
                sds[t] = on ? T.ds[t] : 0.0;
                sdw[t] = on ? T.dw[t] : 0.0;
            }
            period_sums<HM>(adw, adw, sh.red, nw);
            period_sums<HM>(sds, sds, sh.red, nw);
            period_sums<HM>(sdw, sdw, sh.red, nw);
            if (threadIdx.x == 0) {
#pragma unroll
                for (int t = 0; t < HM; ++t) { sh.t_adw[t] = adw[t]; sh.t_sds[t] = sds[t]; sh.t_sdw[t] = sdw[t]; }
            }
            __syncthreads();
        }
        double r0[HM], r1[HM], sw[HM], ss[HM];
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            r0[t] = r1[t] = 0.0;
            if (T.act && t < H) {
                double dl1, dl2, dl3, n1 = 0.0, n2 = 0.0, n3 = 0.0, rdw, rds;
                dual_dirs<HM>(T, t, dl1, dl2, dl3);
                if (t + 1 < HM && t + 1 < H) dual_dirs<HM>(T, t + 1, n1, n2, n3);
                dual_residual<HM>(T, sh, t, rdw, rds);
                const double dl4 = T.ht ? (sh.b5[t] + sh.l4[t] * sh.t_sds[t]) / sh.z4[t] : 0.0;
                r0[t] = -rdw - (T.alpha(t, sh) * sh.t_adw[t] - (dl1 + (dl3 - dl2) - (n3 - n2)) + sh.dnu[t]);
                r1[t] = T.hs ? -rds + (dl2 + dl3 - dl4) : 0.0;
            }
            sw[t] = T.dw[t];
            ss[t] = T.ds[t];
        }
        {
            double rn = 0.0;
#pragma unroll
            for (int t = 0; t < HM; ++t) {
                rn = fmax(rn, fmax(fabs(r0[t]), fabs(r1[t])));
                if (threadIdx.x == 0 && t < H) rn = fmax(rn, fabs(sh.b6[t] - sh.t_sdw[t]));
            }
            rn = block_max1(rn, sh.red, nw);
            if (rn <= REFINE_RTOL * bn) break;
        }
        if (threadIdx.x == 0) {
#pragma unroll
            for (int t = 0; t < HM; ++t) {
                const double dl4 = (T.ht && t < H) ? (sh.b5[t] + sh.l4[t] * sh.t_sds[t]) / sh.z4[t] : 0.0;
                sh.sv_nu[t] = sh.dnu[t];
                sh.sv_b5[t] = sh.b5[t];
                sh.sv_b6[t] = sh.b6[t];
                sh.b5[t] = (T.ht && t < H) ? sh.b5[t] - (-sh.l4[t] * sh.t_sds[t] + sh.z4[t] * dl4) : 0.0;
                sh.b6[t] = (t < H) ? sh.b6[t] - sh.t_sdw[t] : 0.0;
            }
        }
        __syncthreads();
        lsolve<HM>(T, sh, r0, r1, false, nw);
        __syncthreads();
#pragma unroll
        for (int t = 0; t < HM; ++t) { T.dw[t] += sw[t]; T.ds[t] += ss[t]; }
        if (threadIdx.x < HM) {
            const int t = threadIdx.x;
            sh.dnu[t] += sh.sv_nu[t];
            sh.b5[t] = sh.sv_b5[t];
            sh.b6[t] = sh.sv_b6[t];
        }
        __syncthreads();
    }
#ifdef KMPC_STATS
    if (threadIdx.x == 0) { atomicAdd(&g_stats[0], (unsigned long long)r); atomicAdd(&g_stats[1], 1ull); }
#else
    (void)r;
#endif
    // dz4 / dl4 of the final direction
    double sds[HM];
#pragma unroll
    for (int t = 0; t < HM; ++t) sds[t] = (T.act && t < H) ? T.ds[t] : 0.0;
    period_sums<HM>(sds, sds, sh.red, nw);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            const bool on = T.ht && t < H;
            sh.dz4[t] = on ? -sds[t] + sh.rg4[t] : 0.0;
            sh.dl4[t] = on ? (sh.b5[t] + sh.l4[t] * sds[t]) / sh.z4[t] : 0.0;
        }
    }
    __syncthreads();
}

// Largest step for the current direction (before the caller's fraction-to-boundary).
template <int HM>
__device__ __forceinline__ double max_step(const Thread<HM>& T, Shared<HM>& sh, int nw) {
    const int H = T.H;
    double a = 1e300, mdw[HM];
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        mdw[t] = 0.0;
        if (T.act && t < H) {
            double dl1, dl2, dl3;
            dual_dirs<HM>(T, t, dl1, dl2, dl3);
            const double d = T.w[t] - T.wprev(t);
            const double dd = T.dw[t] - (t ? T.dw[t - 1] : 0.0);
            if (T.hw) { a = to_bound(T.w[t], T.dw[t], a); a = to_bound(T.l1[t], dl1, a); }
            if (T.hs) {
                a = to_bound(T.s[t] - d, T.ds[t] - dd, a);
                a = to_bound(T.s[t] + d, T.ds[t] + dd, a);
                a = to_bound(T.l2[t], dl2, a);
                a = to_bound(T.l3[t], dl3, a);
            }
            mdw[t] = T.m[t] * T.dw[t];
        }
    }
    period_sums<HM>(mdw, mdw, sh.red, nw);
    a = block_min1(a, sh.red, nw);
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        if (t < H) {
            a = to_bound(sh.den[t], mdw[t], a);
            if (T.ht) { a = to_bound(sh.z4[t], sh.dz4[t], a); a = to_bound(sh.l4[t], sh.dl4[t], a); }
        }
    }
    return a;
}

template <int HM>
__device__ __forceinline__ double complementarity(const Thread<HM>& T, Shared<HM>& sh, double a,
                                                  int nw) {
    const int H = T.H;
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        if (T.act && t < H) {
            double dl1, dl2, dl3;
            dual_dirs<HM>(T, t, dl1, dl2, dl3);
            const double d = T.w[t] - T.wprev(t);
            const double dd = T.dw[t] - (t ? T.dw[t - 1] : 0.0);
            if (T.hw) acc += (T.w[t] + a * T.dw[t]) * (T.l1[t] + a * dl1);
            if (T.hs) {
                acc += (T.s[t] - d + a * (T.ds[t] - dd)) * (T.l2[t] + a * dl2);
                acc += (T.s[t] + d + a * (T.ds[t] + dd)) * (T.l3[t] + a * dl3);
            }
        }
    }
    double r = block_sum1(acc, sh.red, nw);
    if (T.ht)
        for (int t = 0; t < H; ++t) r += (sh.z4[t] + a * sh.dz4[t]) * (sh.l4[t] + a * sh.dl4[t]);
    return r;
}

// One panel of the Gram: entries P*PW .. P*PW+PW-1 (ordered by c = max(tj, tl)). For columns j, l:
//   G_jl = sum_i c_j c_l (Qi[tj][tl] - [vj] Qi[tj-1][tl] - [vl] Qi[tj][tl-1] + [vj vl] Qi[tj-1][tl-1])
// with c = alpha_t (a), eps_t (v), 1 (budget). Q^{-1} columns are generated from the LDL^T:
//   Qi[c][c] = dq_c,  Qi[r][c] = Lr_{r+1} Qi[r+1][c]  (r < c).
template <int HM, int P>
__device__ __forceinline__ void gram_panel(const Thread<HM>& T, Shared<HM>& sh, const double (&dq)[HM],
                                           int nw) {
    constexpr int KM = 3 * HM;
    constexpr Tri<HM> tab{};
    constexpr int C0 = tab.clo[P] > 0 ? tab.clo[P] - 1 : 0;
    constexpr int C1 = tab.chi[P];
    // columns C0..C1 of Q^{-1} (rows 0..c), column k stored at qc[k - C0]
    double qc[C1 - C0 + 1][HM];
#pragma unroll
    for (int k = C0; k <= C1; ++k) {
        qc[k - C0][k] = dq[k];
#pragma unroll
        for (int r = k - 1; r >= 0; --r) qc[k - C0][r] = T.Lr[r + 1] * qc[k - C0][r + 1];
    }
    double acc[PW];
#pragma unroll
    for (int q = 0; q < PW; ++q) {
        const int j = tab.row[P * PW + q], l = tab.col[P * PW + q];
        double v = 0.0;
        if (j >= 0 && T.act) {
            const int tj = j % HM, tl = l % HM, yj = j / HM, yl = l / HM;
            // Qi[a][b] with a, b <= c: read from column max(a, b)
            auto qi = [&](int a, int b) -> double {
                if (a < 0 || b < 0) return 0.0;
                const int cc = a > b ? a : b, rr = a > b ? b : a;
                return qc[cc - C0][rr];
            };
            double qq = qi(tj, tl);
            if (yj == 1) qq -= qi(tj - 1, tl);
            if (yl == 1) qq -= qi(tj, tl - 1);
            if (yj == 1 && yl == 1) qq += qi(tj - 1, tl - 1);
            auto coef = [&](int ty, int t) -> double {
                if (t >= T.H) return 0.0;
                if (ty == 0) return T.alpha(t, sh);
                if (ty == 1) return T.ht ? T.eps(t, sh) : 0.0;
                return 1.0;
            };
            v = coef(yj, tj) * coef(yl, tl) * qq;
        }
        acc[q] = v;
    }
    block_sum_lds<PW>(acc, sh.red, sh.panel, nw);
    if (threadIdx.x < PW) {
        // (j, l) of this lane's entry via compile-time selects (no runtime table lookup)
        int j = -1, l = -1;
#pragma unroll
        for (int q = 0; q < PW; ++q)
            if ((int)threadIdx.x == q) { j = tab.row[P * PW + q]; l = tab.col[P * PW + q]; }
        if (j >= 0) {
            sh.G[j * KM + l] = sh.panel[threadIdx.x];
            sh.G[l * KM + j] = sh.panel[threadIdx.x];
        }
    }
    __syncthreads();
    if constexpr (P + 1 < Tri<HM>::NP) gram_panel<HM, P + 1>(T, sh, dq, nw);
}

// Factor: per-asset LDL^T of Q and explicit Q^{-1} (registers), Schur matrix + Cholesky (LDS).
// Returns false on breakdown (non-positive pivot).
template <int HM>
__device__ __forceinline__ bool factor(Thread<HM>& T, Shared<HM>& sh, int nw) {
    constexpr int KM = 3 * HM;
    const int H = T.H;
    double E[HM], W1[HM], sp[HM];
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        W1[t] = E[t] = T.P[t] = T.bma[t] = sp[t] = 0.0;
        if (T.act && t < H) {
            const double d = T.w[t] - T.wprev(t);
            W1[t] = T.hw ? T.l1[t] / T.w[t] : 0.0;
            if (T.hs) {
                const double al = T.l2[t] / (T.s[t] - d), be = T.l3[t] / (T.s[t] + d);
                const double P = 1.0 / (al + be);
                T.P[t] = P;
                E[t] = 4.0 * al * be * P;
                T.bma[t] = be - al;
                sp[t] = P;
            }
        }
    }
    period_sums<HM>(sp, sp, sh.red, nw);
    if (threadIdx.x == 0) {
        sh.flag = 0;
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            const double ga = (T.ht && t < H) ? sh.l4[t] / sh.z4[t] : 0.0;
            sh.rho[t] = (T.ht && t < H) ? ga / (1.0 + ga * sp[t]) : 0.0;
            sh.sr[t] = sqrt(sh.rho[t]);
        }
    }
    // per-asset LDL^T of Q = diag(W1) + D^T E D, cancellation free
    bool ok = true;
    {
        double pi = W1[0] + E[0];
#pragma unroll
        for (int t = 0; t < HM; ++t) {
            T.Dd[t] = 1.0;
            T.Lr[t] = 0.0;
            if (T.act && t < H) {
                if (t > 0) {
                    T.Lr[t] = E[t] / T.Dd[t - 1];
                    pi = W1[t] + T.Lr[t] * pi;
                }
                T.Dd[t] = pi + ((t + 1 < HM && t + 1 < H) ? E[t + 1] : 0.0);
                ok = ok && (T.Dd[t] > 0.0) && (T.Dd[t] < 1e300);
            }
        }
    }
    __syncthreads();
    if (!ok) sh.flag = 1;
    // diagonal of Q^{-1}: dq_s = 1/Dd_s + Lr_{s+1}^2 dq_{s+1}
    double dq[HM];
#pragma unroll
    for (int sidx = HM - 1; sidx >= 0; --sidx) {
        double v = 0.0;
        if (T.act && sidx < H) {
            v = 1.0 / T.Dd[sidx];
            if (sidx + 1 < HM && sidx + 1 < H) v += T.Lr[sidx + 1] * T.Lr[sidx + 1] * dq[sidx + 1];
        }
        dq[sidx] = v;
    }
    __syncthreads();   // sh.rho / sh.sr (thread 0) visible to alpha/eps
    gram_panel<HM, 0>(T, sh, dq, nw);
    // wave 0: identity on the U columns and unused padding columns, then Cholesky in place
    if (threadIdx.x < WAVE) {
        const int lane = threadIdx.x;
        if (lane < KM) {
            const int tt = lane % HM, ty = lane / HM;
            const bool used = tt < H && (ty != 1 || T.ht);
            if (!used) {
                for (int l = 0; l < KM; ++l) { sh.G[lane * KM + l] = 0.0; sh.G[l * KM + lane] = 0.0; }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane < KM) {
            const int tt = lane % HM, ty = lane / HM;
            const bool used = tt < H && (ty != 1 || T.ht);
            if (ty < 2 || !used) sh.G[lane * KM + lane] += 1.0;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // left-looking Cholesky, lane r owns row r
        bool bad = false;
        for (int j = 0; j < KM; ++j) {
            double v = 0.0;
            if (lane >= j && lane < KM) {
                v = sh.G[lane * KM + j];
                for (int p = 0; p < j; ++p) v -= sh.G[lane * KM + p] * sh.G[j * KM + p];
            }
            const double dj = __shfl(v, j, WAVE);
            bad = bad || !(dj > 0.0) || !(dj < 1e300);
            const double sd = sqrt(fmax(dj, 1e-300));
            if (lane == j) sh.G[j * KM + j] = sd;
            if (lane > j && lane < KM) sh.G[lane * KM + j] = v / sd;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (bad && lane == 0) sh.flag = 1;
    }
    __syncthreads();
    return sh.flag == 0;
}

// Write the current iterate as the answer (W[0] or W) and return problem.value at it:
// sum_t log(w_t . exp(y_t)) - c sum_t ||w_t - w_{t-1}||_1  (mpc.py:66-103).
template <int HM>
__device__ __forceinline__ double record_best(const Thread<HM>& T, Shared<HM>& sh, double* wout,
                                              const float* yh, double c, int tw, int nw) {
    const int H = T.H, N = T.N;
    double rw[HM], l1n[HM];
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        rw[t] = l1n[t] = 0.0;
        if (T.act && t < H) {
            if (t < tw) wout[t * N + T.i] = T.w[t];
            rw[t] = exp((double)yh[t * N + T.i]) * T.w[t];
            l1n[t] = fabs(T.w[t] - T.wprev(t));
        }
    }
    period_sums<HM>(rw, rw, sh.red, nw);
    period_sums<HM>(l1n, l1n, sh.red, nw);
    double f = 0.0;
#pragma unroll
    for (int t = 0; t < HM; ++t)
        if (t < H) f += log(rw[t]) - c * l1n[t];
    return f;
}

template <int HM, int MAXT>
__global__ void __launch_bounds__(MAXT) ipm_kernel(SolveArgs args) {
    static_assert(3 * HM <= WAVE, "Schur system must fit one wave");
    __shared__ Shared<HM> sh;
    const int b = blockIdx.x;
    const int nw = blockDim.x / WAVE;
    Thread<HM> T;
    T.H = args.H;
    T.N = args.N;
    T.i = threadIdx.x;
    T.act = T.i < args.N;
    T.hw = !args.allow_short;
    T.hs = (args.c > 0.0) || (args.tau > 0.0);
    T.ht = args.tau > 0.0;
    T.tau = args.tau;
    const int H = T.H, N = T.N;
    const double* wp = args.wp + (size_t)b * N;
    const float* yh = args.yhat + (size_t)b * H * N;
    T.wpi = T.act ? wp[T.i] : 0.0;

    // ---- inputs: m = expm1(yhat), objective scale, finiteness ----
    double mx = 0.0;
    bool finite = true;
#pragma unroll
    for (int t = 0; t < HM; ++t) {
        T.m[t] = 0.0;
        if (T.act && t < H) {
            const double y = (double)yh[t * N + T.i];
            finite = finite && isfinite(y);
            T.m[t] = expm1(y);
            mx = fmax(mx, fabs(T.m[t]));
        }
    }
    if (T.act) finite = finite && isfinite(T.wpi);
    mx = block_max1(mx, sh.red, nw);
    const double nonfinite = block_max1(finite ? 0.0 : 1.0, sh.red, nw);
    double sig = fmax(mx, args.c);
    if (!(sig > 0.0)) sig = 1.0;
    T.sig = sig;
    T.rsig = sqrt(sig);
    T.c = args.c / sig;

    int status = KMPC_STATUS_SOLVER_ERROR;
    int it = 0;
    double* wout = args.wout + (size_t)b * (args.return_full ? H * N : N);
    const int tw = args.return_full ? H : 1;   // periods written out
    double best_obj = __builtin_nan("");

    if (nonfinite == 0.0 && isfinite(args.c) && isfinite(args.tau)) {
        if (args.allow_short && !T.hs) {
            // no bounds and no turnover terms: unbounded unless every period is flat
            double msum[HM];
#pragma unroll
            for (int t = 0; t < HM; ++t) msum[t] = (T.act && t < H) ? T.m[t] : 0.0;
            period_sums<HM>(msum, msum, sh.red, nw);
            double spread = 0.0;
#pragma unroll
            for (int t = 0; t < HM; ++t)
                if (T.act && t < H) spread = fmax(spread, fabs(T.m[t] - msum[t] / N));
            spread = block_max1(spread, sh.red, nw);
            if (spread == 0.0) {
                const double swp = block_sum1(T.act ? T.wpi : 0.0, sh.red, nw);
#pragma unroll
                for (int t = 0; t < HM; ++t) T.w[t] = swp != 0.0 ? T.wpi / swp : 1.0 / N;
                best_obj = record_best<HM>(T, sh, wout, yh, args.c, tw, nw);
                status = KMPC_STATUS_OPTIMAL;
            } else {
                status = KMPC_STATUS_UNBOUNDED;
            }
        } else {
            // ---- initial point ----
#pragma unroll
            for (int t = 0; t < HM; ++t) {
                const double b0 = T.hw ? fmax(T.wpi, 0.0) : T.wpi;
                T.w[t] = (T.act && t < H) ? 0.5 * b0 + 0.5 / N : 0.0;
            }
            double ss0[HM];
#pragma unroll
            for (int t = 0; t < HM; ++t) {
                const bool on = T.act && t < H;
                const double d = T.w[t] - T.wprev(t);
                T.s[t] = (on && T.hs) ? fabs(d) + 1.0 / N : 0.0;
                ss0[t] = T.s[t];
                T.l1[t] = (on && T.hw) ? 1.0 : 0.0;
                T.l2[t] = T.l3[t] = (on && T.hs) ? 1.0 : 0.0;
            }
            period_sums<HM>(ss0, ss0, sh.red, nw);
            if (threadIdx.x == 0) {
#pragma unroll
                for (int t = 0; t < HM; ++t) {
                    sh.z4[t] = (T.ht && t < H) ? fmax(T.tau - ss0[t], 0.5 * T.tau) : 1.0;
                    sh.l4[t] = (T.ht && t < H) ? 1.0 : 0.0;
                    sh.nu[t] = 0.0;
                }
            }
            __syncthreads();
            const int ncon = (T.hw ? H * N : 0) + (T.hs ? 2 * H * N : 0) + (T.ht ? H : 0);
            const double inv_ncon = 1.0 / (ncon > 0 ? ncon : 1);
            double best = 1e300, best_pr = 1e300, best_dr = 1e300, best_mu = 1e300, min_pr = 1e300;

            for (it = 0; it < args.max_iter; ++it) {
                // ---- residuals: den_t = 1 + m.w, 1'w_t - 1, tau - 1's_t - z4 ----
                {
                    double mw[HM], sw[HM], ssum[HM];
#pragma unroll
                    for (int t = 0; t < HM; ++t) {
                        const bool on = T.act && t < H;
                        mw[t] = on ? T.m[t] * T.w[t] : 0.0;
                        sw[t] = on ? T.w[t] : 0.0;
                        ssum[t] = on ? T.s[t] : 0.0;
                    }
                    period_sums<HM>(mw, mw, sh.red, nw);
                    period_sums<HM>(sw, sw, sh.red, nw);
                    period_sums<HM>(ssum, ssum, sh.red, nw);
                    if (threadIdx.x == 0) {
#pragma unroll
                        for (int t = 0; t < HM; ++t) {
                            const bool on = t < H;
                            sh.den[t] = 1.0 + mw[t];
                            sh.rp[t] = on ? sw[t] - 1.0 : 0.0;
                            sh.rg4[t] = (T.ht && on) ? T.tau - ssum[t] - sh.z4[t] : 0.0;
                            sh.rc4[t] = (T.ht && on) ? sh.z4[t] * sh.l4[t] : 0.0;
                        }
                    }
                    __syncthreads();
                }
                double mu_l = 0.0, rd = 0.0;
#pragma unroll
                for (int t = 0; t < HM; ++t) {
                    if (T.act && t < H) {
                        const double d = T.w[t] - T.wprev(t);
                        double rdw, rds;
                        dual_residual<HM>(T, sh, t, rdw, rds);
                        mu_l += (T.hw ? T.w[t] * T.l1[t] : 0.0) +
                                (T.hs ? (T.s[t] - d) * T.l2[t] + (T.s[t] + d) * T.l3[t] : 0.0);
                        rd = fmax(rd, fmax(fabs(rdw), fabs(rds)));
                    }
                }
                double mu = block_sum1(mu_l, sh.red, nw);
                rd = block_max1(rd, sh.red, nw);
                double pr = 0.0;
                bool domain_ok = true;
                for (int t = 0; t < H; ++t) {
                    mu += sh.rc4[t];
                    pr = fmax(pr, fmax(fabs(sh.rp[t]), fabs(sh.rg4[t])));
                    domain_ok = domain_ok && sh.den[t] > 0.0;
                }
                mu *= inv_ncon;
                const double merit = fmax(mu, fmax(rd, pr));
                min_pr = fmin(min_pr, pr);
                if (args.trace && b == 0 && threadIdx.x == 0) {
                    args.trace[4 * it + 0] = mu; args.trace[4 * it + 1] = rd; args.trace[4 * it + 2] = pr;
                }
                if (!domain_ok || !isfinite(merit)) break;
                if (merit < best) {
                    best = merit; best_pr = pr; best_dr = rd; best_mu = mu;
                    best_obj = record_best<HM>(T, sh, wout, yh, args.c, tw, nw);
                } else if (best < 1e-6 && merit > 1e4 * best) {
                    break;   // numerical breakdown after convergence: keep the best iterate
                }
                if (mu < args.tol && rd < 10.0 * args.tol && pr < 10.0 * args.tol) break;
                if (!factor<HM>(T, sh, nw)) break;
#pragma unroll
                for (int t = 0; t < HM; ++t) {
                    T.rc1[t] = T.rc2[t] = T.rc3[t] = 0.0;
                    if (T.act && t < H) {
                        const double d = T.w[t] - T.wprev(t);
                        T.rc1[t] = T.hw ? T.w[t] * T.l1[t] : 0.0;
                        T.rc2[t] = T.hs ? (T.s[t] - d) * T.l2[t] : 0.0;
                        T.rc3[t] = T.hs ? (T.s[t] + d) * T.l3[t] : 0.0;
                    }
                }

                // ---- predictor (pass 0) and corrector (pass 1) share one Newton body ----
                double step = 0.0;
                for (int pass = 0; pass < 2; ++pass) {
                    newton<HM>(T, sh, nw, args.n_refine);
                    const double amax = max_step<HM>(T, sh, nw);
                    if (pass == 1) { step = fmin(1.0, 0.99 * amax); break; }
                    const double ap = fmin(1.0, amax);
                    double sg = complementarity<HM>(T, sh, ap, nw) * inv_ncon / mu;
                    sg = sg * sg * sg;
                    const double smu = sg * mu;
#pragma unroll
                    for (int t = 0; t < HM; ++t) {
                        if (T.act && t < H) {
                            double dl1, dl2, dl3;
                            dual_dirs<HM>(T, t, dl1, dl2, dl3);
                            const double dd = T.dw[t] - (t ? T.dw[t - 1] : 0.0);
                            if (T.hw) T.rc1[t] += T.dw[t] * dl1 - smu;
                            if (T.hs) {
                                T.rc2[t] += (T.ds[t] - dd) * dl2 - smu;
                                T.rc3[t] += (T.ds[t] + dd) * dl3 - smu;
                            }
                        }
                    }
                    if (threadIdx.x < HM && T.ht && (int)threadIdx.x < H) {
                        const int t = threadIdx.x;
                        sh.rc4[t] += sh.dz4[t] * sh.dl4[t] - smu;
                    }
                    __syncthreads();
                }
                if (args.trace && b == 0 && threadIdx.x == 0) args.trace[4 * it + 3] = step;
                // ---- update ----
#pragma unroll
                for (int t = 0; t < HM; ++t) {
                    if (T.act && t < H) {
                        double dl1, dl2, dl3;
                        dual_dirs<HM>(T, t, dl1, dl2, dl3);
                        T.l1[t] += step * dl1;
                        T.l2[t] += step * dl2;
                        T.l3[t] += step * dl3;
                    }
                }
#pragma unroll
                for (int t = 0; t < HM; ++t) {
                    if (T.act && t < H) {
                        T.w[t] += step * T.dw[t];
                        T.s[t] += step * T.ds[t];
                    }
                }
                if (threadIdx.x < HM && (int)threadIdx.x < H) {
                    const int t = threadIdx.x;
                    sh.z4[t] += step * sh.dz4[t];
                    sh.l4[t] += step * sh.dl4[t];
                    sh.nu[t] += step * sh.dnu[t];
                }
                __syncthreads();
            }
            if (best <= 1e-7) status = KMPC_STATUS_OPTIMAL;
            else if (best <= 1e-4) status = KMPC_STATUS_OPTIMAL_INACCURATE;
            else if (min_pr > 1e-6) status = KMPC_STATUS_INFEASIBLE;   // primal residual never closed
            else status = KMPC_STATUS_SOLVER_ERROR;
            (void)best_pr; (void)best_dr; (void)best_mu;
        }
    }
    __syncthreads();
    // ---- outputs: W was written by record_best; fallback (mpc.py:113-115) otherwise ----
    const bool ok = status == KMPC_STATUS_OPTIMAL || status == KMPC_STATUS_OPTIMAL_INACCURATE;
    if (!ok && T.act) {
#pragma unroll
        for (int t = 0; t < HM; ++t)
            if (t < tw) wout[t * N + T.i] = T.wpi;
    }
    if (threadIdx.x == 0) {
        args.obj[b] = ok ? best_obj : __builtin_nan("");
        args.status[b] = status;
        if (args.iters) args.iters[b] = it;
    }
}

template <int HM>
static int launch_ipm(const SolveArgs& a, hipStream_t stream) {
    const int nt = WAVE * ((a.N + WAVE - 1) / WAVE);
    if (nt <= 256)
        hipLaunchKernelGGL((ipm_kernel<HM, 256>), dim3(a.B), dim3(nt), 0, stream, a);
    else
        hipLaunchKernelGGL((ipm_kernel<HM, 1024>), dim3(a.B), dim3(nt), 0, stream, a);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

int solve_launch(const kmpc_solve_desc* d, const float* yhat, const double* w_prev, double* w_out,
                 int* status, double* obj, int* iters, hipStream_t stream, double* trace) {
    SolveArgs a;
    a.B = d->B; a.N = d->N; a.H = d->H;
    a.c = d->cost_coeff;
    a.tau = d->max_turnover > 0.0 ? d->max_turnover : 0.0;
    a.allow_short = d->allow_short;
    a.max_iter = d->max_iter > 0 ? d->max_iter : 80;
    a.tol = d->tol > 0.0 ? d->tol : 1e-11;
    a.return_full = d->return_full_W;
    a.n_refine = d->n_refine > 0 ? d->n_refine : (d->n_refine < 0 ? 0 : 3);
    a.yhat = yhat; a.wp = w_prev; a.wout = w_out; a.status = status; a.obj = obj; a.iters = iters;
    a.trace = trace;
    if (a.B == 0) return KMPC_OK;
#ifndef KMPC_DEV_ONLY_H10
    if (a.H <= 2) return launch_ipm<2>(a, stream);
    if (a.H <= 5) return launch_ipm<5>(a, stream);
#endif
    if (a.H <= 10) return launch_ipm<10>(a, stream);
#ifndef KMPC_DEV_ONLY_H10
    if (a.H <= 21) return launch_ipm<21>(a, stream);
#endif
    return KMPC_ERR_UNSUPPORTED;
}

}  // namespace kmpc

#ifdef KMPC_STATS
extern "C" int kmpc_debug_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmpc::g_stats), sizeof(unsigned long long) * 2) != hipSuccess)
        return KMPC_ERR_LAUNCH;
    if (reset) {
        unsigned long long z[2] = {0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(kmpc::g_stats), z, sizeof(z)) != hipSuccess) return KMPC_ERR_LAUNCH;
    }
    return KMPC_OK;
}
#endif
