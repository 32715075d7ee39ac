// kmpc_mv.hip — batched mean-variance MPC solve (replaces solve_mpc_mean_variance, mpc.py:119-184)
// and the Markowitz rolling moments (MarkowitzStrategy.rebalance, baselines.py:70-88).
//
// Program per window (mpc.py:128, 145-172):
//   maximize  sum_t [ w_t . mu_t - gamma w_t' Sigma w_t ] - c sum_t ||w_t - w_{t-1}||_1
//   s.t.      1'w_t = 1, w_t >= 0 unless allow_short          (no turnover cap), w_{-1} = w_prev.
// One workgroup per window, one element (t, i) of W per thread (n = H N <= 1024). Algorithm:
// Mehrotra predictor-corrector primal-dual interior point on the epigraph form (s_ti >= |d_ti|,
// d = w_t - w_{t-1}), float64, objective scaled by max(|mu|, 2 gamma |Sigma|, c). The s rows and
// all multipliers are eliminated per element, leaving the dense SPD system
//   M dw + A' dnu = r,  A dw = r2,   M = 2 gamma (I_H (x) Sigma) + diag(l1 / w) + D' diag(E) D
// (D: differencing in t, E = 4 alpha beta / (alpha + beta) from the two |d| rows), solved with a
// right-looking Cholesky of M in LDS (thread r owns row r) and the H x H Schur complement
// S = A M^{-1} A' for the budget multipliers. Test-side restatement: oracle/mv_ref.py.
// Storage: M (n x n) and M^{-1} A' sit in LDS while they fit (n <= 128); past that in a per-block
// slab of the caller's workspace (L2-resident: 2 MB at n = 500), with a persistent grid of
// min(B, MV_SLOTS) blocks walking the windows.
//
// Status / fallback as mpc.py:180-181: non-optimal -> W = tile(w_prev), obj = NaN.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kmpc_internal.h"

namespace kmpc {
namespace {

struct MvArgs {
    int B, N, H;
    double gamma, c;
    int allow_short, max_iter, return_full;
    double tol;
    const double* mu;       // [B, H, N]
    const double* sigma;    // [B, N, N], or one [N, N] when sigma_stride == 0
    size_t sigma_stride;    // elements between consecutive windows' Sigma
    const double* wp;       // [B, N]
    double* wout;           // [B, N] or [B, H, N]
    int* status;
    double* obj;
    int* iters;
    double* ws;             // workspace slabs (global-M variant)
    size_t slab;            // doubles per slab
};

constexpr int MV_SLOTS = 512;   // windows in flight of the global-M variant

__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
// block reductions (<= 2 waves): wave reduce, one slot per wave, fixed summation order
__device__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += red[q];
    return s;
}
__device__ double block_max(double v, double* red) {
    v = wave_max(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = red[0];
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q) s = fmax(s, red[q]);
    return s;
}
__device__ double block_min(double v, double* red) {
    v = wave_min(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = red[0];
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q) s = fmin(s, red[q]);
    return s;
}
// value of element k - N (previous period) / k + N (next period) of a per-thread vector
__device__ double prev_period(double v, double* vec, int k, int n, int N, double first) {
    __syncthreads();
    if (k < n) vec[k] = v;
    __syncthreads();
    return (k < n && k >= N) ? vec[k - N] : first;
}
__device__ double next_period(double v, double* vec, int k, int n, int N) {
    __syncthreads();
    if (k < n) vec[k] = v;
    __syncthreads();
    return (k + N < n) ? vec[k + N] : 0.0;
}
// per-period sums of a per-thread vector into pv[H] (visible to all threads on return)
__device__ void period_sums(double v, double* vec, double* pv, int k, int n, int N, int H) {
    __syncthreads();
    if (k < n) vec[k] = v;
    __syncthreads();
    if (k < H) {
        double s = 0.0;
        for (int j = 0; j < N; ++j) s += vec[k * N + j];
        pv[k] = s;
    }
    __syncthreads();
}
__device__ __forceinline__ double to_bound(double v, double dv, double a) {
    return dv < 0.0 ? fmin(a, -v / dv) : a;
}

// M and its factor L are stored packed lower-triangular, row r at r (r + 1) / 2: the factorization
// and the solves only touch entries (r, c <= r), and the packed window fits three per CU at n = 100.
__device__ __forceinline__ size_t tri(int r, int c) { return (size_t)r * (r + 1) / 2 + c; }

// x = M^{-1} b with M = L L' (lower factor in place, packed); thread r owns row r. (A
// single-wave variant with the vector in registers and v_readlane broadcasts measured no faster at
// n = 100 and 11% slower at n = 300: the factorization, not the solves, bounds this kernel.)
__device__ double chol_solve(const double* M, int n, double b, double* vec) {
    const int r = threadIdx.x;
    double x = b;
    for (int j = 0; j < n; ++j) {
        if (r == j) vec[j] = x / M[tri(j, j)];
        __syncthreads();
        if (r > j && r < n) x -= M[tri(r, j)] * vec[j];
    }
    double y = r < n ? vec[r] : 0.0;
    __syncthreads();
    for (int j = n - 1; j >= 0; --j) {
        if (r == j) vec[j] = y / M[tri(j, j)];
        __syncthreads();
        if (r < j) y -= M[tri(j, r)] * vec[j];
    }
    const double out = r < n ? vec[r] : 0.0;
    __syncthreads();
    return out;
}


// One window. GM: M and Y in the block's workspace slab (else in LDS after the small arrays).
template <bool GM>
__device__ __forceinline__ void mv_window(const MvArgs& a, int b, double* lds) {
    const int N = a.N, H = a.H, n = N * H;
    double* vec = lds;                      // [n] broadcast vector
    double* Sm = vec + n;                   // [H][H] A M^{-1} A', then its Cholesky factor
    double* idg = Sm + H * H + 4 * H + 18;  // [n] 1 / L_jj of the Cholesky factor
    double* M = GM ? a.ws + (size_t)blockIdx.x * a.slab : idg + n;   // packed lower: M, then L
    double* Y = M + tri(n, 0);              // [H][n] M^{-1} A'
    double* pv = Sm + H * H;                // [H] period sums (after Sm in LDS, both variants)
    double* nu = pv + H;                    // [H] budget multipliers
    double* dnu = nu + H;                   // [H]
    double* rpv = dnu + H;                  // [H] primal residuals 1'w_t - 1
    double* red = rpv + H;                  // [16] reduction slots (one per wave)
    int* flag = (int*)(red + 16);

    const int k = threadIdx.x;
    const bool act = k < n;
    const int t = act ? k / N : 0, i = act ? k - (k / N) * N : 0;
    const double* Sig = a.sigma + a.sigma_stride * (size_t)b;
    const double* wpv = a.wp + (size_t)b * N;
    const double* muv = a.mu + (size_t)b * n;
    const bool hw = !a.allow_short, hs = a.c > 0.0;
    const double wpi = act ? wpv[i] : 0.0;
    const double mk = act ? muv[k] : 0.0;
    double* wout = a.wout + (size_t)b * (a.return_full ? n : N);
    const int nout = a.return_full ? n : N;

    // scale and finiteness
    double smax = 0.0;
    bool finite = isfinite(mk) && isfinite(wpi);
    for (int j = k; j < N * N; j += blockDim.x) {
        const double v = Sig[j];
        finite = finite && isfinite(v);
        smax = fmax(smax, fabs(v));
    }
    const double nonfinite = block_max(finite ? 0.0 : 1.0, red);
    double sc = block_max(fmax(fabs(mk), 2.0 * a.gamma * smax), red);
    sc = fmax(sc, a.c);
    if (!(sc > 0.0) || !isfinite(sc)) sc = 1.0;
    const double g2 = 2.0 * a.gamma / sc, cs = a.c / sc, mus = mk / sc;

    int status = KMPC_STATUS_SOLVER_ERROR, it = 0;
    double best = 1e300, best_obj = __builtin_nan("");
    bool unbounded = false;

    if (nonfinite == 0.0 && isfinite(a.gamma) && isfinite(a.c) && !hw && !hs && !(a.gamma > 0.0)) {
        // no bounds, no cost, no curvature: a linear program over the budget planes, unbounded
        // unless every period's returns are flat (then any budget point is optimal: w_prev scaled)
        period_sums(mk, vec, pv, k, n, N, H);
        const double spread = block_max(act ? fabs(mk - pv[t] / N) : 0.0, red);
        if (spread == 0.0) {
            const double swp = block_sum(k < N ? wpi : 0.0, red);
            const double w = swp != 0.0 ? wpi / swp : 1.0 / N;
            best_obj = block_sum(act ? mk * w : 0.0, red);
            if (act && k < nout) wout[k] = w;
            status = KMPC_STATUS_OPTIMAL;
        } else {
            status = KMPC_STATUS_UNBOUNDED;
        }
    } else if (nonfinite == 0.0 && isfinite(a.gamma) && isfinite(a.c)) {
        double w = act ? 0.5 * (hw ? fmax(wpi, 0.0) : wpi) + 0.5 / N : 0.0;
        double wm = prev_period(w, vec, k, n, N, wpi);
        double s = (act && hs) ? fabs(w - wm) + 1.0 / N : 0.0;
        // slacks of the two |d| rows kept as variables (no cancellation in s -+ d near the optimum)
        double z2 = (act && hs) ? fmax(s - (w - wm), 1e-2) : 1.0, z3 = (act && hs) ? fmax(s + (w - wm), 1e-2) : 1.0;
        double l1 = (act && hw) ? 1.0 : 0.0, l2 = (act && hs) ? 1.0 : 0.0, l3 = l2;
        if (k < H) nu[k] = 0.0;
        const int mcon = (hw ? n : 0) + (hs ? 2 * n : 0);
        const double inv_m = 1.0 / (mcon > 0 ? mcon : 1);

        for (it = 0; it < a.max_iter; ++it) {
            // ---- residuals ----
            wm = prev_period(w, vec, k, n, N, wpi);   // vec holds w afterwards
            double Sw = 0.0;
            if (act)
            {   // Sigma w per element: column i (= row i, symmetric: coalesced across the block),
                // four partial sums so the L2 loads of a group are in flight together
                double s4[4] = {0.0, 0.0, 0.0, 0.0};
                int j = 0;
                for (; j + 4 <= N; j += 4) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) s4[e] += Sig[(size_t)(j + e) * N + i] * vec[t * N + j + e];
                }
                for (; j < N; ++j) s4[0] += Sig[(size_t)j * N + i] * vec[t * N + j];
                Sw = (s4[0] + s4[1]) + (s4[2] + s4[3]);
            }
            const double d = w - wm;
            const double rg2 = (act && hs) ? (s - d) - z2 : 0.0, rg3 = (act && hs) ? (s + d) - z3 : 0.0;
            const double eta = l2 - l3;
            const double etan = next_period(eta, vec, k, n, N);
            period_sums(w, vec, pv, k, n, N, H);
            if (k < H) rpv[k] = pv[k] - 1.0;
            double prmax = 0.0;
            for (int q = 0; q < H; ++q) prmax = fmax(prmax, fabs(pv[q] - 1.0));
            const double rw = act ? -mus + g2 * Sw - l1 + eta - etan + nu[t] : 0.0;
            const double rs = (act && hs) ? cs - l2 - l3 : 0.0;
            const double mu_c = block_sum(act ? w * l1 + z2 * l2 + z3 * l3 : 0.0, red) * inv_m;
            const double rd = block_max(fmax(fmax(fabs(rw), fabs(rs)), fmax(fabs(rg2), fabs(rg3))), red);
            const double wabs = block_max(act ? fabs(w) : 0.0, red);
            const double merit = fmax(mu_c, fmax(rd, prmax));
            if (!isfinite(merit)) break;
            if (wabs > 1e7) { unbounded = true; break; }
            if (merit < best) {
                best = merit;
                // problem.value (mpc.py:172) in the reference's maximize form, unscaled
                const double f = block_sum(act ? mk * w - a.gamma * w * Sw - a.c * fabs(d) : 0.0, red);
                best_obj = f;
                if (act && k < nout) wout[k] = w;
            }
            if (mu_c < a.tol && rd < 10.0 * a.tol && prmax < 10.0 * a.tol) break;

            // ---- factor: M = 2 gamma (I (x) Sigma) + diag(W1) + D' diag(E) D ----
            const double W1 = (act && hw) ? l1 / w : 0.0;
            const double al = (act && hs) ? l2 / z2 : 0.0, be = (act && hs) ? l3 / z3 : 0.0;
            const double P = (act && hs) ? 1.0 / (al + be) : 0.0;
            const double E = 4.0 * al * be * P;
            const double En = next_period(E, vec, k, n, N);
            if (act) {   // column k, rows l >= k (M symmetric): lanes write consecutive entries
                for (int l = k; l < n; ++l) {
                    const int tl = l / N, j = l - tl * N;
                    double v = (tl == t) ? g2 * Sig[(size_t)j * N + i] : 0.0;
                    if (l == k) v += W1 + E + En;
                    if (l == k + N) v -= En;
                    M[tri(l, k)] = v;
                }
            }
            if (k == 0) *flag = 0;
            __syncthreads();
            // right-looking Cholesky in panels of PB columns (thread k owns row k): inside a panel
            // column by column (pivot, scale, update of the panel's remaining columns); then the
            // trailing matrix at once, M[k][c] -= L[k][panel] . L[c][panel] with row k's panel in
            // registers — one read-modify-write per entry per panel instead of per column
            constexpr int PB = 8;
            for (int jb = 0; jb < n; jb += PB) {
                const int je = jb + PB < n ? jb + PB : n;
                for (int j = jb; j < je; ++j) {
                    if (k == j) {
                        const double dj = M[tri(j, j)];
                        if (!(dj > 0.0) || !(dj < 1e300)) *flag = 1;
                        const double lj = sqrt(fmax(dj, 1e-300));
                        M[tri(j, j)] = lj;
                        idg[j] = 1.0 / lj;
                    }
                    __syncthreads();
                    if (k > j && k < n) M[tri(k, j)] *= idg[j];
                    __syncthreads();   // column j of L complete before any row reads it
                    if (k > j && k < n) {
                        double* mr = M + tri(k, 0);
                        const double lkj = mr[j];
                        const int qe = k < je - 1 ? k : je - 1;   // the panel's columns in row k
                        for (int q = j + 1; q <= qe; ++q) mr[q] = fma(-lkj, M[tri(q, j)], mr[q]);
                    }
                }
                __syncthreads();
                if (k >= je && k < n) {
                    double* mr = M + tri(k, 0);
                    double lk[PB];
#pragma unroll
                    for (int p = 0; p < PB; ++p) lk[p] = jb + p < je ? mr[jb + p] : 0.0;
                    for (int c = je; c <= k; ++c) {
                        const double* mc = M + tri(c, jb);
                        double lc[PB];
#pragma unroll
                        for (int p = 0; p < PB; ++p) lc[p] = jb + p < je ? mc[p] : 0.0;
                        double v = mr[c];
#pragma unroll
                        for (int p = 0; p < PB; ++p) v = fma(-lk[p], lc[p], v);
                        mr[c] = v;
                    }
                }
                __syncthreads();
            }
            __syncthreads();
            if (*flag) break;
            // Y = M^{-1} A' (one column per period) and S = A Y
            for (int q = 0; q < H; ++q) {
                const double bq = (act && t == q) ? 1.0 : 0.0;
                const double yq = chol_solve(M, n, bq, vec);
                if (act) Y[(size_t)q * n + k] = yq;
                period_sums(yq, vec, pv, k, n, N, H);
                if (k < H) Sm[k * H + q] = pv[k];
                __syncthreads();
            }
            if (k == 0) {   // Cholesky of the H x H Schur complement
                for (int j = 0; j < H; ++j) {
                    double dj = Sm[j * H + j];
                    for (int q = 0; q < j; ++q) dj -= Sm[j * H + q] * Sm[j * H + q];
                    if (!(dj > 0.0) || !isfinite(dj)) *flag = 1;
                    dj = sqrt(fmax(dj, 1e-300));
                    Sm[j * H + j] = dj;
                    for (int r = j + 1; r < H; ++r) {
                        double v = Sm[r * H + j];
                        for (int q = 0; q < j; ++q) v -= Sm[r * H + q] * Sm[j * H + q];
                        Sm[r * H + j] = v / dj;
                    }
                }
            }
            __syncthreads();
            if (*flag) break;

            // ---- predictor (pass 0) / corrector (pass 1) ----
            double rc1 = (act && hw) ? w * l1 : 0.0, rc2 = (act && hs) ? z2 * l2 : 0.0;
            double rc3 = (act && hs) ? z3 * l3 : 0.0;
            double dw = 0.0, ds = 0.0, dl1 = 0.0, dl2 = 0.0, dl3 = 0.0, step = 0.0, prev_dw = 0.0;
            for (int pass = 0; pass < 2; ++pass) {
                const double p2 = rc2 / z2 + al * rg2, p3 = rc3 / z3 + be * rg3;
                const double qs = (act && hs) ? -rs - p2 - p3 : 0.0;
                const double v = (act && hs) ? (be - al) * P * qs + p3 - p2 : 0.0;
                const double vn = next_period(v, vec, k, n, N);
                const double rhs = act ? -rw - (hw ? rc1 / w : 0.0) - (v - vn) : 0.0;
                const double x = chol_solve(M, n, rhs, vec);
                period_sums(x, vec, pv, k, n, N, H);
                if (k == 0) {   // dnu = S^{-1} (A x + r_p)
                    for (int j = 0; j < H; ++j) {
                        double u = pv[j] + rpv[j];
                        for (int q = 0; q < j; ++q) u -= Sm[j * H + q] * dnu[q];
                        dnu[j] = u / Sm[j * H + j];
                    }
                    for (int j = H - 1; j >= 0; --j) {
                        double u = dnu[j];
                        for (int q = j + 1; q < H; ++q) u -= Sm[q * H + j] * dnu[q];
                        dnu[j] = u / Sm[j * H + j];
                    }
                }
                __syncthreads();
                dw = x;
                if (act)
                    for (int q = 0; q < H; ++q) dw -= Y[(size_t)q * n + k] * dnu[q];
                const double dwm = prev_period(dw, vec, k, n, N, 0.0);
                prev_dw = dwm;
                const double dd = dw - dwm;
                ds = (act && hs) ? P * (qs - (be - al) * dd) : 0.0;
                const double dz2 = ds - dd + rg2, dz3 = ds + dd + rg3;
                dl1 = (act && hw) ? -(l1 * dw + rc1) / w : 0.0;
                dl2 = (act && hs) ? -(l2 * dz2 + rc2) / z2 : 0.0;
                dl3 = (act && hs) ? -(l3 * dz3 + rc3) / z3 : 0.0;
                double am = 1e300;
                if (act && hw) { am = to_bound(w, dw, am); am = to_bound(l1, dl1, am); }
                if (act && hs) {
                    am = to_bound(z2, dz2, am); am = to_bound(z3, dz3, am);
                    am = to_bound(l2, dl2, am); am = to_bound(l3, dl3, am);
                }
                am = block_min(am, red);
                if (pass == 1) { step = fmin(1.0, 0.99 * am); break; }
                const double ap = fmin(1.0, am);
                const double mua = block_sum(act ? (w + ap * dw) * (l1 + ap * dl1) + (z2 + ap * dz2) * (l2 + ap * dl2) +
                                                       (z3 + ap * dz3) * (l3 + ap * dl3) : 0.0, red) * inv_m;
                double sg = mua / mu_c;
                sg = sg * sg * sg;
                const double smu = sg * mu_c;
                if (act && hw) rc1 = w * l1 + dw * dl1 - smu;
                if (act && hs) { rc2 = z2 * l2 + dz2 * dl2 - smu; rc3 = z3 * l3 + dz3 * dl3 - smu; }
            }
            w += step * dw;
            s += step * ds;
            if (act && hs) {
                z2 += step * (ds - (dw - prev_dw) + rg2);
                z3 += step * (ds + (dw - prev_dw) + rg3);
            }
            l1 += step * dl1;
            l2 += step * dl2;
            l3 += step * dl3;
            __syncthreads();
            if (k < H) nu[k] += step * dnu[k];
            __syncthreads();
        }
        if (unbounded) status = KMPC_STATUS_UNBOUNDED;
        else if (best <= 1e-7) status = KMPC_STATUS_OPTIMAL;
        else if (best <= 1e-4) status = KMPC_STATUS_OPTIMAL_INACCURATE;
        else status = KMPC_STATUS_SOLVER_ERROR;
    }
    __syncthreads();
    const bool ok = status == KMPC_STATUS_OPTIMAL || status == KMPC_STATUS_OPTIMAL_INACCURATE;
    if (!ok && k < nout) wout[k] = wpv[k % N];   // tile(current_weights), mpc.py:180-181
    if (k == 0) {
        a.obj[b] = ok ? best_obj : __builtin_nan("");
        a.status[b] = status;
        if (a.iters) a.iters[b] = it;
    }
}

template <int MAXT, bool GM>
__global__ void __launch_bounds__(MAXT) mv_ipm_kernel(MvArgs a) {
    extern __shared__ double lds[];
    if (GM) {
        for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
            mv_window<true>(a, b, lds);
            __syncthreads();
        }
    } else {
        mv_window<false>(a, blockIdx.x, lds);
    }
}

// Markowitz moments (baselines.py:70-88) for window b at test index t = ts[b]:
// r_s = z_s * std + mean (float32, data_finance.py:740-742) for the rows s of the last `lookback`
// of [0, t]; mu = mean (float32, as np.mean of the float32 history), Sigma = np.cov (float64,
// ddof 1) + 1e-6 I; valid[b] = (t + 1 >= 5) (baselines.py:76-78).
__global__ void rolling_moments_kernel(int B, int T, int N, int lookback, const float* z, int ldz,
                                       const float* mean, const float* stdv, const int* ts,
                                       double* mu, double* sigma, int* valid) {
    extern __shared__ double ml[];   // [N] float64 means
    const int b = blockIdx.x;
    const int t = ts[b];
    const int hi = min(t + 1, T), lo = max(0, hi - lookback), rows = hi - lo;
    if (threadIdx.x == 0) valid[b] = (t + 1 >= 5 && t < T) ? 1 : 0;
    // z * std + mean as two float32 roundings (torch's mul then add): no FMA contraction here
    auto ret = [&](int s, int j) -> float {
#pragma clang fp contract(off)
        const float p = z[(size_t)s * ldz + j] * stdv[j];
        return p + mean[j];
    };
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
        double acc = 0.0;
        for (int s = lo; s < hi; ++s) acc += (double)ret(s, j);
        const double m = rows > 0 ? acc / rows : 0.0;
        ml[j] = m;
        mu[(size_t)b * N + j] = (double)(float)m;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < N * N; q += blockDim.x) {
        const int r = q / N, c = q - r * N;
        double acc = 0.0;
        for (int s = lo; s < hi; ++s) acc += ((double)ret(s, r) - ml[r]) * ((double)ret(s, c) - ml[c]);
        double v = rows > 1 ? acc / (rows - 1) : 0.0;
        if (r == c) v += 1e-6;
        sigma[(size_t)b * N * N + q] = v;
    }
}

}  // namespace

// LDS of the small arrays (vec, Sm, pv, nu, dnu, rpv, red, flag, idg) and, for the LDS variant, M and Y
size_t mv_small_bytes(int N, int H) {
    return sizeof(double) * (2 * (size_t)N * H + (size_t)H * H + 4 * (size_t)H + 18);
}
size_t mv_lds_bytes(int N, int H) {
    const size_t n = (size_t)N * H;
    return mv_small_bytes(N, H) + sizeof(double) * (n * (n + 1) / 2 + H * n);
}
static bool mv_in_lds(int N, int H) { return (size_t)N * H <= 128 && mv_lds_bytes(N, H) <= 160 * 1024; }
static size_t mv_slab(int N, int H) {
    const size_t n = (size_t)N * H;
    return n * (n + 1) / 2 + H * n;
}
size_t mv_workspace_bytes(const kmpc_mv_desc* d) {
    if (!d || d->B <= 0 || mv_in_lds(d->N, d->H)) return 0;
    const size_t slots = d->B < MV_SLOTS ? d->B : MV_SLOTS;
    return sizeof(double) * mv_slab(d->N, d->H) * slots;
}

int mv_solve_launch(const kmpc_mv_desc* d, const double* mu, const double* sigma, size_t sigma_stride,
                    const double* w_prev, double* w_out, int* status, double* obj, int* iters,
                    void* ws, size_t ws_bytes, hipStream_t stream) {
    MvArgs a;
    a.B = d->B; a.N = d->N; a.H = d->H;
    a.gamma = d->gamma; a.c = d->cost_coeff;
    a.allow_short = d->allow_short;
    a.max_iter = d->max_iter > 0 ? d->max_iter : 100;
    a.tol = d->tol > 0.0 ? d->tol : 1e-10;
    a.return_full = d->return_full_W;
    a.mu = mu; a.sigma = sigma; a.sigma_stride = sigma_stride; a.wp = w_prev;
    a.wout = w_out; a.status = status; a.obj = obj; a.iters = iters;
    a.ws = (double*)ws; a.slab = mv_slab(d->N, d->H);
    const int n = d->N * d->H;
    const int nt = 64 * ((n + 63) / 64);
    if (mv_in_lds(d->N, d->H)) {
        hipLaunchKernelGGL((mv_ipm_kernel<128, false>), dim3(d->B), dim3(nt), mv_lds_bytes(d->N, d->H), stream, a);
    } else {
        if (n > 1024 || mv_small_bytes(d->N, d->H) > 160 * 1024) return KMPC_ERR_UNSUPPORTED;
        if (!ws || ws_bytes < mv_workspace_bytes(d)) return KMPC_ERR_WORKSPACE;
        const int grid = d->B < MV_SLOTS ? d->B : MV_SLOTS;
        hipLaunchKernelGGL((mv_ipm_kernel<1024, true>), dim3(grid), dim3(nt), mv_small_bytes(d->N, d->H), stream, a);
    }
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

int rolling_moments_launch(int B, int T, int N, int lookback, const float* z, int ldz, const float* mean,
                           const float* stdv, const int* ts, double* mu, double* sigma, int* valid,
                           hipStream_t stream) {
    hipLaunchKernelGGL(rolling_moments_kernel, dim3(B), dim3(256), sizeof(double) * N, stream, B, T, N,
                       lookback, z, ldz, mean, stdv, ts, mu, sigma, valid);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

}  // namespace kmpc
