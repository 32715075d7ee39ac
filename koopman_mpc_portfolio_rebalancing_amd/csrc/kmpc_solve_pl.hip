// kmpc_solve_pl.hip — batched MPC solve (replaces solve_mpc_log_utility, mpc.py:27-117) with one
// (period, asset) pair of the window per lane: the period-lane kernel.
//
// Same program and the same Mehrotra predictor-corrector interior point as ipm_kernel /
// ipm_big / oracle/kmpc_oracle.c (epigraph form, exact Newton reduction, Schur matrix on the f64
// MFMA, adaptive refinement, one step length, best-iterate tracking, statuses and fallback), laid
// out for the CDNA4 execution model instead of the per-asset register layout:
//
//   * lane k = t N + i of a workgroup of 64 ceil(H N / 64) <= 1024 threads holds period t of asset
//     i: ~25 doubles of state in registers (the register kernel carries all H periods of an asset
//     per lane, ~660 live dwords, one wave per SIMD with spills); the H N-fold parallelism of a
//     window fills 16 waves at C3 (N = 100, H = 10), 4 per SIMD, so LDS and barrier latency is
//     hidden by the window's other waves; small windows (C1: N = 10, H = 5 -> 50 lanes) pack one
//     window per wave, many per CU.
//   * sums over the assets of a period (1'w_t, m.w_t, sum P, the Schur right-hand side, ...) are
//     segmented wave reduce-scatters (a one-hot slot per period segment, permlane / DPP
//     butterflies) plus one LDS partial per wave and segment: one barrier per reduction point,
//     with the window's scalar sums / maxima riding the same barrier.
//   * the per-asset recursions in t (the tridiagonal LDL^T pivots of Q, the two O(H) sweeps of each
//     Q^{-1} application) run on the asset's owner lane (t = 0) over LDS arrays [t][i]; the other
//     lanes exchange neighbour periods (w_{t-1}, eta_{t+1}, ...) through the same arrays.
//   * the Schur matrix G = I' + Z^T Q^{-1} Z is the GEMM of the semiseparable generators of Q^{-1}
//     (kmpc_solve_big.h) on v_mfma_f64_16x16x4_f64 straight from LDS; wave 0 factors it (L D L^T)
//     and runs the triangular solves.
//
// State never leaves the CU: HBM sees yhat and w_prev once and the outputs once.
#include "kmpc_solve_kernel.h"

namespace kmpc {
namespace pl {

extern __shared__ double pl_lds[];

constexpr int MAXT = 1024;
constexpr int NWMAX = MAXT / WAVE;
constexpr double LR_FLOOR = 1e-14;   // as kmpc_solve_big.h: pi_t stays in the normal range
constexpr int NSCAL = 8;              // block scalars per reduction point
constexpr int NSCR = 4;               // scratch lane arrays (aliased by the generators)

typedef double d4 __attribute__((ext_vector_type(4)));

// dev builds only (make plprof): s_memtime cycles per phase of block 0 of every 64, thread 0
#ifdef KMPC_PL_PROF
__device__ unsigned long long pl_phase[16];
#define PL_CLK_DECL unsigned long long pl_last = __builtin_amdgcn_s_memtime(); const bool pl_on = threadIdx.x == 0 && (blockIdx.x & 63) == 0;
#define PL_PH(k) do { const unsigned long long now_ = __builtin_amdgcn_s_memtime(); if (pl_on) atomicAdd(&pl_phase[k], now_ - pl_last); pl_last = now_; } while (0)
#else
#define PL_CLK_DECL
#define PL_PH(k) (void)0
#endif

// per-period LDS rows written by the period's lane i == 0 (read by wave 0 / at the end)
enum : int { PER_LB6, PER_BRW, PER_BL1, N_PER };

// LDS layout of one window (doubles), computed on the host and passed to the kernel
struct Lay {
    int HN, K3, LDG, NP4, NB, NW, PS;
    int oG, oGid, oQ, oPart, oScal, oPer, oTf, oLR, oIDD, oEP, oGG, oBB, oDQ, oScr;
    int total;   // doubles
};

// S: segments (periods) one wave can touch, rounded to a power of two; a reduction group holds
// 64 / S quantities
__host__ __device__ constexpr int seg_groups(int S, int Q) { return (Q + ((64 / S) < Q ? (64 / S) : Q) - 1) / ((64 / S) < Q ? (64 / S) : Q); }

__host__ inline Lay make_lay(int N, int H, int S) {
    Lay L{};
    L.HN = H * N;
    L.K3 = 3 * H;
    L.LDG = L.K3 | 1;                              // odd row stride: conflict-free row and column reads
    L.NP4 = (N + 3) & ~3;
    if (L.NP4 % 32 == 0) L.NP4 += 4;               // generator rows off the bank period
    L.NB = (L.K3 + 15) / 16;
    L.NW = (L.HN + WAVE - 1) / WAVE;
    L.PS = 64 * seg_groups(S, 4);                  // partial slots per wave (<= 4 quantities)
    int o = 0;
    L.oG = o; o += L.K3 * L.LDG;
    L.oGid = o; o += L.K3;
    L.oQ = o; o += L.K3 + 3;
    L.oPart = o; o += 2 * L.NW * L.PS;
    L.oScal = o; o += 2 * L.NW * NSCAL;
    L.oPer = o; o += N_PER * H;
    L.oTf = o; o += NWMAX / 2 + 2;                 // first period of each wave (ints) + a flag
    L.oLR = o; o += L.HN;
    L.oIDD = o; o += L.HN;
    L.oEP = o; o += L.HN;
    L.oGG = o; o += L.HN;
    L.oBB = o; o += L.HN;
    L.oDQ = o; o += L.HN;
    L.oScr = o;
    const int gen = 2 * L.K3 * L.NP4;             // Lgen, Rgen rows 3t + type (pad rows never read)
    o += (NSCR * L.HN > gen ? NSCR * L.HN : gen);
    L.total = o;
    return L;
}

template <int S, int FL>
struct Ctx : Case<FL> {
    using Case<FL>::hw;
    using Case<FL>::hs;
    using Case<FL>::ht;
    const Lay& L;
    int N, H, k, t, i, lane, wv, seg, buf;
    bool act, own;

    __device__ __forceinline__ Ctx(const Lay& lay, int n, int h) : L(lay), N(n), H(h) {
        k = threadIdx.x;
        lane = k & (WAVE - 1);
        wv = k / WAVE;
        act = k < L.HN;
        t = act ? k / N : 0;
        i = act ? k - t * N : 0;
        own = act && t == 0;
        seg = 0;   // (set once the wave table is in LDS)
        buf = 0;
    }
    __device__ __forceinline__ double* a(int off) const { return pl_lds + off; }
    __device__ __forceinline__ int tf(int w) const { return ((const int*)(pl_lds + L.oTf))[w]; }
    // scratch lane array j (aliased by the generators during the Gram)
    __device__ __forceinline__ double* scr(int j) const { return pl_lds + L.oScr + j * L.HN; }

    // ---- one reduction point: Q period sums (every lane gets its own period's totals), NS block
    // sums and NM block maxima, one barrier ----
    template <int Q, int NS, int NM>
    __device__ __forceinline__ void reduce(double (&pv)[Q], double (&bsum)[NS], double (&bmax)[NM]) {
        static_assert(Q <= 4 && NS + NM <= NSCAL, "reduction slots");
        constexpr int QG = (64 / S) < Q ? (64 / S) : Q;
        constexpr int NG = (Q + QG - 1) / QG;
        double* part = a(L.oPart) + (buf * L.NW + wv) * L.PS;
        static_for<NG>([&](auto gi) {
            constexpr int g = decltype(gi)::value;
            constexpr int q0 = g * QG;
            constexpr int nq = (Q - q0) < QG ? (Q - q0) : QG;
            constexpr int M = pow2_at_least(S * nq);
            double v[M];
            static_for<M>([&](auto ji) {
                constexpr int j = decltype(ji)::value;
                constexpr int q = j / S, sg = j % S;
                if constexpr (q < nq) v[j] = (act && seg == sg) ? pv[q0 + q] : 0.0;
                else v[j] = 0.0;
            });
            const int slot = wave_reduce_scatter<M>(v);
            if ((lane & (WAVE / M - 1)) == 0) part[g * 64 + slot] = v[0];
        });
        double* sc = a(L.oScal) + (buf * L.NW + wv) * NSCAL;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const double x = wave_sum(bsum[j]);
            if (lane == 0) sc[j] = x;
        }
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            const double x = wave_max(bmax[j]);
            if (lane == 0) sc[NS + j] = x;
        }
        __syncthreads();
        if (act) {
#pragma unroll
            for (int q = 0; q < Q; ++q) pv[q] = ptot(q, Q, t, buf);
        }
        const double* s0 = a(L.oScal) + buf * L.NW * NSCAL;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            double x = s0[j];
            for (int w = 1; w < L.NW; ++w) x += s0[w * NSCAL + j];
            bsum[j] = x;
        }
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            double x = s0[NS + j];
            for (int w = 1; w < L.NW; ++w) x = fmax(x, s0[w * NSCAL + NS + j]);
            bmax[j] = x;
        }
        buf ^= 1;
    }
    // period total of quantity q (of a Q-quantity reduction just completed) for period tt: the
    // partials of the waves the period spans, in wave order (identical on every reader)
    // (bf: the buffer of that reduction — after reduce() returns it is buf ^ 1)
    __device__ __forceinline__ double ptot(int q, int Q, int tt, int bf) const {
        const int QG = (64 / S) < Q ? (64 / S) : Q;
        const int g = q / QG, qq = q - g * QG;
        const double* part = a(L.oPart) + bf * L.NW * L.PS + g * 64 + qq * S;
        const int w0 = (tt * N) >> 6, w1 = (tt * N + N - 1) >> 6;
        double s = 0.0;
        for (int w = w0; w <= w1; ++w) s += part[w * L.PS + (tt - tf(w))];
        return s;
    }
};

// ratio tests (as ipm_kernel)
__device__ __forceinline__ double bound(double v, double dv, double amax) { return to_bound(v, dv, amax); }

template <int S, int FL>
__global__ void __launch_bounds__(MAXT) pl_kernel(SolveArgs A, Lay L) {
    Ctx<S, FL> C(L, A.N, A.H);
    C.set_case(!A.allow_short, (A.c > 0.0) || (A.tau > 0.0), A.tau > 0.0);
    const bool hw = C.hw, hs = C.hs, ht = C.ht;
    const int N = A.N, H = A.H, HN = L.HN, K3 = L.K3, LDG = L.LDG;
    const int k = C.k, t = C.t, i = C.i, lane = C.lane, wv = C.wv;
    const bool act = C.act, own = C.own;
    const bool hasn = act && t + 1 < H;     // period t + 1 of this asset exists
    const int b = blockIdx.x;
    double* G = C.a(L.oG);
    double* gid = C.a(L.oGid);
    double* Qs = C.a(L.oQ);
    double* PER = C.a(L.oPer);
    double* LR = C.a(L.oLR);
    double* IDD = C.a(L.oIDD);
    double* EP = C.a(L.oEP);
    double* GG = C.a(L.oGG);
    double* BB = C.a(L.oBB);
    double* DQ = C.a(L.oDQ);
    double* SA = C.scr(0);
    double* SB = C.scr(1);
    double* SC = C.scr(2);
    double* SD = C.scr(3);

    int* flag = (int*)(pl_lds + L.oTf) + NWMAX + 1;   // Schur breakdown
    if (threadIdx.x < NWMAX) ((int*)(pl_lds + L.oTf))[threadIdx.x] = (WAVE * (int)threadIdx.x) / N;
    if (threadIdx.x == 0) *flag = 0;
    __syncthreads();
    C.seg = act ? t - C.tf(wv) : 0;

    const double* wpb = A.wp + (size_t)b * N;
    const float* yh = A.yhat + (size_t)b * HN;
    const int tw = A.return_full ? H : 1;
    double* wout = A.wout + (size_t)b * (A.return_full ? HN : N);
    const double wpi = act ? wpb[i] : 0.0;

    // ---- inputs: m = R - 1, R = np.exp(yhat) in float32 (mpc.py:55), scale, finiteness ----
    const double m = act ? np_expm1_d(yh[k]) : 0.0;
    double sig, nonfin;
    {
        double pz[1] = {0.0};
        double bs0[1] = {0.0};
        double bm[2] = {act ? fabs(m) : 0.0, (act && !(isfinite(m) && isfinite(wpi))) ? 1.0 : 0.0};
        C.template reduce<1, 1, 2>(pz, bs0, bm);
        sig = fmax(bm[0], A.c);
        nonfin = bm[1];
    }
    if (!(sig > 0.0)) sig = 1.0;
    const double isig = 1.0 / sig, irsig = 1.0 / sqrt(sig), cs = A.c / sig, tau = A.tau;

    int status = KMPC_STATUS_SOLVER_ERROR, it = 0;
    double best = 1e300, min_pr = 1e300;
    bool recorded = false;

    if (nonfin == 0.0 && isfinite(A.c) && isfinite(A.tau)) {
        if (A.allow_short && !hs) {
            // no bounds and no turnover terms: unbounded unless every period is flat
            double pv[2] = {m, wpi};
            double z0[1] = {0.0}, z1[1] = {0.0};
            C.template reduce<2, 1, 1>(pv, z0, z1);
            double sp[1] = {0.0};
            double mx[2] = {act ? fabs(m - pv[0] / N) : 0.0, 0.0};
            double swp[1] = {(act && t == 0) ? wpi : 0.0};
            C.template reduce<1, 1, 2>(sp, swp, mx);
            if (mx[0] == 0.0) {
                const double w = swp[0] != 0.0 ? wpi / swp[0] : 1.0 / N;
                if (act && t < tw) wout[k] = w;
                double rwp[1] = {act ? (1.0 + m) * w : 0.0};
                double z2[1] = {0.0}, z3[1] = {0.0};
                C.template reduce<1, 1, 1>(rwp, z2, z3);
                if (act && i == 0) PER[PER_BRW * H + t] = rwp[0];
                if (act && i == 0) PER[PER_BL1 * H + t] = 0.0;   // (c = 0 in this case)
                best = 0.0;
                recorded = true;
                status = KMPC_STATUS_OPTIMAL;
            } else {
                status = KMPC_STATUS_UNBOUNDED;
            }
        } else {
            // ---- initial point ----
            double w, s, l1, l2, l3, z4, l4, nu;
            {
                const double b0 = hw ? fmax(wpi, 0.0) : wpi;
                w = act ? 0.5 * b0 + 0.5 / N : 0.0;
            }
            // w_{t-1}: the previous period's initial point, or w_prev
            {
                const double wprev0 = t ? 0.5 * (hw ? fmax(wpi, 0.0) : wpi) + 0.5 / N : wpi;
                const double d0 = w - wprev0;
                s = (act && hs) ? fabs(d0) + 1.0 / N : 0.0;
            }
            l1 = (act && hw) ? 1.0 : 0.0;
            l2 = l3 = (act && hs) ? 1.0 : 0.0;
            {
                double pv[1] = {s};
                double z0[1] = {0.0}, z1[1] = {0.0};
                C.template reduce<1, 1, 1>(pv, z0, z1);
                z4 = ht ? fmax(tau - pv[0], 0.5 * tau) : 1.0;
                l4 = ht ? 1.0 : 0.0;
                nu = 0.0;
            }
            const int ncon = (hw ? HN : 0) + (hs ? 2 * HN : 0) + (ht ? H : 0);
            const double inv_ncon = 1.0 / (ncon > 0 ? ncon : 1);
            const bool lead = act && i == 0;   // the lane that speaks for its period in block sums

            PL_CLK_DECL
            for (it = 0; it < A.max_iter; ++it) {
                PL_PH(0);
                // ================= residuals =================
                if (act) { SA[k] = w; SB[k] = l3 - l2; }
                double mw, sw, ss;
                {
                    double pv[3] = {m * w, w, s};
                    double z0[1] = {0.0}, z1[1] = {0.0};
                    C.template reduce<3, 1, 1>(pv, z0, z1);
                    mw = pv[0]; sw = pv[1]; ss = pv[2];
                }
                const double wprev = t ? SA[k - N] : wpi;
                const double etan = hasn ? SB[k + N] : 0.0;
                const double d = w - wprev;
                const double den = 1.0 + mw, iden = 1.0 / den;
                const double rp = sw - 1.0;
                const double rg4 = ht ? tau - ss - z4 : 0.0;
                double rc4 = ht ? z4 * l4 : 0.0;
                const double iz4 = 1.0 / z4;
                const double al = m * iden * irsig;   // alpha_t (Z's a-column entry)
                double rdw = -m * iden * isig - (l1 + (l3 - l2) - etan) + nu;
                double rds = hs ? cs - (l2 + l3 - l4) : 0.0;
                double rc1 = hw ? w * l1 : 0.0;
                double rc2 = hs ? (s - d) * l2 : 0.0;
                double rc3 = hs ? (s + d) * l3 : 0.0;
                double mu, mu_assets, rd, pr;
                double l1n;
                bool dom;
                {
                    double pv[1] = {act ? fabs(d) : 0.0};
                    // asset complementarity (c0 of the step polynomial) and the cap terms, counted
                    // once per period by its lead lane
                    double bsum[2] = {act ? rc1 + rc2 + rc3 : 0.0, lead ? rc4 : 0.0};
                    double bmax[3] = {act ? fmax(fabs(rdw), fabs(rds)) : 0.0, act ? fmax(fabs(rp), fabs(rg4)) : 0.0,
                                      (act && !(den > 0.0)) ? 1.0 : 0.0};
                    if (!act) { rdw = rds = rc1 = rc2 = rc3 = 0.0; }
                    C.template reduce<1, 2, 3>(pv, bsum, bmax);
                    l1n = pv[0];
                    mu_assets = bsum[0];
                    mu = bsum[0] + bsum[1];
                    rd = bmax[0];
                    pr = bmax[1];
                    dom = bmax[2] == 0.0;
                }
                mu *= inv_ncon;
                const double merit = fmax(mu, fmax(rd, pr));
                min_pr = fmin(min_pr, pr);
                if (A.trace && b == 0 && k == 0) {
                    A.trace[4 * it + 0] = mu; A.trace[4 * it + 1] = rd; A.trace[4 * it + 2] = pr;
                }
                if (!dom || !isfinite(merit)) break;
                if (merit < best) {
                    best = merit;
                    recorded = true;
                    if (act && t < tw) wout[k] = w;
                    if (lead) {
                        PER[PER_BRW * H + t] = sw + mw;   // sum_i R w = sum w + sum (R - 1) w
                        PER[PER_BL1 * H + t] = l1n;
                    }
                } else if (best < 1e-6 && merit > 1e4 * best) {
                    break;   // numerical breakdown after convergence: keep the best iterate
                }
                if (mu < A.tol && rd < 10.0 * A.tol && pr < 10.0 * A.tol) break;

                PL_PH(1);
                // ================= factor =================
                // slack reciprocals, s-elimination coefficients, LDL^T inputs of Q
                const double iw = (act && hw) ? rcp_nr(w) : 0.0;
                const double iz2 = (act && hs) ? rcp_nr(s - d) : 0.0;
                const double iz3 = (act && hs) ? rcp_nr(s + d) : 0.0;
                double P = 0.0, bma = 0.0;
                if (act && hs) {
                    const double a2 = l2 * iz2, b3 = l3 * iz3;
                    P = rcp_nr(a2 + b3);
                    bma = b3 - a2;
                    SB[k] = 4.0 * a2 * b3 * P;       // E
                } else if (act) {
                    SB[k] = 0.0;
                }
                if (act) SA[k] = hw ? l1 * iw : 0.0;  // W1
                double rho, sr;
                {
                    double pv[1] = {P};
                    double z0[1] = {0.0}, z1[1] = {0.0};
                    C.template reduce<1, 1, 1>(pv, z0, z1);
                    const double ga = ht ? l4 * iz4 : 0.0;
                    rho = ht ? ga / (1.0 + ga * pv[0]) : 0.0;
                    sr = sqrt(rho);
                }
                const double BP = bma * P;
                const double ep = ht ? sr * BP : 0.0;   // eps_t (Z's v-column entry)
                if (act) EP[k] = ep;
                // owner: tridiagonal LDL^T pivots (cancellation-free recursion), diagonal of Q^{-1},
                // centred prefix products of Lr -> the semiseparable generators g = 1 / pi, b = dq pi
                bool bad = false;
                if (own) {
                    double pi = SA[i] + SB[i], lr = 0.0;
                    for (int tt = 0; tt < H; ++tt) {
                        const int kk = tt * N + i;
                        const bool nx = tt + 1 < H;
                        const double En = nx ? SB[kk + N] : 0.0;
                        const double Dd = pi + En;
                        bad = bad || !(Dd > 0.0) || !(Dd < 1e300);
                        const double iDd = rcp_nr(fmax(Dd, 1e-300));
                        IDD[kk] = iDd;
                        LR[kk] = lr;
                        if (nx) {
                            lr = En * iDd;
                            pi = SA[kk + N] + lr * pi;
                        }
                    }
                    double dqn = 0.0, lrn = 0.0, pp = 1.0;
                    for (int tt = H - 1; tt >= 0; --tt) {
                        const int kk = tt * N + i;
                        const double dq = IDD[kk] + lrn * lrn * dqn;
                        DQ[kk] = dq;
                        dqn = dq;
                        lrn = LR[kk];
                        if (tt) pp *= fmax(lrn, LR_FLOOR);
                    }
                    int e = 0;
                    frexp(pp, &e);
                    const double cen = ldexp(1.0, -(e / 2));
                    double pr2 = 1.0;
                    for (int tt = 0; tt < H; ++tt) {
                        const int kk = tt * N + i;
                        if (tt) pr2 *= fmax(LR[kk], LR_FLOOR);
                        const double pt = pr2 * cen;
                        GG[kk] = 1.0 / pt;
                        BB[kk] = DQ[kk] * pt;
                    }
                }
                PL_PH(2);
                {
                    double z0[1] = {0.0}, z1[1] = {0.0};
                    double bmx[1] = {bad ? 1.0 : 0.0};
                    C.template reduce<1, 1, 1>(z0, z1, bmx);
                    bad = bmx[0] != 0.0;
                }
                if (bad) break;
                // generators (rows 3t + type of Lgen / Rgen; types v, a, 1) and the (v_t, v_t) entries
                double* LG = C.scr(0);
                double* RG = LG + K3 * L.NP4;
                {
                    double vv = 0.0;
                    if (act) {
                        const double g = GG[k], bb = BB[k], dq = DQ[k];
                        const double gm = t ? GG[k - N] : 0.0, bm = t ? BB[k - N] : 0.0;
                        const double dqm = t ? DQ[k - N] : 0.0, lr = LR[k];
                        const int r0 = 3 * t * L.NP4 + i;
                        LG[r0] = ep * (g - gm);
                        LG[r0 + L.NP4] = al * g;
                        LG[r0 + 2 * L.NP4] = g;
                        RG[r0] = ep * (bb - bm);
                        RG[r0 + L.NP4] = al * bb;
                        RG[r0 + 2 * L.NP4] = bb;
                        vv = t ? ep * ep * (dq - 2.0 * lr * dq + dqm) : ep * ep * dq;
                    }
                    double pv[1] = {vv};
                    double z0[1] = {0.0}, z1[1] = {0.0};
                    C.template reduce<1, 1, 1>(pv, z0, z1);
                    if (lead) G[(3 * t) * LDG + 3 * t] = pv[0];
                }
                PL_PH(3);
                // G (lower triangle, stored at [l][j], j <= l) += Lgen^T Rgen: one 16x16 tile per wave
                {
                    const int NB = L.NB, ntile = NB * (NB + 1) / 2;
                    for (int q = wv; q < ntile; q += L.NW) {
                        int I = 0, J = 0, rem = q;
                        for (int bi = 0; bi < NB; ++bi) {
                            const int n = NB - bi;
                            if (rem < n) { I = bi; J = bi + rem; break; }
                            rem -= n;
                        }
                        const int ra = 16 * I + (lane & 15), rb = 16 * J + (lane & 15);
                        const bool va = ra < K3, vb = rb < K3;
                        const double* pa = LG + ra * L.NP4 + (lane >> 4);
                        const double* pb = RG + rb * L.NP4 + (lane >> 4);
                        d4 acc = {0.0, 0.0, 0.0, 0.0};
                        for (int k0 = 0; k0 < N; k0 += 4) {
                            const bool kin = k0 + (lane >> 4) < N;
                            const double x = (va && kin) ? pa[k0] : 0.0;
                            const double y = (vb && kin) ? pb[k0] : 0.0;
                            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int j = 16 * I + (lane >> 4) + 4 * r, l = 16 * J + (lane & 15);
                            if (j < K3 && l < K3) {
                                const int tj = j / 3, tyj = j - 3 * tj, tl = l / 3, tyl = l - 3 * tl;
                                const bool use = tj < tl || (tj == tl && tyj <= tyl && !(tyj == 0 && tyl == 0));
                                if (use) G[l * LDG + j] = acc[r];
                            }
                        }
                    }
                }
                __syncthreads();
                PL_PH(4);
                // wave 0: G + I' = L D L^T (row per lane, right-looking; unused v rows -> identity)
                if (wv == 0) {
                    const int r = lane;
                    const int ty = r % 3;
                    const bool rused = r < K3 && (ty != 0 || ht);
                    if (r < K3) {
                        for (int c = 0; c <= r; ++c) {
                            const bool cused = (c % 3) != 0 || ht;
                            double v = (rused && cused) ? G[r * LDG + c] : 0.0;
                            if (c == r) v += (ty != 2 || !rused) ? 1.0 : 0.0;
                            G[r * LDG + c] = v;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    bool badg = false;
                    for (int j = 0; j < K3; ++j) {
                        const double dj = G[j * LDG + j];
                        badg = badg || !(dj > 0.0) || !(dj < 1e300);
                        const double id = rcp_nr(fmax(dj, 1e-300));
                        if (r == j) gid[j] = id;
                        const bool below = r > j && r < K3;
                        const double l = below ? G[r * LDG + j] * id : 0.0;
                        __builtin_amdgcn_wave_barrier();
                        if (below)
                            for (int c = j + 1; c <= r; ++c) G[r * LDG + c] = fma(-l, G[c * LDG + j], G[r * LDG + c]);
                        __builtin_amdgcn_wave_barrier();
                        if (below) G[r * LDG + j] = l;
                        __builtin_amdgcn_wave_barrier();
                    }
                    if (badg && r == 0) *flag = 1;
                }
                __syncthreads();
                PL_PH(5);
                if (*flag) break;

                // ================= Newton: predictor (pass 0) and corrector (pass 1) =================
                double dw = 0.0, ds = 0.0, dd = 0.0, dnu = 0.0, dz4 = 0.0, dl4 = 0.0, mdw = 0.0;
                double step = 0.0;
                double b5 = ht ? -rc4 - l4 * rg4 : 0.0;
                double b6 = -rp;
                for (int pass = 0; pass < 2; ++pass) {
                    const int n_ref = (pass == 0 || mu > REFINE_MU) ? 0 : A.n_refine;
                    double bn = 0.0;   // ||b||_inf (only when refinement may run)
                    if (n_ref > 0) {
                        double z0[1] = {0.0}, z1[1] = {0.0};
                        double bm[1] = {act ? fmax(fmax(fmax(fabs(rdw), fabs(rds)), fmax(fabs(rc1), fabs(rc2))),
                                                   fmax(fabs(rc3), fmax(fabs(b5), fabs(b6)))) : 0.0};
                        C.template reduce<1, 1, 1>(z0, z1, bm);
                        bn = bm[0];
                    }
                    double lb5 = b5, lb6 = b6;
                    // right-hand side rows (1), (2) of this solve; (3)-(5) are -rc when with_c
                    double r0 = -rdw, r1 = -rds;
                    double sdw = 0.0, sds = 0.0;
                    for (int rr = 0;; ++rr) {
                        const bool with_c = rr == 0;
                        // ---- A: complementarity rows folded in; rhs_s; sum_i P rhs_s ----
                        double p1 = 0.0, p2 = 0.0, p3 = 0.0;
                        if (with_c) {
                            p1 = hw ? -rc1 * iw : 0.0;
                            p2 = hs ? -rc2 * iz2 : 0.0;
                            p3 = hs ? -rc3 * iz3 : 0.0;
                        }
                        const double qv = p3 - p2;
                        if (act) SA[k] = qv;
                        const double rhss = (act && hs) ? r1 + p2 + p3 - (ht ? lb5 * iz4 : 0.0) : 0.0;
                        double px;
                        {
                            double pv[1] = {P * rhss};
                            double z0[1] = {0.0}, z1[1] = {0.0};
                            C.template reduce<1, 1, 1>(pv, z0, z1);
                            px = pv[0];
                        }
                        PL_PH(6);
                        // ---- B: rhs_w (with the s elimination), x = Q^{-1} rhs_w (owner sweeps) ----
                        {
                            const double pn = hasn ? SA[k + N] : 0.0;
                            const double rhsw0 = act ? r0 + p1 + qv - pn : 0.0;
                            const double g = hs ? BP * (rhss - rho * px) : 0.0;
                            if (act) { SB[k] = rhsw0; SC[k] = g; }
                        }
                        __syncthreads();
                        if (own) {
                            double y = 0.0;
                            for (int tt = 0; tt < H; ++tt) {
                                const int kk = tt * N + i;
                                const double x = SB[kk] - SC[kk] + (tt + 1 < H ? SC[kk + N] : 0.0);
                                y = x + LR[kk] * y;
                                SC[kk] = y;
                            }
                            double x = 0.0, lrn = 0.0;
                            for (int tt = H - 1; tt >= 0; --tt) {
                                const int kk = tt * N + i;
                                x = SC[kk] * IDD[kk] + lrn * x;
                                SB[kk] = x;
                                lrn = LR[kk];
                            }
                        }
                        __syncthreads();
                        PL_PH(7);
                        // ---- C: Schur right-hand side Z^T x (v, a, 1 rows per period) ----
                        const double xv = act ? SB[k] : 0.0;
                        {
                            const double xm = (act && t) ? SB[k - N] : 0.0;
                            double pv[3] = {ep * (xv - xm), al * xv, xv};
                            double z0[1] = {0.0}, z1[1] = {0.0};
                            if (lead) PER[PER_LB6 * H + t] = lb6;
                            C.template reduce<3, 1, 1>(pv, z0, z1);
                        }
                        PL_PH(8);
                        // wave 0: q = G^{-1} (rhs - [0; 0; lb6]) by forward / back substitution
                        if (wv == 0) {
                            double x = 0.0;
                            if (lane < K3) {
                                const int tt = lane / 3, ty = lane - 3 * tt;
                                x = C.ptot(ty, 3, tt, C.buf ^ 1);
                                if (ty == 2) x -= PER[PER_LB6 * H + tt];
                            }
                            const int lr = lane < K3 ? lane : 0;
                            for (int j = 0; j + 1 < K3; ++j) {
                                const double yj = bcast(x, j);
                                if (lane > j) x = fma(-G[lr * LDG + j], yj, x);
                            }
                            x *= gid[lr];
                            for (int j = K3 - 1; j > 0; --j) {
                                const double qj = bcast(x, j);
                                if (lane < j) x = fma(-G[j * LDG + lr], qj, x);
                            }
                            if (lane < K3) Qs[lane] = x;
                            if (lane < 3) Qs[K3 + lane] = 0.0;
                        }
                        __syncthreads();
                        PL_PH(9);
                        // ---- D: Q^{-1} Z q (owner sweeps), dw = x - Q^{-1} Z q ----
                        const double qa = Qs[3 * t + 1], q1 = Qs[3 * t + 2], qvv = Qs[3 * t], qvn = Qs[3 * t + 3];
                        {
                            const double epn = hasn ? EP[k + N] : 0.0;
                            if (act) SA[k] = al * qa + q1 + ep * qvv - epn * qvn;
                        }
                        __syncthreads();
                        if (own) {
                            double y = 0.0;
                            for (int tt = 0; tt < H; ++tt) {
                                const int kk = tt * N + i;
                                y = SA[kk] + LR[kk] * y;
                                SA[kk] = y;
                            }
                            double x = 0.0, lrn = 0.0;
                            for (int tt = H - 1; tt >= 0; --tt) {
                                const int kk = tt * N + i;
                                x = SA[kk] * IDD[kk] + lrn * x;
                                SA[kk] = SB[kk] - x;        // dw_t
                                lrn = LR[kk];
                            }
                        }
                        __syncthreads();
                        PL_PH(10);
                        // ---- E: ds = (diag(alpha + beta) + gamma 1 1')^{-1} (rhs_s - bma dd) ----
                        const double dwc = act ? SA[k] : 0.0;
                        const double ddc = act ? dwc - (t ? SA[k - N] : 0.0) : 0.0;
                        const double bs = hs ? rhss - bma * ddc : 0.0;
                        double dsc;
                        {
                            double pv[1] = {P * bs};
                            double z0[1] = {0.0}, z1[1] = {0.0};
                            C.template reduce<1, 1, 1>(pv, z0, z1);
                            dsc = (act && hs) ? P * (bs - rho * pv[0]) : 0.0;
                        }
                        if (rr == 0) { dw = dwc; ds = dsc; dnu = q1; }
                        else { dw += dwc; ds += dsc; dnu += q1; }
                        dd = act ? (rr == 0 ? ddc : dd + ddc) : 0.0;
                        // multipliers of the direction (complementarity rows, targets rc)
                        const double dl1 = hw ? (-rc1 - l1 * dw) * iw : 0.0;
                        const double dl2 = hs ? (-rc2 - l2 * (ds - dd)) * iz2 : 0.0;
                        const double dl3 = hs ? (-rc3 - l3 * (ds + dd)) * iz3 : 0.0;
                        // period sums for dz4 / dl4, the refinement residual and the step (m.dw)
                        if (act) SD[k] = dl3 - dl2;
                        {
                            double pv[4] = {act ? ds : 0.0, act ? al * dw : 0.0, act ? dw : 0.0, act ? m * dw : 0.0};
                            double z0[1] = {0.0}, z1[1] = {0.0};
                            C.template reduce<4, 1, 1>(pv, z0, z1);
                            sds = pv[0];
                            sdw = pv[2];
                            mdw = pv[3];
                            dl4 = ht ? (b5 + l4 * sds) * iz4 : 0.0;
                            if (rr >= n_ref) break;
                            // residual of rows (1), (2), (7); rows (3)-(6) hold by construction
                            const double adw = pv[1];
                            const double nd = hasn ? SD[k + N] : 0.0;
                            r0 = act ? -rdw - (al * adw - (dl1 + (dl3 - dl2) - nd) + dnu) : 0.0;
                            r1 = (act && hs) ? -rds + (dl2 + dl3 - dl4) : 0.0;
                            double zz[1] = {0.0}, zs[1] = {0.0};
                            double rn[1] = {act ? fmax(fmax(fabs(r0), fabs(r1)), lead ? fabs(b6 - sdw) : 0.0) : 0.0};
                            C.template reduce<1, 1, 1>(zz, zs, rn);
                            if (rn[0] <= REFINE_RTOL * bn) break;
                            lb5 = 0.0;             // row (6) residual is identically 0
                            lb6 = b6 - sdw;
                        }
                    }
                    PL_PH(11);
                    dz4 = ht ? -sds + rg4 : 0.0;
                    // ---- step length and the complementarity along the direction ----
                    double amax, c1 = 0.0, c2 = 0.0;
                    {
                        const double dl1 = hw ? (-rc1 - l1 * dw) * iw : 0.0;
                        const double dl2 = hs ? (-rc2 - l2 * (ds - dd)) * iz2 : 0.0;
                        const double dl3 = hs ? (-rc3 - l3 * (ds + dd)) * iz3 : 0.0;
                        double a = 1e300, qx = 0.0;
                        if (act) {
                            if (hw) {
                                qx = fmax(qx, -dw * iw);
                                a = bound(l1, dl1, a);
                                c1 += w * dl1 + l1 * dw;
                                c2 += dw * dl1;
                            }
                            if (hs) {
                                const double x2 = s - d, dx2 = ds - dd, x3 = s + d, dx3 = ds + dd;
                                qx = fmax(qx, fmax(-dx2 * iz2, -dx3 * iz3));
                                a = bound(l2, dl2, a);
                                a = bound(l3, dl3, a);
                                c1 += x2 * dl2 + l2 * dx2 + x3 * dl3 + l3 * dx3;
                                c2 += dx2 * dl2 + dx3 * dl3;
                            }
                            if (qx > 0.0) a = fmin(a, rcp_nr(qx));
                            a = bound(den, mdw, a);
                            if (ht) { a = bound(z4, dz4, a); a = bound(l4, dl4, a); }
                        }
                        double pz[1] = {0.0};
                        double sums[2] = {c1, c2};
                        double mx[1] = {-a};
                        C.template reduce<1, 2, 1>(pz, sums, mx);
                        c1 = sums[0];
                        c2 = sums[1];
                        amax = -mx[0];
                    }
                    if (pass == 1) { step = fmin(1.0, 0.99 * amax); break; }
                    const double ap = fmin(1.0, amax);
                    // complementarity at the predictor step: assets' c0 + ap c1 + ap^2 c2, plus the
                    // cap terms of every period (one lane per period contributes)
                    double comp;
                    {
                        double pz[1] = {0.0};
                        double sum4[1] = {(lead && ht) ? (z4 + ap * dz4) * (l4 + ap * dl4) : 0.0};
                        double z1[1] = {0.0};
                        C.template reduce<1, 1, 1>(pz, sum4, z1);
                        comp = mu_assets + ap * (c1 + ap * c2) + sum4[0];
                    }
                    double sg = comp * inv_ncon / mu;
                    sg = sg * sg * sg;
                    const double smu = sg * mu;
                    // corrector targets rc + dx_aff dl_aff - sigma mu
                    {
                        const double dl1 = hw ? (-rc1 - l1 * dw) * iw : 0.0;
                        const double dl2 = hs ? (-rc2 - l2 * (ds - dd)) * iz2 : 0.0;
                        const double dl3 = hs ? (-rc3 - l3 * (ds + dd)) * iz3 : 0.0;
                        if (act) {
                            if (hw) rc1 += dw * dl1 - smu;
                            if (hs) {
                                rc2 += (ds - dd) * dl2 - smu;
                                rc3 += (ds + dd) * dl3 - smu;
                            }
                        }
                    }
                    if (ht) rc4 += dz4 * dl4 - smu;
                    b5 = ht ? -rc4 - l4 * rg4 : 0.0;
                    b6 = -rp;
                }
                PL_PH(12);
                if (A.trace && b == 0 && k == 0) A.trace[4 * it + 3] = step;
                // ================= update =================
                {
                    const double dl1 = hw ? (-rc1 - l1 * dw) * iw : 0.0;
                    const double dl2 = hs ? (-rc2 - l2 * (ds - dd)) * iz2 : 0.0;
                    const double dl3 = hs ? (-rc3 - l3 * (ds + dd)) * iz3 : 0.0;
                    if (act) {
                        l1 += step * dl1;
                        l2 += step * dl2;
                        l3 += step * dl3;
                        w += step * dw;
                        s += step * ds;
                    }
                    z4 += step * dz4;
                    l4 += step * dl4;
                    nu += step * dnu;
                }
            }
            if (best <= 1e-7) status = KMPC_STATUS_OPTIMAL;
            else if (best <= 1e-4) status = KMPC_STATUS_OPTIMAL_INACCURATE;
            else if (min_pr > 1e-6) status = KMPC_STATUS_INFEASIBLE;   // primal residual never closed
            else status = KMPC_STATUS_SOLVER_ERROR;
        }
    }
    __syncthreads();
    const bool ok = status == KMPC_STATUS_OPTIMAL || status == KMPC_STATUS_OPTIMAL_INACCURATE;
    if (!ok && act && t < tw) wout[k] = wpi;   // mpc.py:113-115
    if (k == 0) {
        double f = __builtin_nan("");
        if (ok && recorded) {
            // problem.value (mpc.py:103) at the best iterate: sum_t log(R_t . w_t) - c ||w_t - w_{t-1}||_1
            f = 0.0;
            for (int tt = 0; tt < H; ++tt) f += log(PER[PER_BRW * H + tt]) - A.c * PER[PER_BL1 * H + tt];
        }
        A.obj[b] = ok ? f : __builtin_nan("");
        A.status[b] = status;
        if (A.iters) A.iters[b] = it;
    }
}

template <int S>
int launch_s(const SolveArgs& a, hipStream_t stream) {
    const Lay L = make_lay(a.N, a.H, S);
    const size_t lds = sizeof(double) * (size_t)L.total;
    if (lds > 160 * 1024) return KMPC_ERR_UNSUPPORTED;
    const int nt = WAVE * L.NW;
    const int fl = case_of(!a.allow_short, a.c > 0.0 || a.tau > 0.0, a.tau > 0.0);
    if (fl == 7)
        hipLaunchKernelGGL((pl_kernel<S, 7>), dim3(a.B), dim3(nt), lds, stream, a, L);
    else
        hipLaunchKernelGGL((pl_kernel<S, -1>), dim3(a.B), dim3(nt), lds, stream, a, L);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

}  // namespace pl

#ifdef KMPC_PL_PROF
extern "C" int kmpc_debug_pl_phases(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pl::pl_phase), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pl::pl_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

bool pl_supported(const SolveArgs& a) { return (long)a.H * a.N <= pl::MAXT && 3 * a.H <= 63; }

int pl_launch(const SolveArgs& a, hipStream_t stream) {
    if (!pl_supported(a)) return KMPC_ERR_UNSUPPORTED;
    // periods one wave can touch: floor(63 / N) + 2 at most, and never more than H
    int segs = 63 / a.N + 2;
    if (segs > a.H) segs = a.H;
    if (segs <= 2) return pl::launch_s<2>(a, stream);
    if (segs <= 4) return pl::launch_s<4>(a, stream);
    if (segs <= 8) return pl::launch_s<8>(a, stream);
    if (segs <= 16) return pl::launch_s<16>(a, stream);
    return pl::launch_s<32>(a, stream);
}

}  // namespace kmpc
