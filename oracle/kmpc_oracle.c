/*
 * kmpc_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline), never the
 * product. Built twice by oracle/Makefile:
 *   libkmpc_oracle.so     real = double       (CPU baseline timing, "port")
 *   libkmpc_oracle_ld.so  real = long double  (golden fixtures / parity reference)
 *
 * CPU restatement of the reference's per-window MPC solve:
 *
 *   solve_mpc_log_utility(current_weights, predicted_log_returns, config)   mpc.py:27-117
 *     R = np.exp(yhat)  on the float32 yhat (backtest.py:121), numpy's float32 exp,   mpc.py:55
 *                       promoted to float64 by cvxpy (np_expf below)
 *     maximize  sum_t log(w_t . R_t) - c * sum_t ||w_t - w_{t-1}||_1         mpc.py:66-103
 *     s.t.      sum(w_t) == 1                                                mpc.py:83
 *               w_t >= 0                     if not allow_short              mpc.py:85-86
 *               ||w_t - w_{t-1}||_1 <= tau   if tau > 0 (t=0: w_{-1}=w_prev) mpc.py:94-100
 *     status not in {optimal, optimal_inaccurate} -> W = tile(w_prev), value None   mpc.py:113-115
 *
 * The reference hands this program to cvxpy 1.7.5 -> SCS 3.2.9 (ECOS is not in its lock file, so
 * the ECOS call raises SolverError and the SCS fallback runs, mpc.py:107-111). Neither is importable
 * here, so the oracle restates the PROGRAM (its optimum), not SCS's iteration: a Mehrotra
 * predictor-corrector primal-dual interior-point method on the epigraph form
 *
 *   min  -(1/sig) sum_t log(1 + m_t.w_t) + (c/sig) sum_t 1's_t      m = (double)R - 1 (exact)
 *   s.t. w >= 0,  s_t - d_t >= 0,  s_t + d_t >= 0,  tau - 1's_t >= 0,  1'w_t = 1,
 *        d_t = w_t - w_{t-1},  w_{-1} = w_prev,
 *
 * (log(1 + m.w) == log(R.w) on 1'w = 1; sig = max(|m|, c) only rescales the objective).
 * w and s are kept strictly interior (their slacks are never stored); the tau slack is explicit.
 * Each Newton system is reduced exactly:
 *   - complementarity rows eliminate the multipliers,
 *   - s is eliminated per period (diagonal + rank one -> E, e, rho),
 *   - the w-system is Q + U U^T with Q = diag(W1) + D^T E D a per-asset tridiagonal in t (LDL^T by
 *     the cancellation-free recursion pi_t = W1_t + E_t pi_{t-1} / (pi_{t-1} + E_t)) and
 *     U = [a_t | sqrt(rho_t) D^T e_t]; the budget rows 1'w_t = 1 join U in a 3H x 3H Schur system,
 *   - iterative refinement against the unreduced Newton system, adaptive: refine while
 *     ||r||_inf > 1e-7 ||b||_inf, at most n_refine (3) steps. Near the optimum the Schur system
 *     is as ill-conditioned as 1/mu, and a fixed 1-2 steps leave objective errors ~1e-6.
 *
 * Parity of this oracle is pinned in tests/test_oracle.py against the exact optima of the
 * reference's test_mpc cases (reference tests/test_mpc.py:25-55), an independent dense-KKT IPM and
 * scipy SLSQP (oracle/dense_ipm.py), and KKT certificates.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef KMPC_REAL_LONG
typedef long double real;
#define R_(x) x##L
#define RSQRT sqrtl
#define RFABS fabsl
#define RFMAX fmaxl
#define RFMIN fminl
#define API(name) name##_ld
#elif defined(KMPC_REAL_FLOAT)
/* float32 build: only tools/dev/f32phase.c (the mixed-precision measurement of DESIGN §3.2) */
typedef float real;
#define R_(x) x##f
#define RSQRT sqrtf
#define RFABS fabsf
#define RFMAX fmaxf
#define RFMIN fminf
#define API(name) name##_f
#else
typedef double real;
#define R_(x) x
#define RSQRT sqrt
#define RFABS fabs
#define RFMAX fmax
#define RFMIN fmin
#define API(name) name
#endif
#define RISFIN(x) isfinite(x)
#define KMPC_INIT_MULT R_(0.5)   /* the initial point's multipliers, as the kernels' KMPC_INIT_MULT */
#define KMPC_SIGMA_CAP R_(0.2)   /* as the kernels' (kmpc_solve_kernel.h) */
#define KMPC_STEP_NOSHORT R_(0.995)

/*
 * numpy's float32 exp (numpy 2.x, x86-64 AVX2 / AVX512F: simd_exp_f32 in
 * numpy/_core/src/umath/loops_exponent_log.dispatch.c.src) — the function that produces the
 * reference's R at mpc.py:55 and its realized returns np.exp(r) - 1 at backtest.py:188. Restated
 * from its published algorithm: saturation at x >= 88.7228 (+inf) and x <= -103.972 (0);
 * k = rint(x log2 e) by the 1.5*2^23 magic round in float32; Cody-Waite reduction
 * r = x - k ln2 (ln2 split high/low) in float32 FMAs; exp(r) ~ P5(r)/Q2(r) (Remez), Horner in
 * float32 FMAs and one correctly rounded float32 division; scaling by 2^k. Bit-identical to np.exp
 * on every finite float32 with |x| < 100 (checked exhaustively in the build container;
 * tests/test_oracle.py::test_np_expf_restatement_is_bit_exact re-checks 2^24 of them). The
 * volatile temporaries keep the compiler from contracting x*log2e + magic into an FMA.
 */
static float np_expf(float x) {
    if (x != x) return x;
    if (x >= 88.72283935546875f) return INFINITY;
    if (x <= -103.97208404541015625f) return 0.0f;
    volatile float q0 = x * 1.442695040888963407359924681001892137f;
    volatile float q1 = q0 + 0x1.8p+23f;
    const float q = q1 - 0x1.8p+23f;
    float r = fmaf(q, -6.93145752e-1f, x);
    r = fmaf(q, -1.42860677e-6f, r);
    r = fmaf(q, 0.0f, r);
    float p = fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    p = fmaf(p, r, 5.114512081637298353406e-02f);
    p = fmaf(p, r, 2.473615434895520810817e-01f);
    p = fmaf(p, r, 7.257664613233124478488e-01f);
    p = fmaf(p, r, 9.999999999980870924916e-01f);
    float d = fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    d = fmaf(d, r, 1.0f);
    volatile float e = p / d;
    return ldexpf(e, (int)q);
}

void kmpc_oracle_gross_returns(long n, const float* y, float* R) {
    for (long k = 0; k < n; ++k) R[k] = np_expf(y[k]);
}

/* a period whose gross returns sum below this is solved on R / sum(R) (see kmpc_oracle_solve) */
#define KMPC_TINY_PERIOD 0x1p-16

#define ST_OPTIMAL 0
#define ST_INACCURATE 1
#define ST_INFEASIBLE 2
#define ST_UNBOUNDED 3
#define ST_ERROR 4

/* per-problem workspace: HN arrays are [t*N + i], H arrays are [t], K = 3H */
typedef struct {
    int N, H, K, hw, hs, ht, n_refine;
    real c, tau, sig;
    /* state */
    real *wp, *m, *w, *s, *l1, *l2, *l3, *z4, *l4, *nu, *wbest;
    /* per-iteration quantities */
    real *a, *rdw, *rds, *den, *rp, *rg4;
    real *W1, *P, *E, *e, *bma, *Dd, *Lr, *SP, *rho, *sr, *ga;
    real *G, *Gc, *Yrow, *zr, *bsm, *qv;
    /* direction and solve scratch */
    real *dw, *ds, *dl1, *dl2, *dl3, *dl4, *dnu, *dd, *dz4;
    real *rc1, *rc2, *rc3, *rc4;
    real *b[7], *r[7], *sv[7];       /* rhs / residual / saved solution, blocks as in lsolve */
    real *rhsw, *rhss, *g, *yr, *xr, *tmp;
    real *pool;
} ws_t;

static int ws_init(ws_t* W, int N, int H) {
    size_t HN = (size_t)H * N, K = 3 * (size_t)H;
    size_t n_hn = 40 + 15, n_h = 30;
    size_t total = n_hn * HN + n_h * H + 2 * K * K + 5 * K + K + 16;
    W->pool = (real*)calloc(total, sizeof(real));
    if (!W->pool) return -1;
    real* p = W->pool;
#define TAKE(ptr, n) do { (ptr) = p; p += (n); } while (0)
    TAKE(W->wp, N); TAKE(W->m, HN); TAKE(W->w, HN); TAKE(W->s, HN); TAKE(W->l1, HN);
    TAKE(W->l2, HN); TAKE(W->l3, HN); TAKE(W->wbest, HN); TAKE(W->a, HN); TAKE(W->rdw, HN);
    TAKE(W->rds, HN);
    TAKE(W->W1, HN); TAKE(W->P, HN); TAKE(W->E, HN); TAKE(W->e, HN); TAKE(W->bma, HN);
    TAKE(W->Dd, HN); TAKE(W->Lr, HN); TAKE(W->dw, HN); TAKE(W->ds, HN);
    TAKE(W->dl1, HN); TAKE(W->dl2, HN); TAKE(W->dl3, HN); TAKE(W->dd, HN); TAKE(W->rc1, HN);
    TAKE(W->rc2, HN); TAKE(W->rc3, HN); TAKE(W->rhsw, HN); TAKE(W->rhss, HN);
    TAKE(W->g, HN); TAKE(W->yr, HN); TAKE(W->xr, HN);
    TAKE(W->tmp, HN + K);
    for (int j = 0; j < 5; ++j) { TAKE(W->b[j], HN); TAKE(W->r[j], HN); TAKE(W->sv[j], HN); }
    for (int j = 5; j < 7; ++j) { TAKE(W->b[j], H); TAKE(W->r[j], H); TAKE(W->sv[j], H); }
    TAKE(W->z4, H); TAKE(W->l4, H); TAKE(W->nu, H); TAKE(W->den, H); TAKE(W->rp, H);
    TAKE(W->rg4, H); TAKE(W->SP, H); TAKE(W->rho, H); TAKE(W->sr, H); TAKE(W->ga, H);
    TAKE(W->dl4, H); TAKE(W->dnu, H); TAKE(W->dz4, H); TAKE(W->rc4, H);
    TAKE(W->G, K * K); TAKE(W->Gc, K * K); TAKE(W->Yrow, K); TAKE(W->zr, K); TAKE(W->bsm, K);
    TAKE(W->qv, K);
#undef TAKE
    return ((size_t)(p - W->pool) <= total) ? 0 : -1;
}

#define DPREV(W, k, t, i) ((t) ? (W)->w[(k) - (W)->N] : (W)->wp[i])

/* Z row t of asset i (columns: a_t -> t, v_t -> H+t, 1_t -> 2H+t) */
static void z_row(const ws_t* W, int t, int i, real* z) {
    int H = W->H, N = W->N;
    for (int j = 0; j < W->K; ++j) z[j] = 0;
    z[t] = W->a[t * N + i];
    if (W->ht) {
        z[H + t] = W->sr[t] * W->e[t * N + i];
        if (t + 1 < H) z[H + t + 1] = -W->sr[t + 1] * W->e[(t + 1) * N + i];
    }
    z[2 * H + t] = 1;
}

static int factor(ws_t* W) {
    int N = W->N, H = W->H, K = W->K;
    for (int t = 0; t < H; ++t) {
        real sp = 0;
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            real d = W->w[k] - DPREV(W, k, t, i);
            W->W1[k] = W->hw ? W->l1[k] / W->w[k] : 0;
            if (W->hs) {
                real al = W->l2[k] / (W->s[k] - d), be = W->l3[k] / (W->s[k] + d);
                real P = 1 / (al + be);
                W->P[k] = P; W->E[k] = 4 * al * be * P; W->e[k] = (be - al) * P; W->bma[k] = be - al;
                sp += P;
            } else {
                W->P[k] = W->E[k] = W->e[k] = W->bma[k] = 0;
            }
        }
        W->SP[t] = sp;
        W->ga[t] = W->ht ? W->l4[t] / W->z4[t] : 0;
        W->rho[t] = W->ht ? W->ga[t] / (1 + W->ga[t] * sp) : 0;
        W->sr[t] = RSQRT(W->rho[t]);
    }
    for (int i = 0; i < N; ++i) {
        real pi = W->W1[i] + W->E[i];
        for (int t = 0; t < H; ++t) {
            int k = t * N + i;
            if (t > 0) { W->Lr[k] = W->E[k] / W->Dd[k - N]; pi = W->W1[k] + W->Lr[k] * pi; }
            else W->Lr[k] = 0;
            W->Dd[k] = pi + (t + 1 < H ? W->E[k + N] : 0);
            if (!(W->Dd[k] > 0) || !RISFIN(W->Dd[k])) return -1;
        }
    }
    for (int j = 0; j < K * K; ++j) W->G[j] = 0;
    for (int i = 0; i < N; ++i) {
        for (int j = 0; j < K; ++j) W->Yrow[j] = 0;
        for (int t = 0; t < H; ++t) {
            int k = t * N + i;
            z_row(W, t, i, W->zr);
            real lr = W->Lr[k], inv = 1 / W->Dd[k];
            for (int j = 0; j < K; ++j) W->Yrow[j] = W->zr[j] + lr * W->Yrow[j];
            for (int j = 0; j < K; ++j) {
                real yj = W->Yrow[j] * inv;
                if (yj == 0) continue;
                for (int l = j; l < K; ++l) W->G[j * K + l] += yj * W->Yrow[l];
            }
        }
    }
    for (int j = 0; j < 2 * H; ++j) W->G[j * K + j] += 1;
    for (int j = 0; j < K; ++j)
        for (int l = 0; l <= j; ++l) W->Gc[j * K + l] = W->G[l * K + j];
    for (int j = 0; j < K; ++j) {
        real d = W->Gc[j * K + j];
        for (int p = 0; p < j; ++p) d -= W->Gc[j * K + p] * W->Gc[j * K + p];
        if (!(d > 0) || !RISFIN(d)) return -1;
        d = RSQRT(d);
        W->Gc[j * K + j] = d;
        for (int r = j + 1; r < K; ++r) {
            real v = W->Gc[r * K + j];
            for (int p = 0; p < j; ++p) v -= W->Gc[r * K + p] * W->Gc[j * K + p];
            W->Gc[r * K + j] = v / d;
        }
    }
    return 0;
}

/* (diag(alpha+beta) + gamma 1 1')^{-1} x per period = P (x - rho 1'P x) */
static void sinv(const ws_t* W, const real* x, real* out) {
    int N = W->N, H = W->H;
    for (int t = 0; t < H; ++t) {
        real acc = 0;
        for (int i = 0; i < N; ++i) acc += W->P[t * N + i] * x[t * N + i];
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            out[k] = W->P[k] * (x[k] - W->rho[t] * acc);
        }
    }
}

/*
 * Solve the full Newton system for rhs blocks b[0..6]:
 *   b[0] (1) Hf dw - (dl1 + deta_t - deta_{t+1}) + A^T dnu   deta = dl3 - dl2
 *   b[1] (2) -(dl2 + dl3 - dl4)
 *   b[2] (3) l1 dw + w dl1
 *   b[3] (4) l2 (ds - dd) + z2 dl2                            dd_t = dw_t - dw_{t-1}
 *   b[4] (5) l3 (ds + dd) + z3 dl3
 *   b[5] (6) -l4 1'ds + z4 dl4                                (per period)
 *   b[6] (7) 1'dw                                             (per period)
 */
static void lsolve(ws_t* W, real* const* b) {
    int N = W->N, H = W->H, K = W->K;
    size_t HN = (size_t)H * N;
    for (int t = 0; t < H; ++t)
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            real d = W->w[k] - DPREV(W, k, t, i);
            real p1 = W->hw ? b[2][k] / W->w[k] : 0, p2 = 0, p3 = 0, pn = 0;
            if (W->hs) {
                p2 = b[3][k] / (W->s[k] - d);
                p3 = b[4][k] / (W->s[k] + d);
                if (t + 1 < H) {
                    int kn = k + N;
                    real dn = W->w[kn] - W->w[k];
                    pn = b[4][kn] / (W->s[kn] + dn) - b[3][kn] / (W->s[kn] - dn);
                }
            }
            W->rhsw[k] = b[0][k] + p1 + (p3 - p2) - pn;
            W->rhss[k] = W->hs ? b[1][k] + p2 + p3 - (W->ht ? b[5][t] / W->z4[t] : 0) : 0;
        }
    if (W->hs) {
        sinv(W, W->rhss, W->tmp);
        for (size_t k = 0; k < HN; ++k) W->g[k] = W->bma[k] * W->tmp[k];
        for (int t = 0; t < H; ++t)
            for (int i = 0; i < N; ++i) {
                int k = t * N + i;
                W->rhsw[k] -= W->g[k] - (t + 1 < H ? W->g[k + N] : 0);
            }
    }
    for (int j = 0; j < K; ++j) W->bsm[j] = 0;
    for (int i = 0; i < N; ++i) {
        for (int j = 0; j < K; ++j) W->Yrow[j] = 0;
        real prev = 0;
        for (int t = 0; t < H; ++t) {
            int k = t * N + i;
            real y = W->rhsw[k] + W->Lr[k] * prev;
            W->yr[k] = y; prev = y;
            z_row(W, t, i, W->zr);
            real yd = y / W->Dd[k];
            for (int j = 0; j < K; ++j) {
                W->Yrow[j] = W->zr[j] + W->Lr[k] * W->Yrow[j];
                W->bsm[j] += W->Yrow[j] * yd;
            }
        }
    }
    for (int t = 0; t < H; ++t) W->bsm[2 * H + t] -= b[6][t];
    for (int j = 0; j < K; ++j) {
        real v = W->bsm[j];
        for (int p = 0; p < j; ++p) v -= W->Gc[j * K + p] * W->qv[p];
        W->qv[j] = v / W->Gc[j * K + j];
    }
    for (int j = K - 1; j >= 0; --j) {
        real v = W->qv[j];
        for (int p = j + 1; p < K; ++p) v -= W->Gc[p * K + j] * W->qv[p];
        W->qv[j] = v / W->Gc[j * K + j];
    }
    for (int i = 0; i < N; ++i) {
        for (int j = 0; j < K; ++j) W->Yrow[j] = 0;
        for (int t = 0; t < H; ++t) {
            int k = t * N + i;
            z_row(W, t, i, W->zr);
            real acc = 0;
            for (int j = 0; j < K; ++j) {
                W->Yrow[j] = W->zr[j] + W->Lr[k] * W->Yrow[j];
                acc += W->Yrow[j] * W->qv[j];
            }
            W->xr[k] = W->yr[k] - acc;
        }
        real nxt = 0;
        for (int t = H - 1; t >= 0; --t) {
            int k = t * N + i;
            real v = W->xr[k] / W->Dd[k] + (t + 1 < H ? W->Lr[k + N] * nxt : 0);
            W->dw[k] = v; nxt = v;
        }
    }
    for (int t = 0; t < H; ++t) W->dnu[t] = W->qv[2 * H + t];
    for (int t = 0; t < H; ++t)
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            W->dd[k] = W->dw[k] - (t ? W->dw[k - N] : 0);
        }
    if (W->hs) {
        for (size_t k = 0; k < HN; ++k) W->tmp[k] = W->rhss[k] - W->bma[k] * W->dd[k];
        sinv(W, W->tmp, W->ds);
    } else {
        for (size_t k = 0; k < HN; ++k) W->ds[k] = 0;
    }
    for (int t = 0; t < H; ++t) {
        real sds = 0;
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            real d = W->w[k] - DPREV(W, k, t, i);
            W->dl1[k] = W->hw ? (b[2][k] - W->l1[k] * W->dw[k]) / W->w[k] : 0;
            if (W->hs) {
                W->dl2[k] = (b[3][k] - W->l2[k] * (W->ds[k] - W->dd[k])) / (W->s[k] - d);
                W->dl3[k] = (b[4][k] - W->l3[k] * (W->ds[k] + W->dd[k])) / (W->s[k] + d);
            } else {
                W->dl2[k] = W->dl3[k] = 0;
            }
            sds += W->ds[k];
        }
        W->dl4[t] = W->ht ? (b[5][t] + W->l4[t] * sds) / W->z4[t] : 0;
    }
}

/* r = b - Op(direction) for the system of lsolve */
static void nresidual(ws_t* W, real* const* b, real* const* r) {
    int N = W->N, H = W->H;
    for (int t = 0; t < H; ++t) {
        real adw = 0, sds = 0, sdw = 0;
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            adw += W->a[k] * W->dw[k]; sds += W->ds[k]; sdw += W->dw[k];
        }
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            real d = W->w[k] - DPREV(W, k, t, i);
            real dd = W->dw[k] - (t ? W->dw[k - N] : 0);
            real deta = W->dl3[k] - W->dl2[k];
            real detan = (t + 1 < H) ? W->dl3[k + N] - W->dl2[k + N] : 0;
            r[0][k] = b[0][k] - (W->a[k] * adw - (W->dl1[k] + deta - detan) + W->dnu[t]);
            r[1][k] = W->hs ? b[1][k] + (W->dl2[k] + W->dl3[k] - W->dl4[t]) : 0;
            r[2][k] = W->hw ? b[2][k] - (W->l1[k] * W->dw[k] + W->w[k] * W->dl1[k]) : 0;
            if (W->hs) {
                r[3][k] = b[3][k] - (W->l2[k] * (W->ds[k] - dd) + (W->s[k] - d) * W->dl2[k]);
                r[4][k] = b[4][k] - (W->l3[k] * (W->ds[k] + dd) + (W->s[k] + d) * W->dl3[k]);
            } else {
                r[3][k] = r[4][k] = 0;
            }
        }
        r[5][t] = W->ht ? b[5][t] - (-W->l4[t] * sds + W->z4[t] * W->dl4[t]) : 0;
        r[6][t] = b[6][t] - sdw;
    }
}

/* dev statistic (tools/refine_stats.py): refinement steps per Newton solve, atomic under OpenMP */
static long nref_total = 0, nsolve_total = 0;
__attribute__((destructor)) static void refstat(void) {
    if (getenv("KMPC_ORACLE_REFSTAT") && nsolve_total) fprintf(stderr, "refines/solve %.3f over %ld solves\n", (double)nref_total / nsolve_total, nsolve_total);
}
/* Newton direction for complementarity products rc (= z l - target) with iterative refinement */
static void newton(ws_t* W) {
    int N = W->N, H = W->H;
    size_t HN = (size_t)H * N;
    for (size_t k = 0; k < HN; ++k) {
        W->b[0][k] = -W->rdw[k]; W->b[1][k] = -W->rds[k];
        W->b[2][k] = -W->rc1[k]; W->b[3][k] = -W->rc2[k]; W->b[4][k] = -W->rc3[k];
    }
    for (int t = 0; t < H; ++t) {
        W->b[5][t] = W->ht ? -W->rc4[t] - W->l4[t] * W->rg4[t] : 0;
        W->b[6][t] = -W->rp[t];
    }
    lsolve(W, W->b);
    real* sol[7] = {W->dw, W->ds, W->dl1, W->dl2, W->dl3, W->dl4, W->dnu};
    const double adapt = 1e-7;   /* stop refining once ||r||_inf <= adapt ||b||_inf (the kernels' REFINE_RTOL) */
    real bn = 0;
    if (adapt > 0) {
        for (int j = 0; j < 7; ++j) { size_t n = j < 5 ? HN : (size_t)H; for (size_t k = 0; k < n; ++k) bn = RFMAX(bn, RFABS(W->b[j][k])); }
    }
#pragma omp atomic
    nsolve_total++;
    for (int it = 0; it < W->n_refine; ++it) {
        for (int j = 0; j < 7; ++j) memcpy(W->sv[j], sol[j], sizeof(real) * (j < 5 ? HN : (size_t)H));
        nresidual(W, W->b, W->r);
        if (adapt > 0) {
            real rn = 0;
            for (int j = 0; j < 7; ++j) { size_t n = j < 5 ? HN : (size_t)H; for (size_t k = 0; k < n; ++k) rn = RFMAX(rn, RFABS(W->r[j][k])); }
            if (rn <= adapt * bn) break;
        }
#pragma omp atomic
        nref_total++;

        lsolve(W, W->r);
        for (int j = 0; j < 7; ++j) {
            size_t n = j < 5 ? HN : (size_t)H;
            for (size_t k = 0; k < n; ++k) sol[j][k] += W->sv[j][k];
        }
    }
    for (int t = 0; t < H; ++t) {
        real sds = 0;
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            W->dd[k] = W->dw[k] - (t ? W->dw[k - N] : 0);
            sds += W->ds[k];
        }
        W->dz4[t] = W->ht ? -sds + W->rg4[t] : 0;
    }
}

static real to_bound(real v, real dv, real a) {
    if (dv < 0) { real r = -v / dv; if (r < a) a = r; }
    return a;
}

/* largest step keeping w, s -+ d, z4, the multipliers and the log argument positive */
static real max_step(const ws_t* W) {
    int N = W->N, H = W->H;
    real a = R_(1e30);
    for (int t = 0; t < H; ++t) {
        real mdw = 0;
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            if (W->hw) { a = to_bound(W->w[k], W->dw[k], a); a = to_bound(W->l1[k], W->dl1[k], a); }
            if (W->hs) {
                real d = W->w[k] - DPREV(W, k, t, i);
                a = to_bound(W->s[k] - d, W->ds[k] - W->dd[k], a);
                a = to_bound(W->s[k] + d, W->ds[k] + W->dd[k], a);
                a = to_bound(W->l2[k], W->dl2[k], a);
                a = to_bound(W->l3[k], W->dl3[k], a);
            }
            mdw += W->m[k] * W->dw[k];
        }
        a = to_bound(W->den[t], mdw, a);
        if (W->ht) { a = to_bound(W->z4[t], W->dz4[t], a); a = to_bound(W->l4[t], W->dl4[t], a); }
    }
    return a;
}

static real complementarity(const ws_t* W, real a) {
    int N = W->N, H = W->H;
    real acc = 0;
    for (int t = 0; t < H; ++t) {
        for (int i = 0; i < N; ++i) {
            int k = t * N + i;
            real d = W->w[k] - DPREV(W, k, t, i);
            if (W->hw) acc += (W->w[k] + a * W->dw[k]) * (W->l1[k] + a * W->dl1[k]);
            if (W->hs) {
                acc += (W->s[k] - d + a * (W->ds[k] - W->dd[k])) * (W->l2[k] + a * W->dl2[k]);
                acc += (W->s[k] + d + a * (W->ds[k] + W->dd[k])) * (W->l3[k] + a * W->dl3[k]);
            }
        }
        if (W->ht) acc += (W->z4[t] + a * W->dz4[t]) * (W->l4[t] + a * W->dl4[t]);
    }
    return acc;
}

double API(kmpc_oracle_objective)(int N, int H, const double* wp, const float* yhat, double c,
                                  const double* Wm) {
    /* problem.value of mpc.py:103: sum_t log(w_t . exp(y_t)) - c sum_t ||w_t - w_{t-1}||_1 */
    double f = 0;
    for (int t = 0; t < H; ++t) {
        double rw = 0, l1 = 0;
        for (int i = 0; i < N; ++i) {
            rw += (double)np_expf(yhat[t * N + i]) * Wm[t * N + i];
            l1 += fabs(Wm[t * N + i] - (t ? Wm[(t - 1) * N + i] : wp[i]));
        }
        f += log(rw) - c * l1;
    }
    return f;
}

int API(kmpc_oracle_solve)(int N, int H, const double* wp, const float* yhat, double c, double tau,
                           int allow_short, int max_iter, double tol, double* Wout, double* obj,
                           int* iters_out) {
    int status = ST_ERROR, it = 0;
    size_t HN = (size_t)H * N;
    if (iters_out) *iters_out = 0;
    if (N < 1 || H < 1) return ST_ERROR;
    if (max_iter <= 0) max_iter = 80;
    if (tol <= 0) tol = 1e-11;
    int finite = isfinite(c) && isfinite(tau);
    for (size_t k = 0; k < HN; ++k) finite &= isfinite(np_expf(yhat[k])) != 0;   /* R finite */
    for (int i = 0; i < N; ++i) finite &= isfinite(wp[i]) != 0;

    ws_t W;
    memset(&W, 0, sizeof(W));
    if (finite && ws_init(&W, N, H) == 0) {
        W.N = N; W.H = H; W.K = 3 * H;
        W.hw = !allow_short; W.hs = (c > 0) || (tau > 0); W.ht = tau > 0;
        W.n_refine = 3;   /* the kernels' default (kmpc_solve_desc.n_refine = 0 -> 3) */
        real sig = c;
        for (int i = 0; i < N; ++i) W.wp[i] = wp[i];
        for (size_t k = 0; k < HN; ++k)
            W.m[k] = (real)((double)np_expf(yhat[k]) - 1.0);   /* exact for R >= 2^-29: R has 24 bits */

        /* per period S_t = sum_i R_t,i of the float32 R.
           S_t = 0 (every R underflowed: yhat <= -103.97): R_t . w_t = 0 on the whole simplex and the
           reference's exp cone exp(u) <= R_t . w_t has no solution — cvxpy reports infeasible
           (mpc.py:113: fallback, value None).
           0 < S_t < 2^-16 (every yhat below ~ -11): the program is the same for R_t / S_t up to the
           constant log S_t (log(R.w) = log S_t + log((R / S_t).w)), and 1 + m = R would lose R's
           digits (m = R - 1 rounds to -1 below 2^-53), so m = R / S_t - 1 there (KMPC_TINY_PERIOD,
           as the kernels; the objective below is evaluated from R itself) */
        for (int t = 0; t < H; ++t) {
            double S = 0;
            for (int i = 0; i < N; ++i) S += (double)np_expf(yhat[t * N + i]);
            if (S == 0) { status = ST_INFEASIBLE; goto done; }
            if (S < KMPC_TINY_PERIOD)
                for (int i = 0; i < N; ++i)
                    W.m[t * N + i] = (real)((double)np_expf(yhat[t * N + i]) / S - 1.0);
        }
        for (size_t k = 0; k < HN; ++k)
            if (RFABS(W.m[k]) > sig) sig = RFABS(W.m[k]);
        if (!(sig > 0)) sig = 1;
        W.sig = sig; W.c = c / sig; W.tau = tau;

        if (allow_short && !W.hs) {
            /* no bounds and no turnover terms: unbounded unless every period is flat */
            int flat = 1;
            for (int t = 0; t < H; ++t)
                for (int i = 1; i < N; ++i) flat &= W.m[t * N + i] == W.m[t * N];
            if (flat) {
                real sw = 0;
                for (int i = 0; i < N; ++i) sw += wp[i];
                for (size_t k = 0; k < HN; ++k) W.wbest[k] = (sw != 0) ? wp[k % N] / sw : R_(1.0) / N;
                status = ST_OPTIMAL;
            } else {
                status = ST_UNBOUNDED;
            }
            goto done;
        }

        /* initial point: strictly interior w, s; multipliers KMPC_INIT_MULT = 0.5 (scaled problem;
           round 6: 1 -> 0.5 took the C3 bench windows from 16.65 to 16.19 iterations, random C3
           windows 18.43 -> 17.79, N = 10 / H = 5 10.79 -> 10.31, N = 500 / H = 20 26.51 -> 26.01,
           same statuses; the kernels use the same constant, kmpc_solve_kernel.h) */
        for (int t = 0; t < H; ++t)
            for (int i = 0; i < N; ++i) {
                real b0 = W.hw ? (wp[i] > 0 ? wp[i] : 0) : wp[i];
                W.w[t * N + i] = R_(0.5) * b0 + R_(0.5) / N;
            }
        for (int t = 0; t < H; ++t) {
            real ss = 0;
            for (int i = 0; i < N; ++i) {
                int k = t * N + i;
                real d = W.w[k] - DPREV(&W, k, t, i);
                W.s[k] = W.hs ? RFABS(d) + R_(1.0) / N : 0;
                ss += W.s[k];
                W.l1[k] = W.hw ? KMPC_INIT_MULT : 0;
                W.l2[k] = W.l3[k] = W.hs ? KMPC_INIT_MULT : 0;
            }
            W.z4[t] = W.ht ? RFMAX(tau - ss, R_(0.5) * tau) : 1;
            W.l4[t] = W.ht ? KMPC_INIT_MULT : 0;
            W.nu[t] = 0;
        }
        int ncon = (W.hw ? (int)HN : 0) + (W.hs ? 2 * (int)HN : 0) + (W.ht ? H : 0);
        if (ncon == 0) ncon = 1;
        real best = R_(1e30), best_pr = R_(1e30), best_dr = R_(1e30), best_mu = R_(1e30), min_pr = R_(1e30);
        int trace = getenv("KMPC_ORACLE_TRACE") != NULL;

        for (it = 0; it < max_iter; ++it) {
            real mu = 0, rd = 0, pr = 0;
            int domain_ok = 1;
            for (int t = 0; t < H; ++t) {
                real den = 1, sw = 0, ss = 0;
                for (int i = 0; i < N; ++i) {
                    int k = t * N + i;
                    den += W.m[k] * W.w[k]; sw += W.w[k]; ss += W.s[k];
                }
                W.den[t] = den; W.rp[t] = sw - 1;
                W.rg4[t] = W.ht ? tau - ss - W.z4[t] : 0;
                if (!(den > 0)) domain_ok = 0;
                for (int i = 0; i < N; ++i) {
                    int k = t * N + i;
                    real d = W.w[k] - DPREV(&W, k, t, i);
                    W.a[k] = W.m[k] / (den * RSQRT(sig));
                    real eta = W.l3[k] - W.l2[k];
                    real etan = (t + 1 < H) ? W.l3[k + N] - W.l2[k + N] : 0;
                    W.rdw[k] = -W.m[k] / (sig * den) - (W.l1[k] + eta - etan) + W.nu[t];
                    W.rds[k] = W.hs ? W.c - (W.l2[k] + W.l3[k] - W.l4[t]) : 0;
                    W.rc1[k] = W.hw ? W.w[k] * W.l1[k] : 0;
                    W.rc2[k] = W.hs ? (W.s[k] - d) * W.l2[k] : 0;
                    W.rc3[k] = W.hs ? (W.s[k] + d) * W.l3[k] : 0;
                    mu += W.rc1[k] + W.rc2[k] + W.rc3[k];
                    rd = RFMAX(rd, RFMAX(RFABS(W.rdw[k]), RFABS(W.rds[k])));
                }
                W.rc4[t] = W.ht ? W.z4[t] * W.l4[t] : 0;
                mu += W.rc4[t];
                pr = RFMAX(pr, RFMAX(RFABS(W.rp[t]), RFABS(W.rg4[t])));
            }
            if (!domain_ok) break;
            mu /= ncon;
            real merit = RFMAX(mu, RFMAX(rd, pr));
            min_pr = RFMIN(min_pr, pr);
            if (trace) fprintf(stderr, "it %d mu %.3Le rd %.3Le pr %.3Le\n", it, (long double)mu,
                               (long double)rd, (long double)pr);
            if (!RISFIN(merit)) break;
            if (merit < best) {
                best = merit; best_pr = pr; best_dr = rd; best_mu = mu;
                memcpy(W.wbest, W.w, sizeof(real) * HN);
            } else if (best < R_(1e-6) && merit > R_(1e4) * best) {
                break;   /* numerical breakdown after convergence: keep the best iterate */
            }
            if (mu < tol && rd < 10 * tol && pr < 10 * tol) break;
            if (factor(&W) != 0) break;
            /* predictor: rc = z l (no refinement: the affine direction only sets the step
               estimate, sigma and the second-order term; the corrector is refined) */
            {
                const int nr = W.n_refine;
                W.n_refine = 0;
                newton(&W);
                W.n_refine = nr;
            }
            real ap = RFMIN(1, max_step(&W));
            real sg = complementarity(&W, ap) / ncon / mu;
            sg = sg * sg * sg;
            /* no short + turnover cap: sigma capped at 0.2 (the kernels' KMPC_SIGMA_CAP, round 6) */
            if (W.hw && W.ht && sg > KMPC_SIGMA_CAP) sg = KMPC_SIGMA_CAP;
            /* corrector: rc = z l + dz_aff dl_aff - sigma mu */
            for (int t = 0; t < H; ++t) {
                for (int i = 0; i < N; ++i) {
                    int k = t * N + i;
                    if (W.hw) W.rc1[k] += W.dw[k] * W.dl1[k] - sg * mu;
                    if (W.hs) {
                        W.rc2[k] += (W.ds[k] - W.dd[k]) * W.dl2[k] - sg * mu;
                        W.rc3[k] += (W.ds[k] + W.dd[k]) * W.dl3[k] - sg * mu;
                    }
                }
                if (W.ht) W.rc4[t] += W.dz4[t] * W.dl4[t] - sg * mu;
            }
            {   /* corrector refinement only once mu <= 1e-6, 1e-5 with shorting (the kernels'
                   REFINE_MU / REFINE_MU_SHORT; fixed constants: the goldens depend on them) */
                const double rmu = W.hw ? 1e-6 : 1e-5;
                const int nr = W.n_refine;
                if (mu > (real)rmu) W.n_refine = 0;
                newton(&W);
                W.n_refine = nr;
            }
            /* one step length for primal and dual: the objective is nonlinear, so unequal steps
               would re-inject dual residual (alpha_p - alpha_d) Hf dw. 0.995 of the boundary
               without shorting, 0.99 with it (the kernels' KMPC_STEP_NOSHORT, round 6) */
            real a = RFMIN(1, (W.hw ? KMPC_STEP_NOSHORT : R_(0.99)) * max_step(&W));
            for (size_t k = 0; k < HN; ++k) {
                W.w[k] += a * W.dw[k]; W.s[k] += a * W.ds[k];
                W.l1[k] += a * W.dl1[k]; W.l2[k] += a * W.dl2[k]; W.l3[k] += a * W.dl3[k];
            }
            for (int t = 0; t < H; ++t) {
                W.z4[t] += a * W.dz4[t]; W.l4[t] += a * W.dl4[t]; W.nu[t] += a * W.dnu[t];
            }
        }
        if (best <= R_(1e-7)) status = ST_OPTIMAL;
        else if (best <= R_(1e-4)) status = ST_INACCURATE;
        else if (min_pr > R_(1e-6)) status = ST_INFEASIBLE;   /* primal residual never closed */
        else status = ST_ERROR;
        (void)best_pr; (void)best_dr; (void)best_mu;
    }
done:
    if (iters_out) *iters_out = it;
    if (status == ST_OPTIMAL || status == ST_INACCURATE) {
        for (size_t k = 0; k < HN; ++k) Wout[k] = (double)W.wbest[k];
        if (obj) *obj = API(kmpc_oracle_objective)(N, H, wp, yhat, c, Wout);
    } else {
        for (int t = 0; t < H; ++t)
            for (int i = 0; i < N; ++i) Wout[(size_t)t * N + i] = wp[i];   /* mpc.py:113-115 */
        if (obj) *obj = NAN;
    }
    free(W.pool);
    return status;
}

/* B independent windows, OpenMP across windows (CPU baseline). */
int API(kmpc_oracle_solve_batch)(int B, int N, int H, const double* wp, const float* yhat,
                                 double c, double tau, int allow_short, int max_iter, double tol,
                                 double* Wout, double* obj, int* status, int* iters) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int b = 0; b < B; ++b) {
        int itb = 0;
        status[b] = API(kmpc_oracle_solve)(N, H, wp + (size_t)b * N, yhat + (size_t)b * H * N, c,
                                           tau, allow_short, max_iter, tol,
                                           Wout + (size_t)b * H * N, obj + b, &itb);
        if (iters) iters[b] = itb;
    }
    return 0;
}
