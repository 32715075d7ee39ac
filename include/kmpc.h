/*
 * kmpc.h — C ABI of the MI355X-native Koopman-MPC window engine (libkmpc.so).
 *
 * This is the drop-in boundary for the per-window hot path of the reference
 * (yli421/koopman-mpc-portfolio-rebalancing):
 *
 *   KoopmanMPCStrategy.rebalance            backtest.py:80-131
 *     encode -> H x (step_latent, decode, extract[:N], destandardize)
 *                                           backtest.py:99-121, model.py:756-797,839-850,
 *                                           data_finance.py:717-742
 *     solve_mpc_log_utility(w_prev, yhat)   mpc.py:27-117
 *
 * Conventions
 *   - Every pointer argument of kmpc_rollout / kmpc_solve / kmpc_window is a DEVICE pointer owned
 *     by the caller (e.g. torch tensor storage). Arrays are row-major and contiguous.
 *   - Calls are stream-ordered on `stream` (a hipStream_t passed as void*; NULL = default stream),
 *     allocate nothing, hold no global state and are re-entrant per device.
 *   - Return value: KMPC_OK (0) or a negative KMPC_ERR_* code (argument / launch errors).
 *     Per-problem solver outcome is reported in status[] (KMPC_STATUS_*), never as an error:
 *     this mirrors mpc.py:107-117, where solver failure is not raised but reported through
 *     problem.status and answered with the "hold current weights" fallback.
 *   - No torch types cross this boundary.
 */
#ifndef KMPC_H
#define KMPC_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ------------------------------------------------------------------------- */
#define KMPC_OK               0
#define KMPC_ERR_INVALID     -1   /* bad descriptor / null pointer                              */
#define KMPC_ERR_UNSUPPORTED -2   /* shape outside what the kernels were built for             */
#define KMPC_ERR_WORKSPACE   -3   /* ws_bytes smaller than kmpc_workspace_bytes()              */
#define KMPC_ERR_LAUNCH      -4   /* a HIP launch failed (hipGetLastError)                     */

/* ---- per-problem solver status (maps to cvxpy status strings, mpc.py:113) ----------------- */
#define KMPC_STATUS_OPTIMAL            0  /* "optimal"                                         */
#define KMPC_STATUS_OPTIMAL_INACCURATE 1  /* "optimal_inaccurate"                              */
#define KMPC_STATUS_INFEASIBLE         2  /* "infeasible"                                      */
#define KMPC_STATUS_UNBOUNDED          3  /* "unbounded"                                       */
#define KMPC_STATUS_SOLVER_ERROR       4  /* "solver_error" (non-finite inputs, breakdown)     */

/* Maximum horizon / asset count the solver kernels are instantiated for. */
#define KMPC_MAX_H 21   /* the 3H x 3H Schur system is factored by one 64-lane wavefront */
#define KMPC_MAX_N 1024

/* ---- MPC solve: replaces solve_mpc_log_utility (mpc.py:27-117) ---------------------------- */
/*
 * For each problem b (one rolling window):
 *   maximize_W  sum_t log(R_t . w_t) - c * sum_t ||w_t - w_{t-1}||_1        (mpc.py:66-103)
 *   s.t.        1^T w_t = 1;  w_t >= 0 unless allow_short;                  (mpc.py:83-86)
 *               ||w_t - w_{t-1}||_1 <= tau  if tau > 0, w_{-1} = w_prev     (mpc.py:94-100)
 *   with R_t = np.exp(yhat_t) (mpc.py:55) evaluated in float32 exactly as numpy does it
 *   (kmpc_gross_returns below) and then used in float64, as cvxpy receives it; W in [H, N].
 * Inputs:  yhat [B, H, N] float32 (predicted log-returns, the reference passes float32 here,
 *          backtest.py:121), w_prev [B, N] float64 (current_weights).
 * Outputs: w_out [B, N] (W[0], what rebalance() applies, backtest.py:131) or [B, H, N] when
 *          return_full_W != 0; status [B]; obj [B] (problem.value, NaN when not optimal);
 *          iters [B] (may be NULL; interior-point iterations taken, 0 for windows solved by the
 *          closed-form presolve: cost_coeff = 0, max_turnover <= 0, no shorting, where the
 *          program separates into H simplex problems with a vertex optimum).
 * Failure fallback (mpc.py:113-115) is applied in-kernel: w_out = tile(w_prev), obj = NaN.
 *          Non-finite yhat / w_prev, or an R that overflows float32 (yhat >= 88.72), give
 *          solver_error and the fallback.
 * Errors:  cost_coeff < 0 -> KMPC_ERR_INVALID: the reference program is then not convex
 *          and cvxpy raises (DCPError) instead of returning a status.
 * Workspace: always size it with kmpc_workspace_bytes(NULL, desc). It is 0 for windows of
 *          N <= 256 assets and H <= 10 periods (solved in registers); otherwise the large-window
 *          kernel keeps each window's interior-point state there: (22 HM + 128) (64 ceil(N / 64))
 *          doubles per window slot, HM = 10 for H <= 10 and 21 past it (the compiled horizon
 *          bound, not H), for min(B, 768) slots when N <= 256, min(B, 512) otherwise.
 *          The mixed-precision pair (AUTO at >= KMPC_MIXED_MIN_B windows, MIXED) keeps a 64 B record
 *          header per window, B x 64 bytes (ABI 0.6.0: the float32 iterate goes to the float64
 *          finish on chip; 0.5.0 kept a (5 H N + 3 H + 16)-float record per window).
 *          Too little -> KMPC_ERR_WORKSPACE.
 */
#define KMPC_PATH_AUTO     0   /* kernel chosen by shape and batch (and the closed-form presolve);
                                  small windows (N <= 32) are packed 2-4 per wave from
                                  KMPC_PACK_MIN_B windows per call (ABI 0.6.0; any batch for
                                  H <= 2), one per wave below it — the faster form at each size */
#define KMPC_PACK_MIN_B    512
#define KMPC_PATH_REGISTER 1   /* interior point in the register kernels where the shape fits them
                                  (small windows packed at any batch size)                         */
#define KMPC_PATH_LARGE    2   /* interior point in the large-window (workspace) kernel            */
#define KMPC_PATH_REGISTER_UNPACKED 3   /* register kernels, one window per wave even for N <= 32
                                           (no lane-group packing); for A/B and tests             */
/* Arithmetic of the interior point. MIXED: where a mixed-precision kernel pair exists (H = 10,
 * 64 < N < 104, no short, c > 0 or tau > 0 with a cap: BASELINE configs[2..3]) the first iterations
 * run in float32 (the whole state in registers, no spills) until mu <= mu_handoff, and the float64
 * kernel finishes from that iterate to the same tolerance and status rules as F64; elsewhere
 * float64. AUTO: MIXED from KMPC_MIXED_MIN_B windows per call (a throughput win), F64 below it
 * (a latency-bound batch: the lock-step backtest's few paths finish sooner in float64 alone).
 * F64: float64 throughout. The answer's accuracy is that of the float64 finish either way. */
#define KMPC_PRECISION_AUTO  0
#define KMPC_PRECISION_F64   1
#define KMPC_PRECISION_MIXED 2
#define KMPC_MIXED_MIN_B 2048
typedef struct kmpc_solve_desc {
    int    B;              /* number of independent problems (windows); past 2^22
                              the solve runs as equal launches of <= 2^22 windows
                              (same kernels, same results as one launch)          */
    int    N;              /* assets,  1 <= N <= KMPC_MAX_N                       */
    int    H;              /* horizon, 1 <= H <= KMPC_MAX_H                       */
    double cost_coeff;     /* MPCConfig.cost_coeff   (mpc.py:22)                  */
    double max_turnover;   /* MPCConfig.max_turnover (mpc.py:23); <= 0 disables   */
    int    allow_short;    /* MPCConfig.allow_short  (mpc.py:24)                  */
    int    max_iter;       /* interior-point iteration cap (0 -> default 80)      */
    double tol;            /* complementarity tolerance (<= 0 -> default 1e-9)    */
    int    return_full_W;  /* 0: w_out is [B,N] (W[0]); 1: w_out is [B,H,N]       */
    int    n_refine;       /* max iterative-refinement steps per Newton solve; refinement stops once
                              ||r||_inf <= 1e-7 ||b||_inf (<0 -> none, 0 -> default 3)             */
    int    path;           /* KMPC_PATH_* (0 = by shape). Per call: no process-wide switches      */
    int    precision;      /* KMPC_PRECISION_* (ABI 0.3.0; MIXED 0.4.0)                           */
    double mu_handoff;     /* mixed precision: the float32 phase hands its iterate to the float64
                              solve once the scaled complementarity mu <= mu_handoff
                              (<= 0 -> default 3e-5)                                               */
} kmpc_solve_desc;

int kmpc_solve(const kmpc_solve_desc* desc,
               const float*  yhat,     /* [B,H,N] */
               const double* w_prev,   /* [B,N]   */
               double*       w_out,    /* [B,N] or [B,H,N] */
               int*          status,   /* [B] */
               double*       obj,      /* [B] */
               int*          iters,    /* [B] or NULL */
               void* workspace, size_t ws_bytes, void* stream);

/* ---- gross returns: R = np.exp(yhat) on float32, bit for bit as numpy 2.x evaluates it on x86-64
 * (mpc.py:55; the realized returns np.exp(r) - 1 of backtest.py:188 use the same function).
 * yhat and R are device arrays of n floats. */
int kmpc_gross_returns(size_t n, const float* yhat, float* R, void* stream);

/* ---- Koopman rollout: replaces backtest.py:99-121 (+ model.py encode/step/decode) ---------- */
#define KMPC_MODEL_GENERIC 0   /* GenericKM / SparseKM (model.py:701-797)                      */
#define KMPC_MODEL_LISTA   1   /* LISTAKM              (model.py:801-870)                      */
#define KMPC_ACT_RELU 0
#define KMPC_ACT_TANH 1
#define KMPC_ACT_GELU 2
#define KMPC_NORM_ID   0
#define KMPC_NORM_BALL 1
#define KMPC_MAX_LAYERS 8
#define KMPC_DTYPE_F32  0   /* fp32 arithmetic (the reference's). The GEMMs run on the bf16 MFMA with
                               each fp32 operand split exactly into three bf16 planes and the six
                               leading plane products accumulated in fp32: an fp32 GEMM in accuracy
                               (error against a float64 restatement equal to the f32-input MFMA's,
                               DESIGN.md §3.1), 2.7x the f32-input MFMA's peak rate               */
#define KMPC_DTYPE_BF16 1   /* GEMM operands rounded to bf16 (BASELINE configs[4])               */
#define KMPC_DTYPE_F32_F32MFMA 2   /* fp32 arithmetic on the f32-input MFMA (v_mfma_f32_32x32x2_f32,
                                      the round-4 GEMMs; A/B and tests)                          */
/*
 * An MLP (model.py:67-117, MLPCoder): n_layers Linear layers with dims[0] -> dims[1] -> ... ->
 * dims[n_layers]; activation `act` after every layer but the last; ReLU after the last one when
 * last_relu. weights[l] is the nn.Linear weight [dims[l+1], dims[l]] (row-major, [out, in]),
 * bias[l] is [dims[l+1]] or NULL.
 */
typedef struct kmpc_mlp {
    int n_layers;
    int dims[KMPC_MAX_LAYERS + 1];
    int act;
    int last_relu;
    const float* weight[KMPC_MAX_LAYERS];
    const float* bias[KMPC_MAX_LAYERS];
} kmpc_mlp;

#define KMPC_LATENT_AUTO       0   /* kmpc_rollout_desc.latent_unfused */
#define KMPC_LATENT_UNFUSED    1
#define KMPC_LATENT_SEQUENTIAL 2

typedef struct kmpc_rollout_desc {
    int B;            /* windows                                                  */
    int N;            /* assets (first N outputs of the decoder, data_finance.py:729) */
    int H;            /* horizon                                                  */
    int L;            /* latent size (MODEL.TARGET_SIZE)                          */
    int obs;          /* observation size N * EMBEDDING_DIM                       */
    int model_kind;   /* KMPC_MODEL_*                                             */
    int norm_fn;      /* KMPC_NORM_* (GenericKM only, model.py:740-754)           */
    /* encoder: GenericKM MLP encoder, or LISTA's We (MLP, or 1 linear layer)      */
    kmpc_mlp encoder;
    /* LISTA (model.py:190-209): z = shrink(We x, thr); loops x z = shrink(z S + c, thr) */
    const float* lista_S;     /* [L, L]   */
    int   lista_loops;
    float lista_thresh;       /* alpha / L */
    /* Koopman matrix, z <- z @ K (row-vector convention, model.py:311-321) */
    const float* kmat;        /* [L, L]   */
    /* decoder (GenericKM: MLP decoder; LISTAKM: one linear layer = normalised dictionary^T).
       Only the first N outputs of the last layer are evaluated. For a 1-layer decoder
       decoder.weight[0] may point at the first N rows of the [obs, L] weight (ld = L).   */
    kmpc_mlp decoder;
    const float* mean;        /* [N] de-standardisation (data_finance.py:740-742) */
    const float* std;         /* [N] */
    int obs_ld;               /* row stride of obs in floats (0 -> obs). With obs_ld = N, obs may
                                 point into a standardized [T, N] return panel: window i reads the
                                 rows i .. i+d-1 (kmpc_standardize below) — the time-delay
                                 embedding without materialising it; the first encoder layer's
                                 column blocks must then be in oldest-lag-first order.          */
    int dtype;                /* KMPC_DTYPE_F32 (0, the reference's fp32 arithmetic), KMPC_DTYPE_BF16
                                 (1: GEMM operands rounded to bf16 on MFMA, fp32 accumulation and
                                 epilogues; BASELINE configs[4]) or KMPC_DTYPE_F32_F32MFMA (2)   */
    int latent_unfused;       /* the H-step latent loop (KMPC_LATENT_*, same fp32 arithmetic up to
                                 summation order; A/B and tests):
                                 0 AUTO: the library's choice — from KMPC_LATPOW_MINB (8,192) windows
                                   with a linear latent step (norm 'id', LISTA) one GEMM of z_0 against
                                   the latent powers D_N (K^T)^t, else one fused launch;
                                 1 UNFUSED: one GEMM launch per step;
                                 2 SEQUENTIAL: the fused step-by-step loop at every batch size
                                   (ABI 0.6.0; the three-plane latent_steps_x3_kernel at L = 256) */
} kmpc_rollout_desc;

int kmpc_rollout(const kmpc_rollout_desc* desc,
                 const float* obs,    /* [B, obs] standardized time-delay embedding */
                 float*       yhat,   /* [B, H, N] */
                 void* workspace, size_t ws_bytes, void* stream);

/* ---- data format before the path: standardize a log-return panel (data_finance.py:243-260, 331) */
/* z[t, n] = (float)((log_returns[t, n] - mean[n]) / std[n]), float64 arithmetic then float32, as
 * the reference standardizes in pandas and casts with .astype(np.float32). */
int kmpc_standardize(int T, int N, const double* log_returns, const double* mean, const double* std,
                     float* z, void* stream);

/* ---- fused window: rollout -> solve on one stream (KoopmanMPCStrategy.rebalance) ---------- */
int kmpc_window(const kmpc_rollout_desc* rdesc, const kmpc_solve_desc* sdesc,
                const float*  obs,      /* [B, obs] */
                const double* w_prev,   /* [B, N]   */
                float*        yhat,     /* [B, H, N] (written; may be NULL -> kept in workspace) */
                double*       w_out, int* status, double* obj, int* iters,
                void* workspace, size_t ws_bytes, void* stream);

/* ---- lock-step backtest bookkeeping for P paths: run_backtest / calculate_metrics ------------ */
/*
 * Replaces the per-step body of run_backtest (backtest.py:173-217) for P independent paths run in
 * lock step (each path's target weights come from kmpc_window / kmpc_solve), and calculate_metrics
 * (backtest.py:221-249) per path. History layout: hist [P, S, 4] float64 rows
 * (portfolio_value, return, turnover, cost) — the reference DataFrame columns.
 */
typedef struct kmpc_backtest_desc {
    int    P;            /* paths run in lock step                                   */
    int    N;            /* assets                                                   */
    int    S;            /* history rows per path                                    */
    double cost_coeff;   /* BacktestConfig.cost_coeff (backtest.py:28)               */
} kmpc_backtest_desc;

/* Step `step` (history row) for every path: cost from the turnover to `target` [P,N] f64, the
 * realized float32 log-returns of t+1 `realized_next` [P,N] (NULL when t+1 is past the data:
 * no market move), value [P] and weights [P,N] updated in place (drift with the 1e-8 guard). */
int kmpc_backtest_step(const kmpc_backtest_desc* desc, int step, const double* target,
                       const float* realized_next, double* weights, double* value, double* hist,
                       void* stream);

/* A whole run_backtest per path in ONE launch (ABI 0.5.0): steps step0 .. step0 + n_steps - 1 of
 * every path, each the kmpc_solve of that step's window then the kmpc_backtest_step bookkeeping,
 * run back to back by one workgroup per path — no per-step launches, and no path waits for the
 * slowest window of the step (the lock-step loop's bound at small P). The results are bit-identical
 * to that loop (kmpc_solve of the P windows + kmpc_backtest_step per step): the same window solve
 * and the same bookkeeping code.
 *   sdesc:    the solve's program (B is ignored: the batch is desc->P; return_full_W must be 0).
 *   yhat:     [n_steps, P, H, N] float32 forecasts of the steps (kmpc_rollout of their windows).
 *   realized: [n_steps, P, N] float32 log-returns of each step's t + 1; steps k >= n_real have none
 *             (realized_next = NULL in kmpc_backtest_step).
 *   weights [P,N] f64, value [P] f64, hist [P,S,4]: as kmpc_backtest_step, updated in place.
 *   target [P,N] f64, status [P] int, obj [P] f64: scratch (on return: the last step's W0, status,
 *             objective).
 * KMPC_ERR_UNSUPPORTED unless kmpc_solve would solve a batch of P such windows with a float64
 * register kernel of the constant case (no short, cost and cap) — one window per workgroup for
 * H = 10 or 5 and 32 < N <= 256 (the BASELINE C3 shape among them), or (ABI 0.6.0) the packed
 * kernels for N <= 32 and H = 2, 5 or 10 (BASELINE configs[0]'s 10 assets, H = 5: one path per
 * lane group, 64 / GL paths per wave) — and not the mixed pair, i.e. float64 for this batch size;
 * the caller then runs the lock-step loop. */
int kmpc_backtest_run(const kmpc_backtest_desc* desc, const kmpc_solve_desc* sdesc, int step0, int n_steps,
                      const float* yhat, const float* realized, int n_real, double* weights, double* value,
                      double* hist, double* target, int* status, double* obj, void* stream);

/* metrics [P,5]: Sharpe Ratio, Max Drawdown, Avg Turnover, Final Value, Total Return. */
int kmpc_backtest_metrics(const kmpc_backtest_desc* desc, const double* hist, double* metrics,
                          void* stream);

/* ---- mean-variance MPC: replaces solve_mpc_mean_variance (mpc.py:119-184) ------------------ */
/*
 * For each problem b:
 *   maximize_W  sum_t [ w_t . mu_t - gamma w_t' Sigma w_t ] - c sum_t ||w_t - w_{t-1}||_1
 *   s.t.        1' w_t = 1;  w_t >= 0 unless allow_short  (mpc.py:145-169; no turnover cap)
 * with w_{-1} = w_prev. mu [B,H,N] float64 (the reference passes predicted log-returns / the
 * Markowitz rolling mean as mu), Sigma [B,N,N] float64 (sigma_stride = N*N) or one shared [N,N]
 * (sigma_stride = 0). Outputs as kmpc_solve; failure fallback tile(w_prev), obj = NaN
 * (mpc.py:180-181). Shapes: H*N <= KMPC_MV_MAX_HN, H <= KMPC_MV_MAX_H. Past H*N = 128 the
 * dense Newton matrix leaves LDS for a workspace slab (kmpc_mv_workspace_bytes; use
 * kmpc_solve_mv_ws — kmpc_solve_mv, which has no workspace argument, then returns
 * KMPC_ERR_WORKSPACE).
 */
#define KMPC_MV_MAX_HN 1024
#define KMPC_MV_MAX_H  16
typedef struct kmpc_mv_desc {
    int    B, N, H;
    double gamma;          /* MPCConfig.gamma (risk aversion, mpc.py:20)        */
    double cost_coeff;     /* MPCConfig.cost_coeff                              */
    int    allow_short;    /* MPCConfig.allow_short                             */
    int    max_iter;       /* interior-point iteration cap (0 -> 100)           */
    double tol;            /* complementarity tolerance (<= 0 -> 1e-10)         */
    int    return_full_W;  /* 0: w_out [B,N] (W[0]); 1: [B,H,N]                  */
} kmpc_mv_desc;

int kmpc_solve_mv(const kmpc_mv_desc* desc,
                  const double* mu,        /* [B,H,N] */
                  const double* sigma,     /* [B,N,N] or [N,N] */
                  size_t sigma_stride,     /* elements between windows' Sigma (0: shared) */
                  const double* w_prev,    /* [B,N] */
                  double* w_out, int* status, double* obj, int* iters, void* stream);
/* kmpc_solve_mv with a caller-provided workspace of kmpc_mv_workspace_bytes(desc) bytes */
size_t kmpc_mv_workspace_bytes(const kmpc_mv_desc* desc);
int kmpc_solve_mv_ws(const kmpc_mv_desc* desc, const double* mu, const double* sigma, size_t sigma_stride,
                     const double* w_prev, double* w_out, int* status, double* obj, int* iters,
                     void* workspace, size_t ws_bytes, void* stream);

/* ---- Markowitz rolling moments: MarkowitzStrategy.rebalance (baselines.py:70-88) ------------ */
/* For window b at test row t = ts[b]: returns r_s = z_s * std + mean (float32, as
 * destandardize_returns, data_finance.py:740-742) of the standardized rows z [T, ldz] (first N
 * columns = extract_current_returns), s in the last `lookback` rows of [0, t]; mu[b] = mean
 * (rounded to float32 as the reference's float32 np.mean), sigma[b] = np.cov (ddof 1, float64)
 * + 1e-6 I; valid[b] = 1 when t + 1 >= 5 (else the strategy holds its weights). */
int kmpc_rolling_moments(int B, int T, int N, int lookback, const float* z, int ldz,
                         const float* mean, const float* std, const int* ts,
                         double* mu, double* sigma, int* valid, void* stream);

/* Workspace needed by kmpc_rollout / kmpc_solve / kmpc_window (either desc may be NULL; with both,
   the sum for kmpc_window: rollout scratch + yhat + the solve's). */
size_t kmpc_workspace_bytes(const kmpc_rollout_desc* rdesc, const kmpc_solve_desc* sdesc);

/* Human-readable text for a return code or (status + 100) for a per-problem status. */
const char* kmpc_strerror(int code);

/* Library version string, "kmpc <ABI> (gfx950)". ABI 0.2.0 appended kmpc_solve_desc.path and
   kmpc_rollout_desc.latent_unfused; 0.3.0 appended kmpc_solve_desc.precision and .mu_handoff:
   callers built against an older ABI must rebuild. 0.4.0 added enum values only
   (KMPC_PRECISION_MIXED, KMPC_DTYPE_F32_F32MFMA; AUTO precision now float64 below KMPC_MIXED_MIN_B
   windows; KMPC_DTYPE_F32's GEMMs on three bf16 planes), no layout change. 0.5.0 added a function
   (kmpc_backtest_run), no layout change. 0.6.0 added enum values only (KMPC_LATENT_SEQUENTIAL) and
   kmpc_backtest_run's packed shapes, no layout change. */
const char* kmpc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KMPC_H */
