// kmpc_capi.hip — the extern "C" boundary of libkmpc.so (declared in include/kmpc.h).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kmpc_internal.h"

namespace {

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int check_solve(const kmpc_solve_desc* d) {
    if (!d) return KMPC_ERR_INVALID;
    if (d->B < 0 || d->N < 1 || d->H < 1) return KMPC_ERR_INVALID;
    if (d->N > KMPC_MAX_N || d->H > KMPC_MAX_H) return KMPC_ERR_UNSUPPORTED;
    if (d->H > 21) return KMPC_ERR_UNSUPPORTED;   // Schur system (3H) must fit one wavefront
    // c < 0 makes -c ||dw||_1 concave in the maximization: not DCP, cvxpy raises (mpc.py:66-103)
    if (d->cost_coeff < 0.0) return KMPC_ERR_INVALID;
    if (d->path < KMPC_PATH_AUTO || d->path > KMPC_PATH_REGISTER_UNPACKED) return KMPC_ERR_INVALID;
    if (d->precision < KMPC_PRECISION_AUTO || d->precision > KMPC_PRECISION_MIXED) return KMPC_ERR_INVALID;
    if (!(d->mu_handoff < 1.0)) return KMPC_ERR_INVALID;   // (NaN too)
    return KMPC_OK;
}

}  // namespace

extern "C" {

const char* kmpc_version(void) { return "kmpc 0.6.0 (gfx950)"; }

const char* kmpc_strerror(int code) {
    switch (code) {
        case KMPC_OK: return "ok";
        case KMPC_ERR_INVALID: return "invalid argument";
        case KMPC_ERR_UNSUPPORTED: return "unsupported shape";
        case KMPC_ERR_WORKSPACE: return "workspace too small";
        case KMPC_ERR_LAUNCH: return "HIP launch failed";
        case 100 + KMPC_STATUS_OPTIMAL: return "optimal";
        case 100 + KMPC_STATUS_OPTIMAL_INACCURATE: return "optimal_inaccurate";
        case 100 + KMPC_STATUS_INFEASIBLE: return "infeasible";
        case 100 + KMPC_STATUS_UNBOUNDED: return "unbounded";
        case 100 + KMPC_STATUS_SOLVER_ERROR: return "solver_error";
        default: return "unknown";
    }
}

size_t kmpc_workspace_bytes(const kmpc_rollout_desc* rdesc, const kmpc_solve_desc* sdesc) {
    size_t bytes = 0;
    if (rdesc) bytes += kmpc::rollout_workspace_bytes(rdesc);
    if (rdesc && sdesc) bytes += align256(sizeof(float) * (size_t)rdesc->B * rdesc->H * rdesc->N);
    if (sdesc && check_solve(sdesc) == KMPC_OK) bytes += align256(kmpc::solve_workspace_bytes(sdesc));
    return bytes;
}

int kmpc_solve(const kmpc_solve_desc* desc, const float* yhat, const double* w_prev, double* w_out,
               int* status, double* obj, int* iters, void* workspace, size_t ws_bytes,
               void* stream) {
    int rc = check_solve(desc);
    if (rc) return rc;
    if (desc->B == 0) return KMPC_OK;
    if (!yhat || !w_prev || !w_out || !status || !obj) return KMPC_ERR_INVALID;
    if (ws_bytes < kmpc::solve_workspace_bytes(desc)) return KMPC_ERR_WORKSPACE;
    return kmpc::solve_launch(desc, yhat, w_prev, w_out, status, obj, iters, workspace, ws_bytes,
                              (hipStream_t)stream);
}

/* Debug entry (not part of include/kmpc.h): kmpc_solve plus a per-iteration trace of problem 0,
   trace[4 * it + {0,1,2,3}] = (mu, dual residual, primal residual, step length). */
int kmpc_solve_trace(const kmpc_solve_desc* desc, const float* yhat, const double* w_prev,
                     double* w_out, int* status, double* obj, int* iters, double* trace,
                     void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_solve(desc);
    if (rc) return rc;
    if (desc->B == 0) return KMPC_OK;
    if (ws_bytes < kmpc::solve_workspace_bytes(desc)) return KMPC_ERR_WORKSPACE;
    return kmpc::solve_launch(desc, yhat, w_prev, w_out, status, obj, iters, workspace, ws_bytes,
                              (hipStream_t)stream, trace);
}

int kmpc_rollout(const kmpc_rollout_desc* desc, const float* obs, float* yhat, void* workspace,
                 size_t ws_bytes, void* stream) {
    return kmpc::rollout_launch(desc, obs, yhat, workspace, ws_bytes, (hipStream_t)stream);
}

int kmpc_window(const kmpc_rollout_desc* rdesc, const kmpc_solve_desc* sdesc, const float* obs,
                const double* w_prev, float* yhat, double* w_out, int* status, double* obj,
                int* iters, void* workspace, size_t ws_bytes, void* stream) {
    if (!rdesc || !sdesc) return KMPC_ERR_INVALID;
    int rc = check_solve(sdesc);
    if (rc) return rc;
    if (rdesc->B != sdesc->B || rdesc->N != sdesc->N || rdesc->H != sdesc->H) return KMPC_ERR_INVALID;
    if (ws_bytes < kmpc_workspace_bytes(rdesc, sdesc)) return KMPC_ERR_WORKSPACE;
    const size_t rbytes = kmpc::rollout_workspace_bytes(rdesc);
    const size_t ybytes = align256(sizeof(float) * (size_t)rdesc->B * rdesc->H * rdesc->N);
    float* y = yhat ? yhat : (float*)((char*)workspace + rbytes);
    rc = kmpc::rollout_launch(rdesc, obs, y, workspace, rbytes, (hipStream_t)stream);
    if (rc) return rc;
    if (sdesc->B == 0) return KMPC_OK;
    return kmpc::solve_launch(sdesc, y, w_prev, w_out, status, obj, iters, (char*)workspace + rbytes + ybytes,
                              ws_bytes - rbytes - ybytes, (hipStream_t)stream);
}

int kmpc_gross_returns(size_t n, const float* yhat, float* R, void* stream) {
    if (n == 0) return KMPC_OK;
    if (!yhat || !R) return KMPC_ERR_INVALID;
    return kmpc::gross_returns_launch(n, yhat, R, (hipStream_t)stream);
}

}  // extern "C"

extern "C" {

int kmpc_backtest_step(const kmpc_backtest_desc* desc, int step, const double* target,
                       const float* realized_next, double* weights, double* value, double* hist,
                       void* stream) {
    if (!desc || desc->P < 0 || desc->N < 1 || desc->S < 1 || step < 0 || step >= desc->S)
        return KMPC_ERR_INVALID;
    if (desc->P > 0 && (!target || !weights || !value || !hist)) return KMPC_ERR_INVALID;
    return kmpc::backtest_step_launch(desc, step, target, realized_next, weights, value, hist,
                                      (hipStream_t)stream);
}

int kmpc_backtest_run(const kmpc_backtest_desc* desc, const kmpc_solve_desc* sdesc, int step0, int n_steps,
                      const float* yhat, const float* realized, int n_real, double* weights, double* value,
                      double* hist, double* target, int* status, double* obj, void* stream) {
    if (!desc || !sdesc || desc->P < 0 || desc->N < 1 || desc->S < 1 || step0 < 0 || n_steps < 0 ||
        step0 + n_steps > desc->S || n_real < 0 || n_real > n_steps || sdesc->N != desc->N)
        return KMPC_ERR_INVALID;
    kmpc_solve_desc sd = *sdesc;   // (the batch is the paths)
    sd.B = desc->P;
    const int rc = check_solve(&sd);
    if (rc) return rc;
    if (desc->P > 0 && n_steps > 0 &&
        (!yhat || !weights || !value || !hist || !target || !status || !obj || (n_real > 0 && !realized)))
        return KMPC_ERR_INVALID;
    return kmpc::backtest_run_launch(desc, &sd, step0, n_steps, yhat, realized, n_real, weights, value, hist,
                                     target, status, obj, (hipStream_t)stream);
}

int kmpc_standardize(int T, int N, const double* log_returns, const double* mean, const double* std,
                     float* z, void* stream) {
    if (T < 0 || N < 1) return KMPC_ERR_INVALID;
    if ((size_t)T * N > 0 && (!log_returns || !mean || !std || !z)) return KMPC_ERR_INVALID;
    return kmpc::standardize_launch(T, N, log_returns, mean, std, z, (hipStream_t)stream);
}

int kmpc_backtest_metrics(const kmpc_backtest_desc* desc, const double* hist, double* metrics,
                          void* stream) {
    if (!desc || desc->P < 0 || desc->S < 0) return KMPC_ERR_INVALID;
    if (desc->P > 0 && (!hist || !metrics)) return KMPC_ERR_INVALID;
    return kmpc::backtest_metrics_launch(desc, hist, metrics, (hipStream_t)stream);
}

}  // extern "C"

extern "C" {

int kmpc_solve_mv(const kmpc_mv_desc* desc, const double* mu, const double* sigma, size_t sigma_stride,
                  const double* w_prev, double* w_out, int* status, double* obj, int* iters,
                  void* stream) {
    return kmpc_solve_mv_ws(desc, mu, sigma, sigma_stride, w_prev, w_out, status, obj, iters, nullptr, 0,
                            stream);
}

size_t kmpc_mv_workspace_bytes(const kmpc_mv_desc* desc) { return kmpc::mv_workspace_bytes(desc); }

int kmpc_solve_mv_ws(const kmpc_mv_desc* desc, const double* mu, const double* sigma, size_t sigma_stride,
                     const double* w_prev, double* w_out, int* status, double* obj, int* iters,
                     void* workspace, size_t ws_bytes, void* stream) {
    if (!desc || desc->B < 0 || desc->N < 1 || desc->H < 1) return KMPC_ERR_INVALID;
    if (desc->H > KMPC_MV_MAX_H || desc->N * desc->H > KMPC_MV_MAX_HN) return KMPC_ERR_UNSUPPORTED;
    if (desc->B == 0) return KMPC_OK;
    if (!mu || !sigma || !w_prev || !w_out || !status || !obj) return KMPC_ERR_INVALID;
    return kmpc::mv_solve_launch(desc, mu, sigma, sigma_stride, w_prev, w_out, status, obj, iters, workspace,
                                 ws_bytes, (hipStream_t)stream);
}

int kmpc_rolling_moments(int B, int T, int N, int lookback, const float* z, int ldz,
                         const float* mean, const float* std, const int* ts,
                         double* mu, double* sigma, int* valid, void* stream) {
    if (B < 0 || T < 0 || N < 1 || lookback < 1 || ldz < N) return KMPC_ERR_INVALID;
    if (B == 0) return KMPC_OK;
    if (!z || !mean || !std || !ts || !mu || !sigma || !valid) return KMPC_ERR_INVALID;
    return kmpc::rolling_moments_launch(B, T, N, lookback, z, ldz, mean, std, ts, mu, sigma, valid,
                                        (hipStream_t)stream);
}

}  // extern "C"
