// kmpc_internal.h — launch entry points shared by the kernels and the C ABI (kmpc_capi.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/kmpc.h"

namespace kmpc {

// kmpc_solve.hip
size_t solve_workspace_bytes(const kmpc_solve_desc* d);
int solve_launch(const kmpc_solve_desc* d, const float* yhat, const double* w_prev, double* w_out,
                 int* status, double* obj, int* iters, void* ws, size_t ws_bytes, hipStream_t stream,
                 double* trace = nullptr);

int backtest_run_launch(const kmpc_backtest_desc* bd, const kmpc_solve_desc* sd, int step0, int n_steps,
                        const float* yhat, const float* realized, int n_real, double* weights, double* value,
                        double* hist, double* target, int* status, double* obj, hipStream_t stream);

// kmpc_backtest.hip
int gross_returns_launch(size_t n, const float* yhat, float* R, hipStream_t stream);
int backtest_step_launch(const kmpc_backtest_desc* d, int step, const double* target,
                         const float* realized_next, double* weights, double* value, double* hist,
                         hipStream_t stream);
int backtest_metrics_launch(const kmpc_backtest_desc* d, const double* hist, double* metrics,
                            hipStream_t stream);

// kmpc_rollout.hip
size_t rollout_workspace_bytes(const kmpc_rollout_desc* d);
int rollout_launch(const kmpc_rollout_desc* d, const float* obs, float* yhat, void* ws,
                   size_t ws_bytes, hipStream_t stream);
int standardize_launch(int T, int N, const double* y, const double* mean, const double* stdv, float* z,
                       hipStream_t stream);

// kmpc_mv.hip
size_t mv_lds_bytes(int N, int H);
size_t mv_workspace_bytes(const kmpc_mv_desc* d);
int mv_solve_launch(const kmpc_mv_desc* d, const double* mu, const double* sigma, size_t sigma_stride,
                    const double* w_prev, double* w_out, int* status, double* obj, int* iters,
                    void* ws, size_t ws_bytes, hipStream_t stream);
int rolling_moments_launch(int B, int T, int N, int lookback, const float* z, int ldz, const float* mean,
                           const float* stdv, const int* ts, double* mu, double* sigma, int* valid,
                           hipStream_t stream);

}  // namespace kmpc
