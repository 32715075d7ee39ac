// kmpc_backtest.hip — lock-step backtest bookkeeping for P independent paths on the device
// (reference run_backtest / calculate_metrics, backtest.py:133-249).
//
// One step of run_backtest per path (backtest.py:173-217), after the window solve produced the
// target weights:
//   turnover = |target - w|_1;  cost = c * turnover * value;  value -= cost;  w = target
//   r = np.exp(y_{t+1}) - 1  (float32: numpy's float32 exp, np_expf, then a float32 subtraction)
//   port = w . r;  value *= 1 + port;  w = w * (1 + r) / guard(1 + port)   (|.| < 1e-8 -> 1e-8)
// and the row (value, return, turnover, cost) of the history. The metrics kernel then reduces each
// path's history exactly as calculate_metrics (population std Sharpe, drawdown on cumprod(1+r),
// mean turnover, final value, total return relative to the first row).
//
// Memory-bound byte work: one workgroup per path streams its N weights once per step (target and
// weights f64, returns f32) — ~20N bytes per path-step; the metrics kernel streams the history.
#include <hip/hip_runtime.h>
#include <math.h>

#include "kmpc_internal.h"
#include "kmpc_npexp.h"
#include "kmpc_bt_step.h"

namespace kmpc {

namespace {

constexpr int BT_THREADS = 256;
using bt::StepArgs;

__global__ void __launch_bounds__(BT_THREADS) bt_step_kernel(StepArgs a) {
    __shared__ double red[BT_THREADS / 64];
    bt::bt_step_body(a, blockIdx.x, red);
}

// one thread per path; the history rows are read in step order (calculate_metrics)
__global__ void bt_metrics_kernel(int P, int S, const double* hist, double* m) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const double* h = hist + (size_t)p * S * 4;
    double* o = m + (size_t)p * 5;
    if (S == 0) {
        for (int j = 0; j < 5; ++j) o[j] = __builtin_nan("");
        return;
    }
    double sr = 0.0, st = 0.0;
    for (int k = 0; k < S; ++k) { sr += h[k * 4 + 1]; st += h[k * 4 + 2]; }
    const double mean = sr / S;
    double var = 0.0, cum = 1.0, peak = 0.0, mdd = 0.0;
    for (int k = 0; k < S; ++k) {
        const double r = h[k * 4 + 1];
        var += (r - mean) * (r - mean);
        cum *= (1.0 + r);
        peak = (k == 0) ? cum : fmax(peak, cum);   // np.maximum.accumulate(cumprod(1 + r))
        const double dd = (cum - peak) / peak;
        mdd = (k == 0) ? dd : fmin(mdd, dd);
    }
    const double sd = sqrt(var / S);
    o[0] = sqrt(252.0) * mean / (sd + 1e-8);
    o[1] = mdd;
    o[2] = st / S;
    o[3] = h[(S - 1) * 4 + 0];
    o[4] = h[(S - 1) * 4 + 0] / h[0] - 1.0;
}

__global__ void gross_returns_kernel(size_t n, const float* __restrict__ y, float* __restrict__ R) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        R[i] = np_expf(y[i]);
}

}  // namespace

int gross_returns_launch(size_t n, const float* yhat, float* R, hipStream_t stream) {
    const size_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(gross_returns_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, stream,
                       n, yhat, R);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

int backtest_step_launch(const kmpc_backtest_desc* d, int step, const double* target,
                         const float* realized_next, double* weights, double* value, double* hist,
                         hipStream_t stream) {
    StepArgs a;
    a.P = d->P; a.N = d->N; a.S = d->S; a.k = step; a.c = d->cost_coeff;
    a.target = target; a.realized = realized_next; a.w = weights; a.value = value; a.hist = hist;
    if (a.P == 0) return KMPC_OK;
    const int nt = a.N >= BT_THREADS ? BT_THREADS : 64 * ((a.N + 63) / 64);
    hipLaunchKernelGGL(bt_step_kernel, dim3(a.P), dim3(nt), 0, stream, a);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

int backtest_metrics_launch(const kmpc_backtest_desc* d, const double* hist, double* metrics,
                            hipStream_t stream) {
    if (d->P == 0) return KMPC_OK;
    hipLaunchKernelGGL(bt_metrics_kernel, dim3((d->P + 255) / 256), dim3(256), 0, stream, d->P, d->S,
                       hist, metrics);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

}  // namespace kmpc
