// kmpc_bt_step.h — one step of run_backtest's bookkeeping for one path (backtest.py:173-217),
// shared by the lock-step kernel (kmpc_backtest.hip: bt_step_kernel, one launch per step) and the
// path-persistent backtest kernel (kmpc_solve_c3.hip: after each step's solve in the same
// workgroup). One code path, so the two are bit-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "kmpc_npexp.h"

namespace kmpc {
namespace bt {

__device__ __forceinline__ double block_sum_bt(double v, double* red) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wv] = v;
    __syncthreads();
    double s = 0.0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += red[q];
    return s;
}

struct StepArgs {
    int P, N, S, k;
    double c;
    const double* target;
    const float* realized;   // [P, N] log-returns of t + 1, or null
    double* w;
    double* value;
    double* hist;            // [P, S, 4]
};

// path p's step a.k; red: >= blockDim / 64 doubles of LDS. Every thread of the block calls it.
__device__ __forceinline__ void bt_step_body(const StepArgs& a, int p, double* red) {
    const double* tg = a.target + (size_t)p * a.N;
    double* w = a.w + (size_t)p * a.N;
    double tv = 0.0;
    for (int i = threadIdx.x; i < a.N; i += blockDim.x) tv += fabs(tg[i] - w[i]);
    const double turnover = block_sum_bt(tv, red);
    double value = a.value[p];
    const double cost = a.c * turnover * value;
    value -= cost;
    double port = 0.0;
    if (a.realized) {
        const float* y = a.realized + (size_t)p * a.N;
        double pv = 0.0;
        for (int i = threadIdx.x; i < a.N; i += blockDim.x) {
            const float r = np_expf(y[i]) - 1.0f;
            pv += tg[i] * (double)r;
        }
        port = block_sum_bt(pv, red);
        value *= (1.0 + port);
        double denom = 1.0 + port;
        if (fabs(denom) < 1e-8) denom = 1e-8;
        for (int i = threadIdx.x; i < a.N; i += blockDim.x) {
            const float g = 1.0f + (np_expf(y[i]) - 1.0f);
            w[i] = tg[i] * (double)g / denom;
        }
    } else {
        for (int i = threadIdx.x; i < a.N; i += blockDim.x) w[i] = tg[i];
    }
    if (threadIdx.x == 0) {
        a.value[p] = value;
        double* h = a.hist + ((size_t)p * a.S + a.k) * 4;
        h[0] = value;
        h[1] = port;
        h[2] = turnover;
        h[3] = cost;
    }
}

// The same step for a path on a GL-lane group of a packed wave (N <= GL, lane i owns asset i):
// the lock-step kernel's sums restricted to the group. There (one 64-lane wave for N <= 64) the
// butterfly levels at and above GL add exact zeros (lanes past N hold 0), and the levels below GL
// are these, in the same order; its total then starts from 0.0 — so the results are bit-identical
// to bt_step_body's (tests/test_backtest_gpu.py, persistent vs lock-step).
template <int GL>
__device__ __forceinline__ double group_sum_bt(double v) {
#pragma unroll
    for (int o = GL / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return 0.0 + v;
}

template <int GL>
__device__ __forceinline__ void bt_step_group(const StepArgs& a, int p, int i) {
    const double* tg = a.target + (size_t)p * a.N;
    double* w = a.w + (size_t)p * a.N;
    const bool on = i < a.N;
    const double tgi = on ? tg[i] : 0.0;
    const double wi = on ? w[i] : 0.0;
    const double turnover = group_sum_bt<GL>(on ? 0.0 + fabs(tgi - wi) : 0.0);
    double value = a.value[p];
    const double cost = a.c * turnover * value;
    value -= cost;
    double port = 0.0;
    if (a.realized) {
        const float y = on ? a.realized[(size_t)p * a.N + i] : 0.0f;
        const float r = np_expf(y) - 1.0f;
        port = group_sum_bt<GL>(on ? 0.0 + tgi * (double)r : 0.0);
        value *= (1.0 + port);
        double denom = 1.0 + port;
        if (fabs(denom) < 1e-8) denom = 1e-8;
        const float g = 1.0f + (np_expf(y) - 1.0f);
        if (on) w[i] = tgi * (double)g / denom;
    } else {
        if (on) w[i] = tgi;
    }
    if (i == 0) {
        a.value[p] = value;
        double* h = a.hist + ((size_t)p * a.S + a.k) * 4;
        h[0] = value;
        h[1] = port;
        h[2] = turnover;
        h[3] = cost;
    }
}

}  // namespace bt
}  // namespace kmpc
