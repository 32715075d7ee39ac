// kmpc_solve_c3.hip — the BASELINE C3 kernel (H = 10, no short + cost + cap, N < 104: 128 threads,
// the per-asset LDL^T arrays in LDS) in its own translation unit, built at -O2: measured 0.6% ahead
// of -Os for this kernel (bit-identical results), while the 256-thread variant of the constant-case
// unit loses 4% at -O2.
//
// Also the path-persistent backtest kernel (bt_run_c3_kernel): run_backtest (backtest.py:133-219)
// for P independent paths, one workgroup per path running every step of its path back to back —
// the step's solve (the same window body as ipm_kernel, kmpc_ipm_body.inc) then the bookkeeping
// (kmpc_bt_step.h, as kmpc_backtest_step) — with no launch and no lock step between steps: a path
// never waits for the slowest window of a batch.
#include "kmpc_solve_kernel.h"
#include "kmpc_bt_step.h"

namespace kmpc {
namespace {
// The mixed pair in one launch: each workgroup runs its window's float32 phase and then its float64
// finish (the same two window bodies as the PH = 1 / PH = 2 kernels, kmpc_ipm_body.inc), so the
// warm record is read back by the CU that wrote it and there is one launch tail instead of two.
template <int HM, int MAXT, bool EXACT, int FL, int CS, bool QL, int GL>
__global__ void __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(1))) ipm_mixed_kernel(SolveArgs args) {
    constexpr int NWM = MAXT / WAVE;
    __shared__ union U {
        Shared<HM, NWM, float> f;
        Shared<HM, NWM, double> d;
    } shu;
    const int b = blockIdx.x;
    if (b >= args.B) return;
    [&]() __attribute__((always_inline)) {
        constexpr int PH = 1;
        using Real = float;
        auto& sh = shu.f;
#include "kmpc_ipm_body.inc"
    }();
    __syncthreads();   // the window's record written by every lane; the LDS structure reused
    [&]() __attribute__((always_inline)) {
        constexpr int PH = 2;
        using Real = double;
        auto& sh = shu.d;
#include "kmpc_ipm_body.inc"
    }();
}
}  // namespace

#ifndef KMPC_MIXED_FUSED   // 1: the float32 phase and the float64 finish in one launch (ipm_mixed_kernel)
#define KMPC_MIXED_FUSED 1
#endif

int launch_ipm_c3(const SolveArgs& a, hipStream_t stream) {
    if (a.warm && KMPC_MIXED_FUSED) {
        const size_t lds = cold_bytes<10, 128, QL_CS, true, 64, 7, double>();
        hipLaunchKernelGGL((ipm_mixed_kernel<10, 128, true, 7, QL_CS, true, 64>), dim3(a.B), dim3(128), lds, stream, a);
        int rc = hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
        if (rc == KMPC_OK) rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 3>(a, 128, stream);
        return rc;
    }
    if (a.warm) {   // mixed precision: the float32 phase, then the float64 finish from its iterates
        int rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 1>(a, 128, stream);
        if (rc == KMPC_OK) rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 2>(a, 128, stream);
        // (the retry of warm starts that did not end optimal: most workgroups exit at once)
        if (rc == KMPC_OK) rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 3>(a, 128, stream);
        return rc;
    }
    return launch_one<10, 128, true, 7, QL_CS, true>(a, 128, stream);
}

namespace {

struct BtRun {
    int n_steps;             // steps run by this launch
    int n_real;              // steps k < n_real have a realized row (later ones: no market move)
    const float* yhat;       // [n_steps, P, H, N] forecasts
    const float* realized;   // [n_steps, P, N] log-returns of each step's t + 1
    bt::StepArgs st;         // bookkeeping: st.k = the first step's history row; st.target = W0 scratch
};

// One workgroup per path (window index b = path). The per-step solve is the float64 C3 kernel's
// (ipm_kernel<10, 128, true, 7, QL_CS, true, 64, 0>, the one kmpc_solve picks for a batch of
// P < KMPC_MIXED_MIN_B such windows), so every step's W0 is bit-identical to the lock-step run's.
template <int HM, int MAXT, bool EXACT, int FL, int CS, bool QL, int GL, int PH>
__global__ void __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(1))) bt_run_kernel(SolveArgs a0, BtRun r) {
    static_assert(PH == 0 && GL == 64, "float64 whole-wave windows");
    using Real = double;
    constexpr int NWM = MAXT / WAVE;
    __shared__ Shared<HM, NWM, Real> shv[1];
    __shared__ double red[NWM];
    auto& sh = shv[0];
    const size_t PHN = (size_t)a0.B * a0.H * a0.N, PN = (size_t)a0.B * a0.N;
    for (int k = 0; k < r.n_steps; ++k) {
        {
            SolveArgs args = a0;
            args.yhat = r.yhat + k * PHN;
            // (laundering b and the argument fields every step — nothing derived from them hoisted
            // out of the loop — cut the scratch from 512 to 448 B per lane but ran slower: P = 64
            // 0.898 -> 0.913 ms per step, P = 1,024 1.92 -> 1.98 ms)
            const int b = blockIdx.x;
#include "kmpc_ipm_body.inc"
        }
        __syncthreads();   // W0 (st.target) of every lane, and the solve's LDS, done
        bt::StepArgs st = r.st;
        st.k = r.st.k + k;
        st.realized = k < r.n_real ? r.realized + k * PN : nullptr;
        bt::bt_step_body(st, blockIdx.x, red);
        __syncthreads();   // the drifted weights are the next solve's w_prev
    }
}

}  // namespace

int launch_bt_run_c3(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                     int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream) {
    BtRun r;
    r.n_steps = n_steps;
    r.n_real = n_real;
    r.yhat = yhat;
    r.realized = realized;
    r.st.P = a.B; r.st.N = a.N; r.st.S = S; r.st.k = step0; r.st.c = c;
    r.st.target = a.wout; r.st.realized = nullptr; r.st.w = weights; r.st.value = value; r.st.hist = hist;
    SolveArgs s = a;
    s.wp = weights;   // each step's w_prev: the path's current (drifted) weights
    const size_t lds = cold_bytes<10, 128, QL_CS, true, 64, 7, double>();
    hipLaunchKernelGGL((bt_run_kernel<10, 128, true, 7, QL_CS, true, 64, 0>), dim3(a.B), dim3(128), lds, stream, s, r);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}
}  // namespace kmpc

#ifdef KMPC_STATS
extern "C" int kmpc_debug_stats_c3(unsigned long long* out, int reset) { return kmpc::debug_stats_tu(out, reset); }
#endif
