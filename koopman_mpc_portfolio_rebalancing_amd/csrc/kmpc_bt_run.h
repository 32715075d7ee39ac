// kmpc_bt_run.h — the path-persistent backtest kernel (kmpc_backtest_run; run_backtest,
// backtest.py:133-219, for P independent paths): one workgroup per path runs every step of its path
// back to back — the step's window solve (the body of ipm_kernel, kmpc_ipm_body.inc) then the
// step's bookkeeping (kmpc_bt_step.h, as kmpc_backtest_step) — with no launch and no lock step
// between steps: a path never waits for the slowest window of a batch. Instantiated next to the
// ipm_kernel it mirrors, in a unit with the same compile options (kmpc_solve_c3.hip for the C3
// kernel, kmpc_solve_hbt*.hip for the constant-case kernels of kmpc_solve_h*_case.hip).
#pragma once
#include "kmpc_solve_kernel.h"
#include "kmpc_bt_step.h"

namespace kmpc {

struct BtRun {
    int n_steps;             // steps run by this launch
    int n_real;              // steps k < n_real have a realized row (later ones: no market move)
    const float* yhat;       // [n_steps, P, H, N] forecasts
    const float* realized;   // [n_steps, P, N] log-returns of each step's t + 1
    bt::StepArgs st;         // bookkeeping: st.k = the first step's history row; st.target = W0 scratch
};

// One workgroup per path (window index b = path), or for the packed kernels (GL < 64: N <= 32)
// one GL-lane group per path, 64 / GL paths per one-wave workgroup. The per-step solve is the
// float64 kernel ipm_kernel<HM, MAXT, EXACT, FL, CS, QL, GL, 0> (the one kmpc_solve picks for a batch
// of P < KMPC_MIXED_MIN_B such windows), so every step's W0 matches the lock-step run's. The paths of
// one packed wave step together (a path whose window has converged waits, masked, for its wave's
// slowest), but never for the rest of the batch.
template <int HM, int MAXT, bool EXACT, int FL, int CS, bool QL, int GL, int PH>
__global__ void __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(HM <= KMPC_WPE2_HM ? 2 : 1)))
bt_run_kernel(SolveArgs a0, BtRun r) {
    static_assert(PH == 0, "float64 windows");
    static_assert(GL == 64 || MAXT == 64, "lane groups pack one-wave blocks");
    using Real = double;
    constexpr int NWM = MAXT / WAVE;
    constexpr int WPB = GL == 64 ? 1 : 64 / GL;   // paths per block
    __shared__ Shared<HM, NWM, Real> shv[WPB];
    __shared__ double red[NWM];
    auto& sh = shv[grp<GL>()];
    if constexpr (GL < 64) {
        if ((int)blockIdx.x * WPB + grp<GL>() >= a0.B) return;   // (whole groups of the last block)
    }
    const size_t PHN = (size_t)a0.B * a0.H * a0.N, PN = (size_t)a0.B * a0.N;
    for (int k = 0; k < r.n_steps; ++k) {
        {
            SolveArgs args = a0;
            args.yhat = r.yhat + k * PHN;
            // (laundering b and the argument fields every step — nothing derived from them hoisted
            // out of the loop — cut the scratch from 512 to 448 B per lane but ran slower: P = 64
            // 0.898 -> 0.913 ms per step, P = 1,024 1.92 -> 1.98 ms)
            const int b = blockIdx.x * WPB + grp<GL>();
#include "kmpc_ipm_body.inc"
        }
        __syncthreads();   // W0 (st.target) of every lane, and the solve's LDS, done
        bt::StepArgs st = r.st;
        st.k = r.st.k + k;
        st.realized = k < r.n_real ? r.realized + k * PN : nullptr;
        if constexpr (GL == 64)
            bt::bt_step_body(st, blockIdx.x, red);
        else
            bt::bt_step_group<GL>(st, blockIdx.x * WPB + grp<GL>(), gvt<GL>());
        __syncthreads();   // the drifted weights are the next solve's w_prev
    }
}


// the launch: a.B = paths, a.wout the [P, N] W0 scratch, a.status / a.obj [P] scratch
template <int HM, int MAXT, bool EXACT, int FL, int CS = MAXT, bool QL = false, int GL = 64>
int launch_bt_run_one(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
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
    const size_t lds = cold_bytes<HM, MAXT, CS, QL, GL, FL, double>();
    constexpr int WPB = GL == 64 ? 1 : 64 / GL;
    hipLaunchKernelGGL((bt_run_kernel<HM, MAXT, EXACT, FL, CS, QL, GL, 0>), dim3((a.B + WPB - 1) / WPB),
                       dim3(GL == 64 ? 64 * ((a.N + 63) / 64) : 64), lds, stream, s, r);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

// The packed shapes (launch_ipm_packed<HM>'s choice for case 7 with H = HM: N <= 32, 3 HM <= 32):
// KMPC_ERR_UNSUPPORTED elsewhere (a ragged H runs the generic packed kernel: no persistent form).
template <int HM>
int launch_bt_run_packed(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                         int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream) {
    const int fl = case_of(!a.allow_short, a.c > 0.0 || a.tau > 0.0, a.tau > 0.0);
    if (a.H != HM || a.N > 32 || 3 * HM > 32 || fl != 7) return KMPC_ERR_UNSUPPORTED;
#define KMPC_BT_ARGS a, n_steps, n_real, yhat, realized, step0, S, c, weights, value, hist, stream
    if constexpr (3 * HM <= 16) {
        if (a.N <= 16) {
            if (a.N <= KMPC_PACK_NS - 1) return launch_bt_run_one<HM, 64, true, 7, 4 * KMPC_PACK_NS, false, 16>(KMPC_BT_ARGS);
            return launch_bt_run_one<HM, 64, true, 7, 64, false, 16>(KMPC_BT_ARGS);
        }
    }
    if constexpr (3 * HM <= 32) return launch_bt_run_one<HM, 64, true, 7, 64, false, 32>(KMPC_BT_ARGS);
#undef KMPC_BT_ARGS
    return KMPC_ERR_UNSUPPORTED;
}

// The constant-case shapes (launch_ipm_case<HM>'s choice for case 7: no short + cost + cap, H = HM,
// N <= 256), except the C3 kernel's (kmpc_solve_c3.hip): KMPC_ERR_UNSUPPORTED elsewhere.
template <int HM>
int launch_bt_run_case(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                       int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream) {
    const int nt = WAVE * ((a.N + WAVE - 1) / WAVE);
    const int fl = case_of(!a.allow_short, a.c > 0.0 || a.tau > 0.0, a.tau > 0.0);
    if (a.H != HM || nt > 256 || fl != 7) return KMPC_ERR_UNSUPPORTED;
#define KMPC_BT_ARGS a, n_steps, n_real, yhat, realized, step0, S, c, weights, value, hist, stream
    if constexpr (HM == 10) {
        if (nt == 128 && a.N < QL_CS) return KMPC_ERR_UNSUPPORTED;   // (the C3 unit's)
        if (nt == 256 && a.N < QL_CS256) return launch_bt_run_one<HM, 256, true, 7, QL_CS256, true>(KMPC_BT_ARGS);
    }
    return nt <= 64 ? launch_bt_run_one<HM, 64, true, 7>(KMPC_BT_ARGS)
                    : (nt <= 128 ? launch_bt_run_one<HM, 128, true, 7>(KMPC_BT_ARGS)
                                 : launch_bt_run_one<HM, 256, true, 7>(KMPC_BT_ARGS));
#undef KMPC_BT_ARGS
}

}  // namespace kmpc
