// kmpc_solve_c3.hip — the BASELINE C3 kernel (H = 10, no short + cost + cap, N < 104: 128 threads,
// the per-asset LDL^T arrays in LDS) in its own translation unit, built at -O2: measured 0.6% ahead
// of -Os for this kernel (bit-identical results), while the 256-thread variant of the constant-case
// unit loses 4% at -O2.
//
// Also the path-persistent backtest kernel of this shape (kmpc_bt_run.h, kmpc_backtest_run).
#include "kmpc_solve_kernel.h"
#include "kmpc_bt_run.h"

#ifndef KMPC_REG_HANDOFF_ON   // ipm_mixed_kernel's handoff: 2 LDS, 1 registers, 0 the warm record in HBM
#define KMPC_REG_HANDOFF_ON 1
#endif

namespace kmpc {
// the handoff's LDS slot of this lane (as the cold arrays: lanes past CS - 1 share its slot, an
// inactive asset whose values are never read)
template <int CS>
__device__ __forceinline__ int hand_lane() { const int t = (int)threadIdx.x; return t < CS ? t : CS - 1; }
}

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
#if KMPC_REG_HANDOFF_ON
    // the float32 phase's iterate handed to the float64 finish on chip, not
    // through the 20 KB warm record in HBM: each lane's w, s, l1..l3 for its asset and the period
    // owners' z4, l4, nu — in the finish's cold-array LDS (2, the default: free during the float32
    // phase) or in registers (1: live across the phase boundary; 12 more spilled VGPRs in the finish)
    static_assert(KMPC_REG_HANDOFF_ON != 2 || (5 * HM * CS + 3 * HM) * 4 <= cold_bytes<HM, MAXT, CS, QL, GL, FL, double>(),
                  "the handoff fits the float64 cold arrays' LDS");
#if KMPC_REG_HANDOFF_ON == 1
    float hand_w[HM], hand_s[HM], hand_l1[HM], hand_l2[HM], hand_l3[HM];
    float hand_z4 = 1.0f, hand_l4 = 0.0f, hand_nu = 0.0f;
#endif
    bool hand_flag = false;
#define KMPC_REG_HANDOFF
#endif
    [&]() __attribute__((always_inline)) {
        constexpr int PH = 1;
        using Real = float;
        auto& sh = shu.f;
#include "kmpc_ipm_body.inc"
    }();
    __syncthreads();   // the window's header written; the LDS structure reused
    [&]() __attribute__((always_inline)) {
        constexpr int PH = 2;
        using Real = double;
        auto& sh = shu.d;
#include "kmpc_ipm_body.inc"
    }();
#undef KMPC_REG_HANDOFF
}
}  // namespace

#ifndef KMPC_MIXED_FUSED   // 1: the float32 phase and the float64 finish in one launch (ipm_mixed_kernel)
#define KMPC_MIXED_FUSED 1
#endif

size_t mixed_warm_floats(int H, int N) {
    return KMPC_MIXED_FUSED && KMPC_REG_HANDOFF_ON ? (size_t)WARM_HEAD : warm_stride(H, N);
}

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

int launch_bt_run_c3(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                     int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream) {
    return launch_bt_run_one<10, 128, true, 7, QL_CS, true>(a, n_steps, n_real, yhat, realized, step0, S, c, weights,
                                                           value, hist, stream);
}
}  // namespace kmpc

#ifdef KMPC_STATS
extern "C" int kmpc_debug_stats_c3(unsigned long long* out, int reset) { return kmpc::debug_stats_tu(out, reset); }
#endif
