// kmpc_solve_args.h — arguments of the batched MPC solve kernel and its per-horizon launchers.
#pragma once
#include <hip/hip_runtime.h>

namespace kmpc {

struct SolveArgs {
    int B, N, H;
    double c, tau;
    int allow_short, max_iter, return_full, n_refine;
    int path;        // kmpc_solve_desc.path (KMPC_PATH_*)
    double tol;
    const float* yhat;
    const double* wp;
    double* wout;
    int* status;
    double* obj;
    int* iters;
    double* trace;   // debug: per-iteration (mu, rd, pr, step) of problem 0, or null
    // mixed precision (kmpc_solve_kernel.h, PH = 1 / 2): one warm record per window, or null
    float* warm;
    size_t warm_floats;   // floats per window in warm (mixed_warm_floats)
    double mu_handoff;   // the float32 phase hands its iterate over at mu <= mu_handoff
};

// A period whose gross returns R = np.exp(yhat) sum below this is solved on R / sum(R) (the same
// program up to the constant log sum(R); 1 + m = R would lose R's digits): every kernel and the oracle
constexpr double TINY_PERIOD = 0x1p-16;

// Warm record of one window: int flag (1 = warm iterate, 0 = cold: start over), int float32
// iterations, padding to WARM_HEAD floats, then w, s, l1, l2, l3 as [5][H][N] and z4, l4, nu as
// [3][H] (float32), padded to 64 B.
constexpr int WARM_HEAD = 16;
__host__ __device__ inline size_t warm_stride(int H, int N) {
    return ((size_t)WARM_HEAD + 5 * (size_t)H * N + 3 * (size_t)H + 15) / 16 * 16;
}
// ... of the C3 mixed launcher (kmpc_solve_c3.hip): the header alone when its fused kernel hands
// the iterate over on chip (the default), the whole record otherwise
size_t mixed_warm_floats(int H, int N);

constexpr int QL_CS = 104;     // cold-array stride of the 128-thread QL variant (N < QL_CS assets)

// ipm_kernel launchers, one translation unit per compile-time horizon bound HM (kmpc_solve_h*.hip)
template <int HM>
int launch_ipm(const SolveArgs& a, hipStream_t stream);
// large-window kernel (kmpc_solve_big.hip): workspace it needs, and the launch
size_t big_ws_bytes(const SolveArgs& a);
int big_launch(const SolveArgs& a, void* ws, size_t ws_size, hipStream_t stream);
// constant-case kernels (kmpc_solve_h*_case.hip); KMPC_ERR_UNSUPPORTED if the case has none
template <int HM>
int launch_ipm_case(const SolveArgs& a, hipStream_t stream);
// the C3 kernel (H = 10, FL = 7, 128 threads, LDL^T arrays in LDS) in its own -O2 unit (kmpc_solve_c3.hip)
int launch_ipm_c3(const SolveArgs& a, hipStream_t stream);
// the path-persistent backtest kernel of the C3 shape (kmpc_solve_c3.hip): a.B = paths, a.wout the
// [P, N] W0 scratch, a.status / a.obj [P] scratch; n_steps steps from history row step0
int launch_bt_run_c3(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                     int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream);
// ... and of the constant-case shapes H = HM (kmpc_solve_hbt*.hip); KMPC_ERR_UNSUPPORTED elsewhere
template <int HM>
int launch_bt_run_case(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                       int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream);
// ... and of the packed shapes (N <= 32, H = HM, one lane group per path; kmpc_solve_p*.hip)
template <int HM>
int launch_bt_run_packed(const SolveArgs& a, int n_steps, int n_real, const float* yhat, const float* realized,
                         int step0, int S, double c, double* weights, double* value, double* hist, hipStream_t stream);
// packed small-window kernels, 64 / GL windows per wave (kmpc_solve_p*.hip); KMPC_ERR_UNSUPPORTED
// outside N <= 32, 3 H <= 32
template <int HM>
int launch_ipm_packed(const SolveArgs& a, hipStream_t stream);

}  // namespace kmpc
