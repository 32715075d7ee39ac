// kmpc_solve_hbt5.hip — the path-persistent backtest kernels (kmpc_bt_run.h) of the H = 5
// constant-case ipm_kernel shapes (kmpc_solve_h5_case.hip), built with the same options as that unit.
#include "kmpc_bt_run.h"

namespace kmpc {
template int launch_bt_run_case<5>(const SolveArgs& a, int n_steps, int n_real, const float* yhat,
                                    const float* realized, int step0, int S, double c, double* weights,
                                    double* value, double* hist, hipStream_t stream);
}  // namespace kmpc
