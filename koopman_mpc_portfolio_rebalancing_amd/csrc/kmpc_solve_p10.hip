// kmpc_solve_p10.hip — packed (lane-group) ipm_kernel instantiations for H <= 10 (see
// kmpc_solve_kernel.h, launch_ipm_packed).
#include "kmpc_solve_kernel.h"
#include "kmpc_bt_run.h"

namespace kmpc {
template int launch_ipm_packed<10>(const SolveArgs& a, hipStream_t stream);
// the path-persistent backtest kernels of the packed shapes (kmpc_bt_run.h)
template int launch_bt_run_packed<10>(const SolveArgs& a, int n_steps, int n_real, const float* yhat,
                                      const float* realized, int step0, int S, double c, double* weights,
                                      double* value, double* hist, hipStream_t stream);
}  // namespace kmpc
