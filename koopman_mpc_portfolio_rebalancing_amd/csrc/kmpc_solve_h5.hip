// kmpc_solve_h5.hip — ipm_kernel instantiations for horizons H <= 5 (see kmpc_solve_kernel.h).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm<5>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc
