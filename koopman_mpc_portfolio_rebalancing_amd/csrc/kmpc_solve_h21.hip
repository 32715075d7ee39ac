// kmpc_solve_h21.hip — ipm_kernel instantiations for horizons H <= 21 (see kmpc_solve_kernel.h).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm<21>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc
