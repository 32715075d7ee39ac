// kmpc_solve_h2.hip — ipm_kernel instantiations for horizons H <= 2 (see kmpc_solve_kernel.h).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm<2>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc
