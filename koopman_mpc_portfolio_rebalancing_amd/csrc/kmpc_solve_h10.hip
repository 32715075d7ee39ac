// kmpc_solve_h10.hip — ipm_kernel instantiations for horizons H <= 10 (see kmpc_solve_kernel.h).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm<10>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc


