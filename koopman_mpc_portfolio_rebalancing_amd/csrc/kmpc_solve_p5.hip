// kmpc_solve_p5.hip — packed (lane-group) ipm_kernel instantiations for H <= 5 (see
// kmpc_solve_kernel.h, launch_ipm_packed).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm_packed<2>(const SolveArgs& a, hipStream_t stream);
template int launch_ipm_packed<5>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc
