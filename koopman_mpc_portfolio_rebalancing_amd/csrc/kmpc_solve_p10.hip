// kmpc_solve_p10.hip — packed (lane-group) ipm_kernel instantiations for H <= 10 (see
// kmpc_solve_kernel.h, launch_ipm_packed).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm_packed<10>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc
