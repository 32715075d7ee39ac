// kmpc_solve_h10_case.hip — constant-case ipm_kernel instantiations for H == 10 (see
// kmpc_solve_kernel.h, launch_ipm_case).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm_case<10>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc

#ifdef KMPC_STATS
extern "C" int kmpc_debug_stats_case(unsigned long long* out, int reset) { return kmpc::debug_stats_tu(out, reset); }
#endif
