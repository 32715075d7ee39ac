// kmpc_solve_h10.hip — ipm_kernel instantiations for horizons H <= 10 (see kmpc_solve_kernel.h).
#include "kmpc_solve_kernel.h"

namespace kmpc {
template int launch_ipm<10>(const SolveArgs& a, hipStream_t stream);
}  // namespace kmpc

#ifdef KMPC_STATS
// dev builds only (tools/phase_stats.py): out[0..1] = refinement steps, Newton solves;
// out[2..17] = s_memtime cycles per solver phase. reset != 0 zeroes the counters afterwards.
extern "C" int kmpc_debug_stats(unsigned long long* out, int reset) {
    unsigned long long h[18];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(kmpc::g_stats), sizeof(unsigned long long) * 2) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(h + 2, HIP_SYMBOL(kmpc::g_phase), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    for (int k = 0; k < 18; ++k) out[k] = h[k];
    if (reset) {
        const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(kmpc::g_stats), z, sizeof(unsigned long long) * 2) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(kmpc::g_phase), z, sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    }
    return 0;
}
#endif
