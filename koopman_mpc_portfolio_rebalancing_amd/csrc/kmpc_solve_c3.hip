// kmpc_solve_c3.hip — the BASELINE C3 kernel (H = 10, no short + cost + cap, N < 104: 128 threads,
// the per-asset LDL^T arrays in LDS) in its own translation unit, built at -O2: measured 0.6% ahead
// of -Os for this kernel (bit-identical results), while the 256-thread variant of the constant-case
// unit loses 4% at -O2.
#include "kmpc_solve_kernel.h"

namespace kmpc {
int launch_ipm_c3(const SolveArgs& a, hipStream_t stream) {
    if (a.warm) {   // mixed precision: the float32 phase, then the float64 finish from its iterates
        int rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 1>(a, 128, stream);
        if (rc == KMPC_OK) rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 2>(a, 128, stream);
        // (the retry of warm starts that did not end optimal: most workgroups exit at once)
        if (rc == KMPC_OK) rc = launch_one<10, 128, true, 7, QL_CS, true, 64, 3>(a, 128, stream);
        return rc;
    }
    return launch_one<10, 128, true, 7, QL_CS, true>(a, 128, stream);
}
}  // namespace kmpc

#ifdef KMPC_STATS
extern "C" int kmpc_debug_stats_c3(unsigned long long* out, int reset) { return kmpc::debug_stats_tu(out, reset); }
#endif
