// kmpc_solve_big.hip — large-window solve kernel instantiations (see kmpc_solve_big.h):
// HM = 10 (H <= 10) and HM = 21 (H <= 21), each for the runtime constraint case and case 7
// (no short + cost + cap).
#include "kmpc_solve_big.h"

namespace kmpc {

size_t big_ws_bytes(const SolveArgs& a) {
    return a.H <= 10 ? big::ws_bytes<10>(a) : big::ws_bytes<21>(a);
}

int big_launch(const SolveArgs& a, void* ws, size_t ws_size, hipStream_t stream) {
    return a.H <= 10 ? big::launch<10>(a, ws, ws_size, stream) : big::launch<21>(a, ws, ws_size, stream);
}

}  // namespace kmpc
