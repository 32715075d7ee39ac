// kmpc_solve.hip — host dispatch of the batched MPC solve (replaces solve_mpc_log_utility,
// mpc.py:27-117). Two kernel families solve the same program with the same interior point:
//   ipm_kernel (kmpc_solve_kernel.h): a window's state in the registers of one workgroup, one
//     asset per lane — for N <= 256 assets and H <= 10 periods; each horizon
//     bound HM is instantiated in its own translation unit (kmpc_solve_h*.hip).
//   ipm_big (kmpc_solve_big.h): the state in a workspace slab, streamed per phase, the Schur
//     matrix on the f64 MFMA — for larger windows (N > 256 or H > 10), which need workspace.
#include "kmpc_internal.h"
#include "kmpc_solve_args.h"

namespace kmpc {

namespace {

// solver path override (debug entry kmpc_debug_solver_path, tools/ A/B only): 0 = by shape,
// 1 = register kernels whenever they support the shape, 2 = the large-window kernel
int g_path = 0;

SolveArgs make_args(const kmpc_solve_desc* d) {
    SolveArgs a;
    a.B = d->B; a.N = d->N; a.H = d->H;
    a.c = d->cost_coeff;
    a.tau = d->max_turnover > 0.0 ? d->max_turnover : 0.0;
    a.allow_short = d->allow_short;
    a.max_iter = d->max_iter > 0 ? d->max_iter : 80;
    a.tol = d->tol > 0.0 ? d->tol : 1e-9;
    a.return_full = d->return_full_W;
    a.n_refine = d->n_refine > 0 ? d->n_refine : (d->n_refine < 0 ? 0 : 3);
    return a;
}

bool use_big(const SolveArgs& a) {
#ifdef KMPC_DEV_ONLY_H10
    return false;
#else
    if (g_path == 1) return false;
    if (g_path == 2) return true;
    // measured on MI355X (tools/path_ab.py): the register kernels win up to 256 assets at
    // H <= 10 (N = 192: 76k vs 41k windows/s); the large-window kernel wins past 10 periods at any
    // N (N = 100, H = 20: 36k vs 24k) and past 256 assets (N = 500, H = 10: 23k vs 13k)
    return a.N > 256 || a.H > 10;
#endif
}

}  // namespace

size_t solve_workspace_bytes(const kmpc_solve_desc* d) {
    if (!d || d->B <= 0) return 0;
    const SolveArgs a = make_args(d);
#ifndef KMPC_DEV_ONLY_H10
    if (use_big(a)) return big_ws_bytes(a);
#endif
    return 0;
}

int solve_launch(const kmpc_solve_desc* d, const float* yhat, const double* w_prev, double* w_out,
                 int* status, double* obj, int* iters, void* ws, size_t ws_bytes, hipStream_t stream,
                 double* trace) {
    SolveArgs a = make_args(d);
    a.yhat = yhat; a.wp = w_prev; a.wout = w_out; a.status = status; a.obj = obj; a.iters = iters;
    a.trace = trace;
    if (a.B == 0) return KMPC_OK;
#ifndef KMPC_DEV_ONLY_H10
    if (use_big(a)) return big_launch(a, ws, ws_bytes, stream);
#endif
    // H == 5 / 10 with N <= 128 in the two common constraint cases: constant-case kernels
    if (a.H == 10 || a.H == 5) {
        const int rc = a.H == 10 ? launch_ipm_case<10>(a, stream) :
#ifndef KMPC_DEV_ONLY_H10
                                   launch_ipm_case<5>(a, stream);
#else
                                   KMPC_ERR_UNSUPPORTED;
#endif
        if (rc != KMPC_ERR_UNSUPPORTED) return rc;
    }
#ifndef KMPC_DEV_ONLY_H10
    if (a.H <= 2) return launch_ipm<2>(a, stream);
    if (a.H <= 5) return launch_ipm<5>(a, stream);
#endif
    if (a.H <= 10) return launch_ipm<10>(a, stream);
    return KMPC_ERR_UNSUPPORTED;   // H > 10: the large-window kernel
}

}  // namespace kmpc

extern "C" int kmpc_debug_solver_path(int path) {
    const int old = kmpc::g_path;
    kmpc::g_path = path;
    return old;
}
