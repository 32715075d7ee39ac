// kmpc_solve.hip — host dispatch of the batched MPC solve (replaces solve_mpc_log_utility,
// mpc.py:27-117). The kernel is kmpc_solve_kernel.h; each horizon bound HM is instantiated in its
// own translation unit (kmpc_solve_h*.hip) so the four compile in parallel.
#include "kmpc_internal.h"
#include "kmpc_solve_args.h"

namespace kmpc {

int solve_launch(const kmpc_solve_desc* d, const float* yhat, const double* w_prev, double* w_out,
                 int* status, double* obj, int* iters, hipStream_t stream, double* trace) {
    SolveArgs a;
    a.B = d->B; a.N = d->N; a.H = d->H;
    a.c = d->cost_coeff;
    a.tau = d->max_turnover > 0.0 ? d->max_turnover : 0.0;
    a.allow_short = d->allow_short;
    a.max_iter = d->max_iter > 0 ? d->max_iter : 80;
    a.tol = d->tol > 0.0 ? d->tol : 1e-9;
    a.return_full = d->return_full_W;
    a.n_refine = d->n_refine > 0 ? d->n_refine : (d->n_refine < 0 ? 0 : 3);
    a.yhat = yhat; a.wp = w_prev; a.wout = w_out; a.status = status; a.obj = obj; a.iters = iters;
    a.trace = trace;
    if (a.B == 0) return KMPC_OK;
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
#ifndef KMPC_DEV_ONLY_H10
    if (a.H <= 21) return launch_ipm<21>(a, stream);
#endif
    return KMPC_ERR_UNSUPPORTED;
}

}  // namespace kmpc
