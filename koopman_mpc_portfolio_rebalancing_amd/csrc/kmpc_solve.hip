// kmpc_solve.hip — host dispatch of the batched MPC solve (replaces solve_mpc_log_utility,
// mpc.py:27-117). Two kernel families solve the same program with the same interior point:
//   ipm_kernel (kmpc_solve_kernel.h): a window's state in the registers of one workgroup, one
//     asset per lane — for N <= 256 assets and H <= 10 periods; each horizon
//     bound HM is instantiated in its own translation unit (kmpc_solve_h*.hip).
//   ipm_big (kmpc_solve_big.h): the state in a workspace slab, streamed per phase, the Schur
//     matrix on the f64 MFMA — for larger windows (N > 256 or H > 10), which need workspace.
// Presolve: without turnover terms (c = tau = 0) and without shorting the program decouples into
// one problem per period, max log(R_t . w_t) over the simplex, whose optimum is exact in closed
// form (simplex_kernel below) — BASELINE configs[1], "no-short simplex projection only".
#include "kmpc_internal.h"
#include "kmpc_npexp.h"
#include "kmpc_solve_args.h"

namespace kmpc {

namespace {

// per-call solver path (kmpc_solve_desc.path): KMPC_PATH_AUTO by shape, KMPC_PATH_REGISTER =
// interior point in the register kernels whenever they support the shape (no presolve),
// KMPC_PATH_LARGE = the large-window kernel, KMPC_PATH_REGISTER_UNPACKED = the register kernels
// with one window per wave even for small windows (no lane-group packing, no presolve); AUTO and
// REGISTER pack small windows (pack_small: AUTO from KMPC_PACK_MIN_B windows, REGISTER always)
bool simplex_case(const SolveArgs& a) {
    return a.path == KMPC_PATH_AUTO && !(a.c > 0.0) && !(a.tau > 0.0) && !a.allow_short;
}

// Lane-group packing of small windows (N <= 32: 2-4 windows per wave) is a throughput layout. For
// a batch that cannot fill the GPU a window's latency decides, and one window per wave is faster:
// AUTO packs only from KMPC_PACK_MIN_B (include/kmpc.h) windows per call (H > 2), or at any batch
// size for H <= 2.
// Measured (tools/pack_cross_probe.py, solve only, packed / one-per-wave ms): N = 10, H = 5:
// B = 256 0.341 / 0.292, 1,024 0.361 / 0.342, 2,048 0.374 / 0.426, 65,536 3.41 / 9.08; N = 20,
// H = 10: B = 256 0.965 / 0.774, 1,024 1.03 / 1.39; N = 8, H = 2: packed ahead at every B. In the
// path-persistent backtest (P = 64, N = 10, H = 5): 0.297 -> 0.239 ms per step.
bool pack_small(const SolveArgs& a) {
    if (a.path == KMPC_PATH_REGISTER_UNPACKED || a.N > 32 || a.H > 10) return false;
    return a.path != KMPC_PATH_AUTO || a.B > KMPC_PACK_MIN_B || a.H <= 2;
}

// c = tau = 0, w >= 0: per period t, log(R_t . w_t) with R = exp(yhat) > 0 is maximized over the
// simplex exactly on the face of the assets with the largest R_t; the returned point is that
// face's centre (equal weights over exact ties: the analytic centre an interior-point method
// converges to, and the vertex e_argmax otherwise). problem.value as the IPM kernels report it
// (mpc.py:103): sum_t log(R_t . w_t) - c sum_t ||w_t - w_{t-1}||_1 (c <= 0 here). One wave per
// window, lanes over the assets (coalesced loads, wave butterflies for max / tie count / sums).
// Non-finite inputs -> solver_error and tile(w_prev).
__device__ __forceinline__ float wmaxf(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wsum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ int wsumi(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
constexpr int SIMPLEX_WAVES = 4;   // waves per 256-thread block
constexpr int SIMPLEX_HR = 16;     // register fast path: N <= 64 assets, H <= 16 periods
// float32 -> float64 handoff of the mixed-precision pair. Measured on the oracle's iteration
// (tools/f32phase_probe.py, 512 C3 windows of the bench's distribution: float32 to mu <= 5e-5 takes
// 7.9 of the 15.9 iterations, every window optimal, float64 finish 8.0 iterations; 2e-5 left 1% of
// the windows optimal_inaccurate) and on MI355X (tools/ab_mixed.sh, 65,536 windows, retry pass in:
// bench yhat 83.3 ms at 1e-4, 82.0 ms at 5e-5; random yhat 91.1 / 90.7 ms, same statuses as float64).
// 3e-5 since round 6's step / sigma rules (tools/gpu_r6v.sh, twice: bench yhat 74.80 / 74.70 ms at
// 5e-5, 74.43 / 74.24 at 3e-5, 74.11 / 73.94 at 2e-5; random yhat 77.92 / 77.75, 77.64 / 77.45,
// 78.88 / 78.69 — 2e-5 loses on random yhat; statuses as float64 at every threshold)
constexpr double MU_HANDOFF = 3e-5;

// butterflies within aligned groups of G lanes (G = 32 or 64)
template <int G>
__device__ __forceinline__ float gmaxf(float v) {
    for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
template <int G>
__device__ __forceinline__ int gsumi(int v) {
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// N <= G (G = 32: two windows per wave; G = 64: one), H <= 16 (BASELINE configs[1]: N = 30, H = 5):
// lane i of the window's lane group holds R_t,i of its asset for every period in registers (one
// pass over yhat, one np_expf per element), and each group reduction runs over all periods at once
// (H independent butterflies interleaved, instead of H dependent rounds). Same arithmetic and order
// as the general loop below (a group butterfly over G lanes adds zeros where the wave-wide one did):
// bit-identical results.
// HR: the period bound; HX = H known at compile time (BASELINE configs[1]: H = 5 — no period guards)
template <int G, int HR = SIMPLEX_HR, bool HX = false>
__device__ __forceinline__ void simplex_regs(const SolveArgs& a, int b, int lane) {
    const int N = a.N, H = HX ? HR : a.H, tw = a.return_full ? H : 1;
    const float* y = a.yhat + (size_t)b * H * N;
    const double* wp = a.wp + (size_t)b * N;
    double* wout = a.wout + (size_t)b * tw * N;
    const bool act = lane < N;
    const double wpi = act ? wp[lane] : 0.0;
    float R[HR];
    int bad = !(isfinite(a.c) && isfinite(a.tau)) || (act && !isfinite(wpi));
#pragma unroll
    for (int t = 0; t < HR; ++t) {
        R[t] = 0.0f;
        if (t < H && act) {
            R[t] = np_expf(y[(size_t)t * N + lane]);
            bad |= !isfinite(R[t]);
        }
    }
    if (gsumi<G>(bad)) {
        if (act)
            for (int t = 0; t < tw; ++t) wout[(size_t)t * N + lane] = wpi;   // mpc.py:113-115
        if (lane == 0) {
            a.status[b] = KMPC_STATUS_SOLVER_ERROR;
            a.obj[b] = __builtin_nan("");
            if (a.iters) a.iters[b] = 0;
        }
        return;
    }
    float rm[HR];
    int cnt[HR];
#pragma unroll
    for (int t = 0; t < HR; ++t) rm[t] = R[t];
    for (int o = G / 2; o > 0; o >>= 1)
#pragma unroll
        for (int t = 0; t < HR; ++t)
            if (t < H) rm[t] = fmaxf(rm[t], __shfl_xor(rm[t], o));
    // a period whose every R underflowed to 0 (yhat <= -103.97): R_t . w_t = 0 on the whole simplex
    // and the reference's exp cone exp(u) <= R_t . w_t has no solution (cvxpy: infeasible) —
    // infeasible and the fallback, as the interior-point kernels report it
    bool flat0 = false;
#pragma unroll
    for (int t = 0; t < HR; ++t) flat0 |= t < H && !(rm[t] > 0.0f);
    if (flat0) {
        if (act)
            for (int t = 0; t < tw; ++t) wout[(size_t)t * N + lane] = wpi;   // mpc.py:113-115
        if (lane == 0) {
            a.status[b] = KMPC_STATUS_INFEASIBLE;
            a.obj[b] = __builtin_nan("");
            if (a.iters) a.iters[b] = 0;
        }
        return;
    }
#pragma unroll
    for (int t = 0; t < HR; ++t) cnt[t] = (t < H && act && R[t] == rm[t]) ? 1 : 0;
    for (int o = G / 2; o > 0; o >>= 1)
#pragma unroll
        for (int t = 0; t < HR; ++t)
            if (t < H) cnt[t] += __shfl_xor(cnt[t], o);
    double rw[HR], l1[HR];
    double wprev = wpi;
#pragma unroll
    for (int t = 0; t < HR; ++t) {
        rw[t] = l1[t] = 0.0;
        if (t < H) {
            const double w = 1.0 / cnt[t];
            const double wi = (act && R[t] == rm[t]) ? w : 0.0;
            rw[t] = (double)R[t] * wi;
            l1[t] = act ? fabs(wi - wprev) : 0.0;
            if (act && t < tw) wout[(size_t)t * N + lane] = wi;
            wprev = wi;
        }
    }
    for (int o = G / 2; o > 0; o >>= 1)
#pragma unroll
        for (int t = 0; t < HR; ++t)
            if (t < H) { rw[t] += __shfl_xor(rw[t], o); l1[t] += __shfl_xor(l1[t], o); }
    if (lane == 0) {
        double f = 0.0;
#pragma unroll
        for (int t = 0; t < HR; ++t)
            if (t < H) f += log(rw[t]) - a.c * l1[t];
        a.status[b] = KMPC_STATUS_OPTIMAL;
        a.obj[b] = f;
        if (a.iters) a.iters[b] = 0;
    }
}

__global__ void __launch_bounds__(64 * SIMPLEX_WAVES) simplex_kernel(SolveArgs a) {
    const int lane = threadIdx.x & 63;
    if (a.N <= 32 && a.H <= SIMPLEX_HR) {
        // two windows per wave, one per 32-lane half
        const int b = (blockIdx.x * SIMPLEX_WAVES + (threadIdx.x >> 6)) * 2 + (lane >> 5);
        if (b < a.B) {   // (whole lane groups)
            if (a.H == 5) simplex_regs<32, 5, true>(a, b, lane & 31);
            else simplex_regs<32>(a, b, lane & 31);
        }
        return;
    }
    const int b = blockIdx.x * SIMPLEX_WAVES + (threadIdx.x >> 6);
    if (b >= a.B) return;   // (whole waves)
    if (a.N <= 64 && a.H <= SIMPLEX_HR) {
        simplex_regs<64>(a, b, lane);
        return;
    }
    const int N = a.N, H = a.H, tw = a.return_full ? H : 1;
    const float* y = a.yhat + (size_t)b * H * N;
    const double* wp = a.wp + (size_t)b * N;
    double* wout = a.wout + (size_t)b * tw * N;
    int bad = !(isfinite(a.c) && isfinite(a.tau));
    for (int i = lane; i < N; i += 64) bad |= !isfinite(wp[i]);
    for (int k = lane; k < H * N; k += 64) bad |= !isfinite(np_expf(y[k]));
    // a period whose every R underflowed to 0: infeasible (see simplex_regs)
    int zero = 0;
    for (int t = 0; t < H; ++t) {
        float rm = 0.0f;
        for (int i = lane; i < N; i += 64) rm = fmaxf(rm, np_expf(y[(size_t)t * N + i]));
        zero |= !(wmaxf(rm) > 0.0f);
    }
    bad = wsumi(bad);
    if (bad || zero) {
        for (int k = lane; k < tw * N; k += 64) wout[k] = wp[k % N];   // mpc.py:113-115
        if (lane == 0) {
            a.status[b] = bad ? KMPC_STATUS_SOLVER_ERROR : KMPC_STATUS_INFEASIBLE;
            a.obj[b] = __builtin_nan("");
            if (a.iters) a.iters[b] = 0;
        }
        return;
    }
    // the face is that of the largest float32 R = np.exp(yhat) (mpc.py:55): distinct yhat can
    // round to the same R, and the program the reference solves only sees R
    double f = 0.0;
    float prm = 0.0f;
    double pw = 0.0;   // the previous period's face weight
    for (int t = 0; t < H; ++t) {
        const float* yt = y + (size_t)t * N;
        float rm = 0.0f;
        for (int i = lane; i < N; i += 64) rm = fmaxf(rm, np_expf(yt[i]));
        rm = wmaxf(rm);
        int cnt = 0;
        for (int i = lane; i < N; i += 64) cnt += np_expf(yt[i]) == rm;
        cnt = wsumi(cnt);
        const double w = 1.0 / cnt;
        double rw = 0.0, l1 = 0.0;
        for (int i = lane; i < N; i += 64) {
            const float ri = np_expf(yt[i]);
            const double wi = ri == rm ? w : 0.0;
            rw += (double)ri * wi;
            const double wprev = t == 0 ? wp[i] : (np_expf(y[(size_t)(t - 1) * N + i]) == prm ? pw : 0.0);
            l1 += fabs(wi - wprev);
            if (t < tw) wout[(size_t)t * N + i] = wi;
        }
        f += log(wsum(rw)) - a.c * wsum(l1);
        prm = rm;
        pw = w;
    }
    if (lane == 0) {
        a.status[b] = KMPC_STATUS_OPTIMAL;
        a.obj[b] = f;
        if (a.iters) a.iters[b] = 0;
    }
}

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
    a.path = d->path;
    a.warm = nullptr;
    a.warm_floats = 0;
    a.mu_handoff = d->mu_handoff > 0.0 ? d->mu_handoff : MU_HANDOFF;
    return a;
}

// Mixed precision (kmpc_solve_kernel.h, PH = 1 / 2): the shapes with a float32 / float64 kernel
// pair — the C3 kernel's (H = 10, 128 threads with N < 104, no short, c > 0 or tau > 0, cap).
// Windows per launch: one workgroup of up to 256 threads per window (the register kernels), so a
// grid of at most 2^22 stays below a dispatch's 2^32 work-items; larger batches go as equal launches.
constexpr int LAUNCH_MAX_B = 1 << 22;

// One warm record per window: its 64 B header alone with the fused kernel's on-chip handoff (the
// whole batch in one launch), else the full record, in chunks of at most WARM_CHUNK windows.
constexpr int WARM_CHUNK = 131072;
// AUTO takes the pair from KMPC_MIXED_MIN_B windows: below it a launch is latency-bound (the
// slowest window's iterations), and float64 alone measured faster — lock-step backtest, C3 model,
// path-steps/s (tools/lockstep_probe.py): P = 64 53.7 k mixed vs 56.1 k float64, P = 256 191 k vs
// 206 k, P = 1,024 404 k vs 430 k, P = 4,096 539 k vs 513 k
bool mixed_case(const SolveArgs& a, const kmpc_solve_desc* d) {
    if (d->precision == KMPC_PRECISION_F64) return false;
    if (d->precision == KMPC_PRECISION_AUTO && a.B < KMPC_MIXED_MIN_B) return false;
    if (a.path != KMPC_PATH_AUTO && a.path != KMPC_PATH_REGISTER && a.path != KMPC_PATH_REGISTER_UNPACKED) return false;
    const bool fl7 = !a.allow_short && (a.c > 0.0 || a.tau > 0.0) && a.tau > 0.0;
    return fl7 && a.H == 10 && a.N > 64 && a.N < 104;
}
// windows per mixed launch: the whole batch when the record is the 64 B header alone
int warm_chunk(const SolveArgs& a) {
    if (mixed_warm_floats(a.H, a.N) == (size_t)WARM_HEAD) return a.B < LAUNCH_MAX_B ? a.B : LAUNCH_MAX_B;
    return a.B < WARM_CHUNK ? a.B : WARM_CHUNK;
}
size_t warm_bytes(const SolveArgs& a) { return sizeof(float) * mixed_warm_floats(a.H, a.N) * (size_t)warm_chunk(a); }

bool use_big(const SolveArgs& a) {
#ifdef KMPC_DEV_ONLY_H10
    return false;
#else
    if (a.path == KMPC_PATH_REGISTER || a.path == KMPC_PATH_REGISTER_UNPACKED) return false;
    if (a.path == KMPC_PATH_LARGE) return true;
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
    if (simplex_case(a)) return 0;
#ifndef KMPC_DEV_ONLY_H10
    if (use_big(a)) return big_ws_bytes(a);
#endif
    if (mixed_case(a, d)) return warm_bytes(a);
    return 0;
}

int solve_launch(const kmpc_solve_desc* d, const float* yhat, const double* w_prev, double* w_out,
                 int* status, double* obj, int* iters, void* ws, size_t ws_bytes, hipStream_t stream,
                 double* trace) {
    if (d->B > LAUNCH_MAX_B) {
        // equal launches of at most LAUNCH_MAX_B windows: each chunk is past every batch threshold
        // (KMPC_MIXED_MIN_B, KMPC_PACK_MIN_B), so AUTO takes the same kernels as for the whole batch
        const int nch = (int)(((size_t)d->B + LAUNCH_MAX_B - 1) / LAUNCH_MAX_B);
        const int per = (int)(((size_t)d->B + nch - 1) / nch);
        const size_t HN = (size_t)d->H * d->N, wo = d->return_full_W ? HN : (size_t)d->N;
        kmpc_solve_desc c = *d;
        for (int b0 = 0; b0 < d->B; b0 += per) {
            c.B = d->B - b0 < per ? d->B - b0 : per;
            const int rc = solve_launch(&c, yhat + (size_t)b0 * HN, w_prev + (size_t)b0 * d->N, w_out + (size_t)b0 * wo,
                                        status + b0, obj + b0, iters ? iters + b0 : nullptr, ws, ws_bytes, stream,
                                        b0 == 0 ? trace : nullptr);
            if (rc != KMPC_OK) return rc;
        }
        return KMPC_OK;
    }
    SolveArgs a = make_args(d);
    a.yhat = yhat; a.wp = w_prev; a.wout = w_out; a.status = status; a.obj = obj; a.iters = iters;
    a.trace = trace;
    if (a.B == 0) return KMPC_OK;
    if (simplex_case(a)) {
        const int per_block = SIMPLEX_WAVES * ((a.N <= 32 && a.H <= SIMPLEX_HR) ? 2 : 1);
        hipLaunchKernelGGL(simplex_kernel, dim3((a.B + per_block - 1) / per_block), dim3(64 * SIMPLEX_WAVES), 0,
                           stream, a);
        return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
    }
#ifndef KMPC_DEV_ONLY_H10
    if (use_big(a)) return big_launch(a, ws, ws_bytes, stream);
#endif
    // N <= 32: several windows per wave on lane groups (16 lanes for N <= 16 at H <= 5, else 32)
    if (pack_small(a)) {
#ifndef KMPC_DEV_ONLY_H10
        const int rc = a.H <= 2 ? launch_ipm_packed<2>(a, stream)
                                : (a.H <= 5 ? launch_ipm_packed<5>(a, stream) : launch_ipm_packed<10>(a, stream));
        if (rc != KMPC_ERR_UNSUPPORTED) return rc;
#endif
    }
    // mixed precision (float32 phase + float64 finish), chunk by chunk
    if (mixed_case(a, d)) {
        if (!ws || ws_bytes < warm_bytes(a)) return KMPC_ERR_WORKSPACE;
        SolveArgs c = a;
        c.warm = (float*)ws;
        c.warm_floats = mixed_warm_floats(a.H, a.N);
        const size_t HN = (size_t)a.H * a.N;
        const int chunk = warm_chunk(a);
        for (int b0 = 0; b0 < a.B; b0 += chunk) {
            c.B = a.B - b0 < chunk ? a.B - b0 : chunk;
            c.yhat = a.yhat + (size_t)b0 * HN;
            c.wp = a.wp + (size_t)b0 * a.N;
            c.wout = a.wout + (size_t)b0 * (a.return_full ? HN : (size_t)a.N);
            c.status = a.status + b0;
            c.obj = a.obj + b0;
            c.iters = a.iters ? a.iters + b0 : nullptr;
            c.trace = b0 == 0 ? a.trace : nullptr;
            const int rc = launch_ipm_c3(c, stream);
            if (rc != KMPC_OK) return rc;
        }
        return KMPC_OK;
    }
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

// kmpc_backtest_run: a path-persistent kernel exists for the shapes whose per-step batch of P
// windows kmpc_solve sends to a float64 constant-case register kernel (case 7: no short, cost and
// cap; H = 10 or 5 with 32 < N <= 256, one window per workgroup; and the packed N <= 32 kernels
// with H = 2, 5 or 10, one path per lane group — not the mixed pair): the persistent kernel runs
// that kernel's window body, so the steps match it
int backtest_run_launch(const kmpc_backtest_desc* bd, const kmpc_solve_desc* sd, int step0, int n_steps,
                        const float* yhat, const float* realized, int n_real, double* weights, double* value,
                        double* hist, double* target, int* status, double* obj, hipStream_t stream) {
    kmpc_solve_desc d = *sd;
    d.B = bd->P;
    SolveArgs a = make_args(&d);
    const bool fl7 = !a.allow_short && (a.c > 0.0 || a.tau > 0.0) && a.tau > 0.0;
    const bool packed = pack_small(a);   // (the kernel kmpc_solve picks for this batch of P windows)
    if (a.return_full || simplex_case(a) || use_big(a) || mixed_case(a, &d) || !fl7 || a.N > 256)
        return KMPC_ERR_UNSUPPORTED;
    // (the packed kernels exist for H = 2, 5, 10 — launch_ipm_packed's HM, exact H only)
    if (packed ? (a.H != 2 && a.H != 5 && a.H != 10) : (a.H != 10 && a.H != 5)) return KMPC_ERR_UNSUPPORTED;
    if (a.path != KMPC_PATH_AUTO && a.path != KMPC_PATH_REGISTER && a.path != KMPC_PATH_REGISTER_UNPACKED)
        return KMPC_ERR_UNSUPPORTED;
    const int nt = 64 * ((a.N + 63) / 64);
#ifdef KMPC_DEV_ONLY_H10   // (dev builds link the C3 unit only)
    if (!(a.H == 10 && nt == 128 && a.N < QL_CS)) return KMPC_ERR_UNSUPPORTED;
#endif
    if (bd->P == 0 || n_steps == 0) return KMPC_OK;
    a.wout = target; a.status = status; a.obj = obj; a.iters = nullptr; a.trace = nullptr;
    a.yhat = yhat; a.wp = weights;
#ifndef KMPC_DEV_ONLY_H10
    if (packed) {
        const auto fn = a.H == 2 ? launch_bt_run_packed<2> : (a.H == 5 ? launch_bt_run_packed<5> : launch_bt_run_packed<10>);
        return fn(a, n_steps, n_real, yhat, realized, step0, bd->S, bd->cost_coeff, weights, value, hist, stream);
    }
#endif
    if (a.H == 10 && nt == 128 && a.N < QL_CS)
        return launch_bt_run_c3(a, n_steps, n_real, yhat, realized, step0, bd->S, bd->cost_coeff, weights, value,
                                hist, stream);
#ifndef KMPC_DEV_ONLY_H10
    if (a.H == 5)
        return launch_bt_run_case<5>(a, n_steps, n_real, yhat, realized, step0, bd->S, bd->cost_coeff, weights,
                                     value, hist, stream);
    return launch_bt_run_case<10>(a, n_steps, n_real, yhat, realized, step0, bd->S, bd->cost_coeff, weights, value,
                                  hist, stream);
#else
    return KMPC_ERR_UNSUPPORTED;
#endif
}

}  // namespace kmpc
