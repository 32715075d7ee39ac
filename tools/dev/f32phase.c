/*
 * f32phase.c — dev measurement only: the oracle's Mehrotra iteration
 * (oracle/kmpc_oracle.c, included verbatim) run as two phases,
 *   phase 1 in `real` = float until mu <= mu_stop (or a float breakdown), state handed out,
 *   phase 2 in `real` = double from that state to the usual tolerance.
 * Built twice (tools/dev/f32phase.sh): -DKMPC_REAL_FLOAT -> kmpc_phase_f, default -> kmpc_phase.
 * Never linked into the product or the tests.
 *
 * State layout (double): w, s, l1, l2, l3 [H*N] each, then z4, l4, nu [H] each.
 * Returns the oracle's status, or 100 = handed off at mu <= mu_stop (state in st_out).
 */
#include "../../oracle/kmpc_oracle.c"

#define HANDOFF 100

static void state_get(const ws_t* W, double* st) {
    size_t HN = (size_t)W->H * W->N;
    for (size_t k = 0; k < HN; ++k) {
        st[k] = W->w[k]; st[HN + k] = W->s[k]; st[2 * HN + k] = W->l1[k];
        st[3 * HN + k] = W->l2[k]; st[4 * HN + k] = W->l3[k];
    }
    for (int t = 0; t < W->H; ++t) {
        st[5 * HN + t] = W->z4[t]; st[5 * HN + W->H + t] = W->l4[t]; st[5 * HN + 2 * W->H + t] = W->nu[t];
    }
}

static void state_put(ws_t* W, const double* st) {
    size_t HN = (size_t)W->H * W->N;
    for (size_t k = 0; k < HN; ++k) {
        W->w[k] = (real)st[k]; W->s[k] = (real)st[HN + k]; W->l1[k] = (real)st[2 * HN + k];
        W->l2[k] = (real)st[3 * HN + k]; W->l3[k] = (real)st[4 * HN + k];
    }
    for (int t = 0; t < W->H; ++t) {
        W->z4[t] = (real)st[5 * HN + t]; W->l4[t] = (real)st[5 * HN + W->H + t];
        W->nu[t] = (real)st[5 * HN + 2 * W->H + t];
    }
}

int API(kmpc_phase)(int N, int H, const double* wp, const float* yhat, double c, double tau,
                    int max_iter, double tol, double mu_stop, const double* st_in, double* st_out,
                    int* iters_out, double* mu_out, double* Wout, double* obj) {
    int status = ST_ERROR, it = 0;
    size_t HN = (size_t)H * N;
    ws_t W;
    memset(&W, 0, sizeof(W));
    if (ws_init(&W, N, H) != 0) return ST_ERROR;
    W.N = N; W.H = H; W.K = 3 * H;
    W.hw = 1; W.hs = (c > 0) || (tau > 0); W.ht = tau > 0;
    W.n_refine = 3;
    real sig = (real)c;
    for (int i = 0; i < N; ++i) W.wp[i] = (real)wp[i];
    for (size_t k = 0; k < HN; ++k) {
        W.m[k] = (real)((double)np_expf(yhat[k]) - 1.0);
        if (RFABS(W.m[k]) > sig) sig = RFABS(W.m[k]);
    }
    if (!(sig > 0)) sig = 1;
    W.sig = sig; W.c = (real)c / sig; W.tau = (real)tau;
    double* prev = (double*)calloc(5 * HN + 3 * H, sizeof(double));
    if (st_in) {
        state_put(&W, st_in);
    } else {
        for (int t = 0; t < H; ++t)
            for (int i = 0; i < N; ++i) W.w[t * N + i] = R_(0.5) * (real)wp[i] + R_(0.5) / N;
        for (int t = 0; t < H; ++t) {
            real ss = 0;
            for (int i = 0; i < N; ++i) {
                int k = t * N + i;
                real d = W.w[k] - DPREV(&W, k, t, i);
                W.s[k] = W.hs ? RFABS(d) + R_(1.0) / N : 0;
                ss += W.s[k];
                W.l1[k] = 1;
                W.l2[k] = W.l3[k] = W.hs ? 1 : 0;
            }
            W.z4[t] = W.ht ? RFMAX((real)tau - ss, R_(0.5) * (real)tau) : 1;
            W.l4[t] = W.ht ? 1 : 0;
            W.nu[t] = 0;
        }
    }
    state_get(&W, prev);
    int ncon = (int)HN + (W.hs ? 2 * (int)HN : 0) + (W.ht ? H : 0);
    real best = R_(1e30), min_pr = R_(1e30), last_mu = R_(1e30);
    int handoff = 0;
    for (it = 0; it < max_iter; ++it) {
        real mu = 0, rd = 0, pr = 0;
        int domain_ok = 1;
        for (int t = 0; t < H; ++t) {
            real den = 1, sw = 0, ss = 0;
            for (int i = 0; i < N; ++i) {
                int k = t * N + i;
                den += W.m[k] * W.w[k]; sw += W.w[k]; ss += W.s[k];
            }
            W.den[t] = den; W.rp[t] = sw - 1;
            W.rg4[t] = W.ht ? (real)tau - ss - W.z4[t] : 0;
            if (!(den > 0)) domain_ok = 0;
            for (int i = 0; i < N; ++i) {
                int k = t * N + i;
                real d = W.w[k] - DPREV(&W, k, t, i);
                W.a[k] = W.m[k] / (den * RSQRT(sig));
                real eta = W.l3[k] - W.l2[k];
                real etan = (t + 1 < H) ? W.l3[k + N] - W.l2[k + N] : 0;
                W.rdw[k] = -W.m[k] / (sig * den) - (W.l1[k] + eta - etan) + W.nu[t];
                W.rds[k] = W.hs ? W.c - (W.l2[k] + W.l3[k] - W.l4[t]) : 0;
                W.rc1[k] = W.w[k] * W.l1[k];
                W.rc2[k] = W.hs ? (W.s[k] - d) * W.l2[k] : 0;
                W.rc3[k] = W.hs ? (W.s[k] + d) * W.l3[k] : 0;
                mu += W.rc1[k] + W.rc2[k] + W.rc3[k];
                rd = RFMAX(rd, RFMAX(RFABS(W.rdw[k]), RFABS(W.rds[k])));
            }
            W.rc4[t] = W.ht ? W.z4[t] * W.l4[t] : 0;
            mu += W.rc4[t];
            pr = RFMAX(pr, RFMAX(RFABS(W.rp[t]), RFABS(W.rg4[t])));
        }
        mu /= ncon;
        real merit = RFMAX(mu, RFMAX(rd, pr));
        if (!domain_ok || !RISFIN(merit)) {
            if (mu_stop > 0) { handoff = 2; break; }   /* float breakdown: hand off the previous iterate */
            break;
        }
        min_pr = RFMIN(min_pr, pr);
        if (mu_out) *mu_out = (double)mu;
        if (mu_stop > 0 && (double)mu <= mu_stop) { state_get(&W, prev); handoff = 1; break; }
        if (mu_stop > 0 && it > 3 && mu > R_(0.9) * last_mu) { handoff = 2; break; }   /* float stagnation */
        last_mu = mu;
        if (merit < best) {
            best = merit;
            memcpy(W.wbest, W.w, sizeof(real) * HN);
        } else if (best < R_(1e-6) && merit > R_(1e4) * best) {
            break;
        }
        if (mu < tol && rd < 10 * tol && pr < 10 * tol) break;
        state_get(&W, prev);
        if (factor(&W) != 0) { if (mu_stop > 0) handoff = 2; break; }
        {
            const int nr = W.n_refine;
            W.n_refine = 0;
            newton(&W);
            W.n_refine = nr;
        }
        real ap = RFMIN(1, max_step(&W));
        real sg = complementarity(&W, ap) / ncon / mu;
        sg = sg * sg * sg;
        for (int t = 0; t < H; ++t) {
            for (int i = 0; i < N; ++i) {
                int k = t * N + i;
                W.rc1[k] += W.dw[k] * W.dl1[k] - sg * mu;
                if (W.hs) {
                    W.rc2[k] += (W.ds[k] - W.dd[k]) * W.dl2[k] - sg * mu;
                    W.rc3[k] += (W.ds[k] + W.dd[k]) * W.dl3[k] - sg * mu;
                }
            }
            if (W.ht) W.rc4[t] += W.dz4[t] * W.dl4[t] - sg * mu;
        }
        {
            const int nr = W.n_refine;
            /* dev knob: F32PH_REFMU refines the corrector from that mu (default 1e-6, the kernels') */
            const char* e = getenv("F32PH_REFMU");
            if (mu > (real)(e ? atof(e) : 1e-6)) W.n_refine = 0;
            newton(&W);
            W.n_refine = nr;
        }
        real a = RFMIN(1, R_(0.99) * max_step(&W));
        for (size_t k = 0; k < HN; ++k) {
            W.w[k] += a * W.dw[k]; W.s[k] += a * W.ds[k];
            W.l1[k] += a * W.dl1[k]; W.l2[k] += a * W.dl2[k]; W.l3[k] += a * W.dl3[k];
        }
        for (int t = 0; t < H; ++t) {
            W.z4[t] += a * W.dz4[t]; W.l4[t] += a * W.dl4[t]; W.nu[t] += a * W.dnu[t];
        }
    }
    if (iters_out) *iters_out = it;
    if (handoff) {
        memcpy(st_out, prev, sizeof(double) * (5 * HN + 3 * H));
        status = HANDOFF;
        for (size_t k = 0; k < HN; ++k) Wout[k] = NAN;
        if (obj) *obj = NAN;
    } else {
        if (best <= R_(1e-7)) status = ST_OPTIMAL;
        else if (best <= R_(1e-4)) status = ST_INACCURATE;
        else if (min_pr > R_(1e-6)) status = ST_INFEASIBLE;
        else status = ST_ERROR;
        if (status <= ST_INACCURATE) {
            for (size_t k = 0; k < HN; ++k) Wout[k] = (double)W.wbest[k];
            if (obj) *obj = API(kmpc_oracle_objective)(N, H, wp, yhat, c, Wout);
        } else {
            for (size_t k = 0; k < HN; ++k) Wout[k] = wp[k % N];
            if (obj) *obj = NAN;
        }
    }
    free(prev);
    free(W.pool);
    return status;
}
