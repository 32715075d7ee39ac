#!/usr/bin/env python3
"""Dev measurement (CPU only): an active-set polish of the log-utility program
(reference mpc.py:66-104) at the interior point's handoff, measured on the oracle before any kernel.

For B C3 windows (the bench model's torch-CPU rollout of window_inputs(0, B), c = 1e-3, tau = 0.2,
no short) it runs the oracle's Mehrotra iteration (tools/dev/f32phase.c) in float32 — the
kernel's float32 phase — until mu <= mu_s, then from that iterate:
  1. classifies every constraint: w_ti = 0 (w < l1), the sign of d_ti = w_ti - w_{t-1,i}
     (up: s - d active, down: s + d active, tied: both), binding caps (z4 < l4);
  2. solves the reduced problem on that face in float64 — min -sum_t log(R_t.w_t) + c sum sgn d
     subject to the budgets, the ties and the binding caps (all equalities) — by Newton's method on
     its KKT system (min-norm steps: the Hessian is rank one per period, so the face's optimum can
     be a segment);
  3. accepts the polished W if it is feasible (w >= 0, the classified signs hold, the slack caps
     <= tau) and the weak-duality certificate (oracle/certificate.py: the LP dual) gives
     gap <= 1e-6 + 1e-5 |f|  (the kernels' objective bar) — else the float64 IPM would continue.
Reports the acceptance rate, the gap distribution and the float64 iterations saved against the
float64 finish from the same handoff (tools/dev/f32phase.c's phase 2).

    python tools/polish_probe.py [B] [mu_s,...]
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from f32phase_probe import build, phase, windows  # noqa: E402


def classify(st, H, N):
    HN = H * N
    w, s, l1, l2, l3 = (st[k * HN:(k + 1) * HN].reshape(H, N) for k in range(5))
    z4, l4 = st[5 * HN:5 * HN + H], st[5 * HN + H:5 * HN + 2 * H]
    return w, s, l1, l2, l3, z4, l4


def polish(st, wp, R, c, tau, newton_iters=8, st0=None):
    """The reduced problem on the classified face, float64. Returns (W, ok, info).
    st0: the previous iterate — then every complementary pair (x, l) is classified by Tapia's
    indicator (x active iff x shrank by more than l did: x1/x0 < l1/l0), else by x < l."""
    H, N = R.shape
    w, s, l1, l2, l3, z4, l4 = classify(st, H, N)
    wprev = np.vstack([wp[None], w[:-1]])
    d = w - wprev
    if st0 is not None:
        w0, s0, m10, m20, m30, z40, l40 = classify(st0, H, N)
        d0 = w0 - np.vstack([wp[None], w0[:-1]])
        act = lambda x1, x0, y1, y0: (x1 / x0) < (y1 / y0)   # noqa: E731
        a_act = act(s - d, s0 - d0, l2, m20)
        b_act = act(s + d, s0 + d0, l3, m30)
        w_zero = act(w, w0, l1, m10)
        cap = act(z4, z40, l4, l40) if tau > 0 else np.zeros(H, bool)
    else:
        a_act = (s - d) < l2                             # s = d   (d >= 0)
        b_act = (s + d) < l3                             # s = -d  (d <= 0)
        w_zero = w < l1
        cap = (z4 < l4) if tau > 0 else np.zeros(H, bool)
    tied = a_act & b_act
    sgn = np.where(tied, 0, np.where(a_act, 1, np.where(b_act, -1, np.sign(d))))
    # w_ti > 0 on the face: a tied w inherits its predecessor's class (w_prev > 0 at t = 0); a
    # moved w by its primal / dual pair (up moves are never to zero)
    free = np.zeros((H, N), bool)
    for t in range(H):
        prev = (wp > 0) if t == 0 else free[t - 1]
        free[t] = np.where(tied[t], prev, np.where(sgn[t] > 0, True, ~w_zero[t]))
    idx = -np.ones((H, N), int)
    idx[free] = np.arange(int(free.sum()))
    nf = int(free.sum())
    rows, rhs = [], []

    def wterm(t, i, coef, row):   # coef * w_ti into a constraint row (fixed-zero w contributes 0)
        if t < 0:
            return coef * wp[i]   # constant
        if idx[t, i] >= 0:
            row[idx[t, i]] += coef
        return 0.0

    for t in range(H):            # budgets
        r = np.zeros(nf)
        for i in range(N):
            wterm(t, i, 1.0, r)
        rows.append(r)
        rhs.append(1.0)
    for t in range(H):            # ties: w_ti - w_{t-1,i} = 0 (only those with a free side)
        for i in range(N):
            if sgn[t, i] != 0:
                continue
            if idx[t, i] < 0 and (t == 0 or idx[t - 1, i] < 0):
                if t == 0 and wp[i] != 0:
                    return None, False, {"why": "tie to w_prev with w fixed at zero"}
                continue
            r = np.zeros(nf)
            k = wterm(t, i, 1.0, r) - wterm(t - 1, i, -1.0, r) if t else wterm(t, i, 1.0, r) - wp[i]
            rows.append(r)
            rhs.append(-k if t else wp[i])
    for t in range(H):            # binding caps: sum_i sgn (w_ti - w_{t-1,i}) = tau
        if not cap[t]:
            continue
        r = np.zeros(nf)
        const = 0.0
        for i in range(N):
            if sgn[t, i] == 0:
                continue
            wterm(t, i, sgn[t, i], r)
            if t == 0:
                const -= sgn[t, i] * wp[i]
            else:
                wterm(t - 1, i, -sgn[t, i], r)
        rows.append(r)
        rhs.append(tau - const)
    A = np.array(rows)
    b = np.array(rhs)
    # linear part of the objective: c sum sgn (w_ti - w_{t-1,i}) over the free w
    g_lin = np.zeros(nf)
    for t in range(H):
        for i in range(N):
            if sgn[t, i] == 0:
                continue
            if idx[t, i] >= 0:
                g_lin[idx[t, i]] += c * sgn[t, i]
            if t + 1 < H and idx[t, i] >= 0 and sgn[t + 1, i] != 0:
                g_lin[idx[t, i]] -= c * sgn[t + 1, i]
    # starting point: the iterate's free w, projected onto A x = b (min-norm correction)
    x = w[free].astype(np.float64)
    x = x - np.linalg.lstsq(A, A @ x - b, rcond=None)[0]
    Rf = [(R[t][free[t]], idx[t][free[t]]) for t in range(H)]

    def grad_hess(x):
        g = g_lin.copy()
        Hm = np.zeros((nf, nf))
        for t in range(H):
            r, ix = Rf[t]
            u = r @ x[ix]
            g[ix] -= r / u
            Hm[np.ix_(ix, ix)] += np.outer(r, r) / u ** 2
        return g, Hm

    m = A.shape[0]
    for _ in range(newton_iters):
        g, Hm = grad_hess(x)
        K = np.block([[Hm, A.T], [A, np.zeros((m, m))]])
        rhs_k = -np.concatenate([g, A @ x - b])
        step = np.linalg.lstsq(K, rhs_k, rcond=1e-14)[0][:nf]
        if np.abs(step).max() < 1e-15:
            break
        x = x + step
    W = np.zeros((H, N))
    W[free] = x
    # feasibility on the classified face
    Wp = np.vstack([wp[None], W[:-1]])
    D = W - Wp
    ok = W.min() >= -1e-12
    ok = ok and bool(np.all(D[sgn == 1] >= -1e-12)) and bool(np.all(D[sgn == -1] <= 1e-12))
    if tau > 0:
        ok = ok and bool(np.all(np.abs(D).sum(1) <= tau + 1e-10))
    W = np.maximum(W, 0.0)
    return W, ok, {"free": nf, "constraints": m, "tied": int(tied.sum()), "caps": int(cap.sum())}


DEBUG = os.environ.get("DEBUG", "0") == "1"


def main():
    from oracle import certificate as cert, solver as osolver
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    MUS = [float(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "5e-5,1e-5,1e-6").split(",")]
    c, tau = 1e-3, 0.2
    F64 = os.environ.get("F64", "0") == "1"
    libs = build()
    wp, y = windows(B)
    Wl, stl, objl, itl = osolver.solve_batch(wp, y, c, tau, False, precision="ld", tol=1e-9)
    print(f"long-double oracle: mean iters {itl.mean():.2f}, optimal {int((stl == 0).sum())}/{B}", flush=True)
    for mu_s in MUS:
        t0 = time.time()
        acc, gaps, dobj, dW0, saved, fin64, n32, reasons = [], [], [], [], [], [], [], {}
        for bi in range(B):
            R = np.exp(y[bi]).astype(np.float64)
            # the iterate at mu <= mu_s (float32 phase, or float64 from scratch with F64=1), then
            # one more float64 iteration (the Tapia classification compares the two)
            s1, it32, state0, _, _, mu0 = phase(libs["d" if F64 else "f"], wp[bi], y[bi], c, tau, mu_s)
            if s1 != 100:      # the float32 phase ended otherwise (stagnation handoff counts as 100)
                reasons["no handoff"] = reasons.get("no handoff", 0) + 1
                acc.append(False)
                continue
            s1b, _, state, _, _, _ = phase(libs["d"], wp[bi], y[bi], c, tau, mu0 * 0.99999, st_in=state0)
            if s1b != 100:
                reasons["converged in one step"] = reasons.get("converged in one step", 0) + 1
                acc.append(False)
                continue
            n32.append(it32 + 1)
            s2, it64, _, W64, ob64, _ = phase(libs["d"], wp[bi], y[bi], c, tau, 0.0, st_in=state)
            fin64.append(it64)
            try:
                W, ok, info = polish(state, wp[bi], R, c, tau, st0=state0)
            except np.linalg.LinAlgError:
                W, ok, info = None, False, {"why": "LinAlgError"}
            if W is None or not ok:
                reasons["infeasible face"] = reasons.get("infeasible face", 0) + 1
                if DEBUG:
                    print(bi, info, flush=True)
                acc.append(False)
                continue
            r = cert.certify(W, wp[bi], y[bi], c, tau)
            bar = 1e-6 + 1e-5 * abs(r["f"])
            good = r["gap"] <= bar and r["violation"] <= 1e-8
            if not good:
                reasons["certificate"] = reasons.get("certificate", 0) + 1
            acc.append(good)
            gaps.append(r["gap"] / (1 + abs(r["f"])))
            if good:
                dobj.append(abs(-r["f"] - objl[bi]))
                dW0.append(float(np.abs(W[0] - Wl[bi, 0]).max()))
                saved.append(it64)
        acc = np.array(acc)
        print({"mu_s": mu_s, "windows": B, "accepted": int(acc.sum()), "rate": float(acc.mean()),
               "reasons": reasons, "f32_iters": float(np.mean(n32)) if n32 else None,
               "f64_finish_iters_mean": float(np.mean(fin64)) if fin64 else None,
               "f64_iters_saved_mean_over_all": float(np.sum(saved) / B),
               "gap_rel_median": float(np.median(gaps)) if gaps else None,
               "gap_rel_max_accepted": float(max(g for g, a in zip(gaps, acc[acc | ~acc]) if a)) if acc.any() else None,
               "max_dobj_vs_ld_oracle": float(max(dobj)) if dobj else None,
               "max_dW0_vs_ld_oracle": float(max(dW0)) if dW0 else None,
               "sec": round(time.time() - t0, 1)}, flush=True)


if __name__ == "__main__":
    main()
