"""Mean-variance MPC and Markowitz restatement — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use this
module, as the checker of the device path; the product never imports it.

Reference semantics restated here (reference files, read as text):

* ``solve_mpc_mean_variance`` (mpc.py:119-184)::

      maximize  sum_t [ w_t . mu_t - gamma * w_t' Sigma w_t ] - c sum_t ||w_t - w_{t-1}||_1
      s.t.      1' w_t = 1,  w_t >= 0 unless allow_short           (no turnover cap)

  with w_{-1} = current_weights (mpc.py:145-146, 166-169); a status outside
  {optimal, optimal_inaccurate} returns ``tile(current_weights)`` and ``{"status": s}`` only
  (mpc.py:180-181, no "value" key).
* ``MarkowitzStrategy.rebalance`` (baselines.py:48-106): past returns = de-standardized first
  embedding block of test rows [0, t] (float32, baselines.py:71-73); fewer than 5 rows -> hold
  ``current_weights`` (baselines.py:76-78); window = last ``lookback_window`` rows
  (baselines.py:81); mu = np.mean (float32), Sigma = np.cov(rowvar=False) (float64) + 1e-6 I
  (baselines.py:84-88); H = 1 solve with gamma = risk_aversion (baselines.py:39-45, 98-106).

cvxpy (pinned 1.7.5 / SCS 3.2.9 in the reference uv.lock) is not installed, so the reference's
own solve cannot run here: :func:`mv_dense_ipm` restates the program's optimum (dense-KKT
Mehrotra interior point, float64) and is pinned by :func:`mv_slsqp` (an unrelated algorithm) and
by closed forms in ``tests/test_mv_cpu.py``.
"""
from __future__ import annotations

import numpy as np


def mv_objective(W, w_prev, mu, sigma, gamma, cost):
    """problem.value of mpc.py:172 (maximize form) at W [H, N]."""
    W = np.asarray(W, np.float64)
    mu = np.asarray(mu, np.float64)
    S = np.asarray(sigma, np.float64)
    f = float(np.sum(W * mu)) - gamma * float(np.einsum("hi,ij,hj->", W, S, W))
    prev = np.asarray(w_prev, np.float64)
    for t in range(W.shape[0]):
        f -= cost * float(np.abs(W[t] - prev).sum())
        prev = W[t]
    return f


def mv_dense_ipm(w_prev, mu, sigma, gamma, cost, allow_short=False, iters=200, tol=1e-13):
    """Dense-KKT Mehrotra IPM on the epigraph form (variables w [HN], s [HN] when cost > 0).

    Returns (W [H, N], status) with status "optimal", "unbounded" or "solver_error".
    """
    wp = np.asarray(w_prev, np.float64)
    mu = np.asarray(mu, np.float64)
    S = np.asarray(sigma, np.float64)
    H, N = mu.shape
    n = H * N
    use_s = cost > 0
    if allow_short and not use_s and not gamma > 0:
        # a linear program over the budget planes: unbounded unless every period is flat
        if np.ptp(mu, axis=1).max() > 0:
            return np.tile(wp, (H, 1)), "unbounded"
        return np.tile(wp / wp.sum(), (H, 1)), "optimal"
    nx = n + (n if use_s else 0)
    # inequality rows G x - h >= 0
    G, h = [], []
    if not allow_short:
        for k in range(n):
            r = np.zeros(nx); r[k] = 1.0
            G.append(r); h.append(0.0)
    if use_s:
        for t in range(H):
            for i in range(N):
                for sgn in (-1.0, 1.0):
                    r = np.zeros(nx)
                    r[n + t * N + i] = 1.0
                    r[t * N + i] += sgn
                    rhs = 0.0
                    if t > 0:
                        r[(t - 1) * N + i] -= sgn
                    else:
                        rhs = sgn * wp[i]
                    G.append(r); h.append(rhs)
    G = np.array(G).reshape(-1, nx)
    h = np.array(h)
    m = G.shape[0]
    A = np.zeros((H, nx))
    for t in range(H):
        A[t, t * N:(t + 1) * N] = 1.0
    b = np.ones(H)
    # minimize 0.5 x'Qx + q'x
    Q = np.zeros((nx, nx))
    for t in range(H):
        Q[t * N:(t + 1) * N, t * N:(t + 1) * N] = 2.0 * gamma * S
    q = np.zeros(nx)
    q[:n] = -mu.ravel()
    if use_s:
        q[n:] = cost
    scale = max(np.abs(q).max(), np.abs(Q).max(), 1e-300)
    Q, q = Q / scale, q / scale
    x = np.zeros(nx)
    w0 = 0.5 * (np.maximum(wp, 0.0) if not allow_short else wp) + 0.5 / N
    x[:n] = np.tile(w0, H)
    if use_s:
        d = np.diff(np.vstack([wp, x[:n].reshape(H, N)]), axis=0)
        x[n:] = np.abs(d).ravel() + 1.0 / N
    z = np.maximum(G @ x - h, 1e-2) if m else np.zeros(0)   # slacks kept as variables
    lam = np.ones(m)
    nu = np.zeros(H)
    status = "solver_error"
    best, best_x = np.inf, x.copy()
    for _ in range(iters):
        rd = Q @ x + q - G.T @ lam + A.T @ nu
        rp = A @ x - b
        rg = G @ x - h - z
        mu_c = (z @ lam) / max(m, 1)
        if np.abs(x[:n]).max() > 1e7:
            return x[:n].reshape(H, N), "unbounded"
        merit = max(mu_c, np.abs(rd).max(), np.abs(rp).max(), np.abs(rg).max() if m else 0.0)
        if not np.isfinite(merit):
            break
        if merit < best:
            best, best_x = merit, x.copy()
        if mu_c < tol and np.abs(rd).max() < 10 * tol and np.abs(rp).max() < 10 * tol and (
                m == 0 or np.abs(rg).max() < 10 * tol):
            status = "optimal"
            break
        Wd = lam / z if m else np.zeros(0)
        M = Q + (G.T @ (Wd[:, None] * G) if m else 0.0)
        K = np.block([[M, A.T], [A, np.zeros((H, H))]])

        def solve(rc):
            rhs1 = -rd - (G.T @ (Wd * rg + rc / z) if m else 0.0)
            try:
                sol = np.linalg.solve(K, np.concatenate([rhs1, -rp]))
            except np.linalg.LinAlgError:
                return None
            dx, dnu = sol[:nx], sol[nx:]
            dz = G @ dx + rg
            dlam = -(lam * dz + rc) / z
            return dx, dnu, dlam, dz

        def maxstep(v, dv):
            neg = dv < 0
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0

        r = solve(z * lam)
        if r is None:
            break
        dx, dnu, dlam, dz = r
        a = min(maxstep(z, dz), maxstep(lam, dlam)) if m else 1.0
        mua = (z + a * dz) @ (lam + a * dlam) / max(m, 1)
        sig = (mua / mu_c) ** 3 if m else 0.0
        r = solve(z * lam + dz * dlam - sig * mu_c)
        if r is None:
            break
        dx, dnu, dlam, dz = r
        a = min(1.0, 0.99 * min(maxstep(z, dz), maxstep(lam, dlam))) if m else 1.0
        x += a * dx
        nu += a * dnu
        lam += a * dlam
        z += a * dz
    if status != "optimal":
        x = best_x
        status = "optimal" if best <= 1e-9 else ("optimal_inaccurate" if best <= 1e-6 else "solver_error")
    return x[:n].reshape(H, N), status


def mv_slsqp(w_prev, mu, sigma, gamma, cost, allow_short=False):
    """scipy SLSQP on the lifted L1 form (w_t - w_{t-1} = u_t - v_t, u, v >= 0)."""
    from scipy.optimize import minimize

    wp = np.asarray(w_prev, np.float64)
    mu = np.asarray(mu, np.float64)
    S = np.asarray(sigma, np.float64)
    H, N = mu.shape
    n = H * N

    def unpack(v):
        return v[:n].reshape(H, N), v[n:2 * n].reshape(H, N), v[2 * n:].reshape(H, N)

    def f(v):
        W, U, V = unpack(v)
        return -(float(np.sum(W * mu)) - gamma * float(np.einsum("hi,ij,hj->", W, S, W))
                 - cost * (U.sum() + V.sum()))

    cons = []
    for t in range(H):
        cons.append({"type": "eq", "fun": (lambda v, t=t: unpack(v)[0][t].sum() - 1.0)})

        def dif(v, t=t):
            W, U, V = unpack(v)
            prev = wp if t == 0 else W[t - 1]
            return W[t] - prev - U[t] + V[t]

        cons.append({"type": "eq", "fun": dif})
    lb = None if allow_short else 0.0
    bounds = [(lb, None)] * n + [(0.0, None)] * (2 * n)
    v0 = np.concatenate([np.tile(wp, H), np.zeros(2 * n)])
    r = minimize(f, v0, method="SLSQP", bounds=bounds, constraints=cons,
                 options={"ftol": 1e-15, "maxiter": 5000})
    return unpack(r.x)[0], bool(r.success)


def solve_mpc_mean_variance_ref(current_weights, predicted_log_returns, cov_matrix, gamma, cost,
                                allow_short=False):
    """mpc.py:119-184 restated: (W [H, N], info) with the reference's fallback."""
    W, st = mv_dense_ipm(current_weights, predicted_log_returns, cov_matrix, gamma, cost, allow_short)
    if st not in ("optimal", "optimal_inaccurate"):
        H = np.asarray(predicted_log_returns).shape[0]
        return np.tile(np.asarray(current_weights, np.float64), (H, 1)), {"status": st}
    return W, {"status": st, "value": mv_objective(W, current_weights, predicted_log_returns,
                                                   cov_matrix, gamma, cost)}


def rolling_moments(past_returns_f32, lookback=60):
    """baselines.py:81-88: mu (float32 np.mean), Sigma (np.cov, float64) + 1e-6 I of the last
    ``lookback`` rows of a float32 [t+1, N] return history; None when fewer than 5 rows."""
    R = np.asarray(past_returns_f32, np.float32)
    if len(R) < 5:
        return None
    window = R[-lookback:]
    mu = np.mean(window, axis=0)
    sigma = np.cov(window, rowvar=False)
    sigma = sigma + np.eye(len(mu)) * 1e-6
    return mu, sigma
