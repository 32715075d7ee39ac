"""Optimality certificates for the log-utility MPC program — TEST INFRASTRUCTURE ONLY.

Only tests/ import this module. It certifies a candidate W of the reference program
(mpc.py:49-117, solve_mpc_log_utility) by weak duality. It does not use the interior-point
iteration the oracle and the kernels share.

In minimisation form, with R_t = np.exp(yhat_t) in float32 (mpc.py:55) and d_t = w_t - w_{t-1}
(w_{-1} = w_prev), the reference program is

    p* = min  sum_t -log(R_t . w_t) + c sum_t ||d_t||_1
         s.t. 1'w_t = 1,  w_t >= 0,  ||d_t||_1 <= tau  (tau > 0; no cap otherwise).

Introduce u_t = R_t . w_t with multiplier y_t > 0, d_t = w_t - w_{t-1} with multiplier z_t in
R^N, and 1'w_t = 1 with multiplier nu_t. Minimising the Lagrangian over u > 0, ||d_t||_1 <= tau
and w >= 0 gives, for ANY y > 0 and z (z_H = 0),

    g(y, z) = sum_t [1 + log y_t + nu_t(y, z) - tau max(0, ||z_t||_inf - c)] + z_0 . w_prev
    nu_t    = min_i (z_{t+1,i} - z_{t,i} - y_t R_{t,i})

and g(y, z) <= p*. Without a cap the d-term requires ||z_t||_inf <= c (z is clipped into that
box, which keeps g a valid bound). So for a feasible W, gap = f(W) - g(y, z) >= 0 bounds how far W
is from optimal, whatever produced W, y and z.

The dual point used here:
* y_t = 1 / (R_t . w_t), from the candidate itself (stationarity in u);
* z is the maximiser of g(y, .) for that y. This is a linear program, solved by HiGHS dual
  simplex (scipy.optimize.linprog), a vertex method unrelated to interior points.

The soundness of the bound does not depend on the LP solve: g is re-evaluated in float64 from z
with the formula above. Maximisation values (problem.value in the reference) are -f and -g.
"""
from __future__ import annotations

import numpy as np


def gross_returns(y):
    """R = np.exp(yhat) on the float32 yhat (mpc.py:55), as float64."""
    return np.exp(np.asarray(y, np.float32)).astype(np.float64)


def primal_value(W, w_prev, yhat, cost):
    """f(W) = sum_t -log(R_t . w_t) + c sum_t ||w_t - w_{t-1}||_1 (minimisation form)."""
    W = np.asarray(W, np.float64)
    R = gross_returns(yhat)
    D = np.diff(np.vstack([np.asarray(w_prev, np.float64)[None], W]), axis=0)
    return float(-np.log(np.einsum("hn,hn->h", R, W)).sum() + cost * np.abs(D).sum())


def primal_violation(W, w_prev, tau, allow_short=False):
    """Largest violation of the budget, no-short and turnover-cap constraints."""
    W = np.asarray(W, np.float64)
    D = np.diff(np.vstack([np.asarray(w_prev, np.float64)[None], W]), axis=0)
    v = float(np.abs(W.sum(1) - 1.0).max())
    if not allow_short:
        v = max(v, float(max(0.0, -W.min())))
    if tau > 0:
        v = max(v, float(max(0.0, (np.abs(D).sum(1) - tau).max())))
    return v


def dual_value(y, z, w_prev, yhat, cost, tau):
    """g(y, z) of the module docstring (no shorting): a lower bound on p* for any y > 0, z."""
    R = gross_returns(yhat)
    H, N = R.shape
    y = np.asarray(y, np.float64)
    z = np.asarray(z, np.float64)
    if not tau > 0:
        z = np.clip(z, -cost, cost)     # the d-term is -inf outside the box when uncapped
    zn = np.vstack([z[1:], np.zeros((1, N))])
    nu = (zn - z - y[:, None] * R).min(1)
    cap = tau * np.maximum(0.0, np.abs(z).max(1) - cost) if tau > 0 else np.zeros(H)
    return float(np.sum(1.0 + np.log(y) + nu - cap) + z[0] @ np.asarray(w_prev, np.float64))


def best_z(y, w_prev, yhat, cost, tau):
    """argmax_z g(y, z) as an LP: variables z [H,N] (free), nu [H] (free), kappa [H] >= 0.
        max  sum nu_t - tau sum kappa_t + z_0 . w_prev
        s.t. nu_t - z_{t+1,i} + z_{t,i} <= -y_t R_{t,i};  |z_{t,i}| <= c + kappa_t
    (kappa = 0 without a cap)."""
    from scipy.optimize import linprog
    from scipy.sparse import coo_matrix, vstack

    R = gross_returns(yhat)
    H, N = R.shape
    nz = H * N
    nv = nz + 2 * H
    iz = lambda t, i: t * N + i          # noqa: E731
    inu = lambda t: nz + t               # noqa: E731
    ika = lambda t: nz + H + t           # noqa: E731
    obj = np.zeros(nv)
    obj[[inu(t) for t in range(H)]] = -1.0
    if tau > 0:
        obj[[ika(t) for t in range(H)]] = tau
    obj[:N] -= np.asarray(w_prev, np.float64)
    rows, cols, vals, rhs = [], [], [], []
    r = 0
    for t in range(H):
        for i in range(N):
            rows += [r, r]
            cols += [inu(t), iz(t, i)]
            vals += [1.0, 1.0]
            if t + 1 < H:
                rows.append(r)
                cols.append(iz(t + 1, i))
                vals.append(-1.0)
            rhs.append(-y[t] * R[t, i])
            r += 1
    A1 = coo_matrix((vals, (rows, cols)), shape=(r, nv))
    rows, cols, vals, rhs2 = [], [], [], []
    r = 0
    for t in range(H):
        for i in range(N):
            for sg in (1.0, -1.0):
                rows += [r, r]
                cols += [iz(t, i), ika(t)]
                vals += [sg, -1.0]
                rhs2.append(cost)
                r += 1
    A2 = coo_matrix((vals, (rows, cols)), shape=(r, nv))
    bounds = [(None, None)] * (nz + H) + ([(0, None)] * H if tau > 0 else [(0, 0)] * H)
    res = linprog(obj, A_ub=vstack([A1, A2]).tocsr(), b_ub=np.array(rhs + rhs2), bounds=bounds,
                  method="highs-ds", options={"primal_feasibility_tolerance": 1e-10,
                                              "dual_feasibility_tolerance": 1e-10})
    if res.status != 0:
        raise RuntimeError(f"certificate LP failed: {res.message}")
    return res.x[:nz].reshape(H, N)


def certify(W, w_prev, yhat, cost, tau):
    """Duality gap of the candidate W (no shorting). Returns a dict with the primal value f, the
    dual bound g (both in minimisation form), gap = f - g and the primal violation."""
    W = np.asarray(W, np.float64)
    R = gross_returns(yhat)
    y = 1.0 / np.einsum("hn,hn->h", R, W)
    z = best_z(y, w_prev, yhat, cost, tau)
    f = primal_value(W, w_prev, yhat, cost)
    g = dual_value(y, z, w_prev, yhat, cost, tau)
    return {"f": f, "g": g, "gap": f - g, "violation": primal_violation(W, w_prev, tau)}
