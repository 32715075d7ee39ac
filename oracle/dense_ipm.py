"""Independent solvers for the reference MPC program — TEST INFRASTRUCTURE ONLY.

Two deliberately simple float64 solvers of the program in ``mpc.py:49-117`` of the reference
(``solve_mpc_log_utility``), used only to pin ``oracle/kmpc_oracle.c`` on small instances:

* :func:`dense_ipm`  — textbook primal-dual (Mehrotra) interior point on the epigraph form with
  the FULL dense KKT matrix solved by LAPACK (no structure exploited; O((HN)^3) per step).
* :func:`slsqp`      — scipy SLSQP on the lifted L1 form ``w_t - w_{t-1} = u_t - v_t``, u, v >= 0,
  i.e. an algorithm unrelated to interior points.

Both use the reference's objective verbatim: ``sum_t log(w_t . R_t) - c sum_t ||w_t - w_{t-1}||_1``
with ``R = np.exp(yhat)`` evaluated on the float32 yhat exactly as the reference does (mpc.py:55;
cvxpy then works with R in float64) (mpc.py:66-103), constraints ``sum w_t = 1`` (mpc.py:83), ``w >= 0`` unless allow_short
(mpc.py:85-86) and ``||w_t - w_{t-1}||_1 <= tau`` when tau > 0 (mpc.py:94-100).
"""
from __future__ import annotations

import numpy as np


def gross_returns(y):
    """R = np.exp(yhat) on the float32 yhat (mpc.py:55), promoted to float64 as cvxpy sees it."""
    return np.exp(np.asarray(y, np.float32)).astype(np.float64)


def reference_objective(W, w_prev, y, cost):
    """problem.value of mpc.py:103 evaluated at W (float64)."""
    W = np.asarray(W, np.float64)
    R = gross_returns(y)
    f = float(np.sum(np.log(np.einsum("hn,hn->h", R, W))))
    prev = np.asarray(w_prev, np.float64)
    for t in range(W.shape[0]):
        f -= cost * float(np.abs(W[t] - prev).sum())
        prev = W[t]
    return f


def _build(wp, y, c, tau, allow_short):
    H, N = y.shape
    nw = H * N
    use_s = (c > 0) or (tau > 0)
    nx = nw + (nw if use_s else 0)
    G, h = [], []
    if not allow_short:
        for k in range(nw):
            row = np.zeros(nx)
            row[k] = 1.0
            G.append(row)
            h.append(0.0)
    if use_s:
        for t in range(H):
            for i in range(N):
                for sgn in (-1.0, 1.0):
                    # s_ti + sgn * (w_ti - w_{t-1,i}) >= 0
                    row = np.zeros(nx)
                    row[nw + t * N + i] = 1.0
                    row[t * N + i] += sgn
                    rhs = 0.0
                    if t > 0:
                        row[(t - 1) * N + i] -= sgn
                    else:
                        rhs = sgn * wp[i]
                    G.append(row)
                    h.append(rhs)
        if tau > 0:
            for t in range(H):
                row = np.zeros(nx)
                row[nw + t * N: nw + (t + 1) * N] = -1.0
                G.append(row)
                h.append(-tau)
    A = np.zeros((H, nx))
    for t in range(H):
        A[t, t * N:(t + 1) * N] = 1.0
    cvec = np.zeros(nx)
    if use_s:
        cvec[nw:] = c
    return np.array(G).reshape(-1, nx), np.array(h), A, np.ones(H), cvec, nw


def dense_ipm(w_prev, y, cost, tau, allow_short=False, iters=100, tol=1e-12):
    """Dense-KKT Mehrotra IPM. Returns (W [H,N], converged: bool)."""
    wp = np.asarray(w_prev, np.float64)
    m = gross_returns(y) - 1.0  # log(R.w) == log(1 + m.w) on sum(w) = 1
    y = np.asarray(y, np.float64)
    H, N = y.shape
    from scipy.linalg import lu_factor, lu_solve
    from scipy.sparse import csr_matrix, diags
    G, h, A, b, cvec, nw = _build(wp, y, cost, tau, allow_short)
    Gs = csr_matrix(G)        # (the KKT matrix below is still formed and factored densely)
    nx = G.shape[1]
    mi = G.shape[0]
    x = np.zeros(nx)
    x[:nw] = np.tile(wp, H)
    if nx > nw:
        Wt = x[:nw].reshape(H, N)
        d = np.diff(np.vstack([wp, Wt]), axis=0)
        x[nw:] = np.abs(d).ravel() + 0.01
    z = np.maximum(G @ x - h, 1e-2) if mi else np.zeros(0)
    lam = np.ones(mi)
    nu = np.zeros(H)
    converged = False
    for _ in range(iters):
        g = cvec.copy()
        Hf = np.zeros((nx, nx))
        for t in range(H):
            wt = x[t * N:(t + 1) * N]
            den = 1.0 + m[t] @ wt
            g[t * N:(t + 1) * N] -= m[t] / den
            Hf[t * N:(t + 1) * N, t * N:(t + 1) * N] += np.outer(m[t], m[t]) / den ** 2
        rd = g - G.T @ lam + A.T @ nu
        rp = A @ x - b
        rg = G @ x - h - z
        mu = (z @ lam) / max(mi, 1)
        if mu < tol and np.abs(rd).max() < 10 * tol and np.abs(rp).max() < 10 * tol and (
                mi == 0 or np.abs(rg).max() < 10 * tol):
            converged = True
            break
        Wd = lam / z
        M = Hf + (Gs.T @ diags(Wd) @ Gs).toarray()
        K = np.block([[M, A.T], [A, np.zeros((H, H))]])
        lu = lu_factor(K)

        def solve(rc):
            rhs1 = -rd - G.T @ (Wd * rg + rc / z)
            sol = lu_solve(lu, np.concatenate([rhs1, -rp]))
            dx, dnu = sol[:nx], sol[nx:]
            dlam = -Wd * (G @ dx + rg) - rc / z
            dz = G @ dx + rg
            return dx, dnu, dlam, dz

        def maxstep(v, dv):
            neg = dv < 0
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0

        dx, dnu, dlam, dz = solve(z * lam)
        a = min(maxstep(z, dz), maxstep(lam, dlam))
        mua = (z + a * dz) @ (lam + a * dlam) / max(mi, 1)
        sig = (mua / mu) ** 3
        dx, dnu, dlam, dz = solve(z * lam + dz * dlam - sig * mu)
        a = 0.99 * min(maxstep(z, dz), maxstep(lam, dlam))
        x += a * dx
        nu += a * dnu
        lam += a * dlam
        z += a * dz
    return x[:nw].reshape(H, N), converged


def slsqp(w_prev, y, cost, tau, allow_short=False):
    """scipy SLSQP on the lifted L1 form. Returns (W [H,N], success: bool)."""
    from scipy.optimize import minimize

    wp = np.asarray(w_prev, np.float64)
    R = gross_returns(y)
    y = np.asarray(y, np.float64)
    H, N = y.shape
    n = H * N

    def unpack(v):
        return v[:n].reshape(H, N), v[n:2 * n].reshape(H, N), v[2 * n:].reshape(H, N)

    def f(v):
        W, U, V = unpack(v)
        return -(float(np.sum(np.log(np.einsum("hn,hn->h", R, W)))) - cost * (U.sum() + V.sum()))

    cons = []
    for t in range(H):
        cons.append({"type": "eq", "fun": (lambda v, t=t: unpack(v)[0][t].sum() - 1.0)})

        def dif(v, t=t):
            W, U, V = unpack(v)
            prev = wp if t == 0 else W[t - 1]
            return W[t] - prev - U[t] + V[t]

        cons.append({"type": "eq", "fun": dif})
        if tau > 0:
            cons.append({"type": "ineq",
                         "fun": (lambda v, t=t: tau - unpack(v)[1][t].sum() - unpack(v)[2][t].sum())})
    lb = None if allow_short else 0.0
    bounds = [(lb, None)] * n + [(0.0, None)] * (2 * n)
    v0 = np.concatenate([np.tile(wp, H), np.zeros(2 * n)])
    r = minimize(f, v0, method="SLSQP", bounds=bounds, constraints=cons,
                 options={"ftol": 1e-14, "maxiter": 3000})
    return unpack(r.x)[0], bool(r.success)
