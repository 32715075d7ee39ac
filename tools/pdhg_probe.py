#!/usr/bin/env python3
"""Dev measurement (CPU only): first-order solvers for the reference program
against the interior point, on the bench's own C3 windows.

north_star names "a batched ADMM / projected-gradient kernel"; the reference's own solver, SCS
(mpc.py:107-111), is an ADMM. This probe runs a Condat-Vu primal-dual (PDHG) iteration on

    min_W  -sum_t log(R_t . w_t) + c sum_t ||d_t||_1   s.t.  w_t in simplex,  ||d_t||_1 <= tau,
           d = K W - b  (d_t = w_t - w_{t-1}, w_{-1} = w_prev)

    W+ = proj_simplex(W - s (grad f(W) + K^T Y))                       (per period: sort projection)
    Y+ = prox_{r g*}(Y + r (K (2 W+ - W) - b)),  g(d) = sum_t c ||d_t||_1 + [||d_t||_1 <= tau]
         (Moreau: prox_{g/r} is soft(u, c/r) followed, when needed, by the L1-ball projection)

vectorised over windows in numpy, in float64 and float32, with restarts to the running average
every 500 iterations (or none), over a small grid of primal weights (s / r). Reported per precision: the
iterations until every window's objective is within the kernels' bar 1e-6 + 1e-5 |f*| of the
long-double oracle with turnover violation <= 1e-6, the same at SCS's default eps 1e-4 (relative
objective and violation), and the FLOPs that takes against the interior point's (bench.py
solve_flop_model x the oracle's iteration count).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def proj_simplex(V):
    """Euclidean projection of every row (last axis) onto the probability simplex."""
    n = V.shape[-1]
    U = -np.sort(-V, axis=-1)
    css = np.cumsum(U, axis=-1) - 1
    k = np.arange(1, n + 1, dtype=V.dtype)
    cond = U - css / k > 0
    rho = n - 1 - np.argmax(cond[..., ::-1], axis=-1)
    theta = np.take_along_axis(css, rho[..., None], -1) / (rho[..., None] + 1).astype(V.dtype)
    return np.maximum(V - theta, 0)


def soft(V, t):
    return np.sign(V) * np.maximum(np.abs(V) - t, 0)


def prox_l1_cap(U, lam, tau):
    """argmin_d lam ||d||_1 + [||d||_1 <= tau] + 1/2 ||d - u||^2 per row: soft(u, max(lam, theta))
    with theta the L1-ball threshold of u (soft(u, theta) has norm tau)."""
    lam = np.broadcast_to(np.asarray(lam, U.dtype), U.shape[:-1] + (1,))
    D = soft(U, lam)
    over = np.abs(D).sum(-1) > tau
    if over.any():
        A = -np.sort(-np.abs(U[over]), axis=-1)
        n = A.shape[-1]
        css = np.cumsum(A, axis=-1) - tau
        k = np.arange(1, n + 1, dtype=U.dtype)
        cond = A - css / k > 0
        rho = n - 1 - np.argmax(cond[..., ::-1], axis=-1)
        theta = np.take_along_axis(css, rho[..., None], -1) / (rho[..., None] + 1).astype(U.dtype)
        D[over] = soft(U[over], np.maximum(theta, lam[over]))
    return D


def objective(W, wp, R, c):
    D = np.diff(np.concatenate([wp[:, None], W], 1), axis=1)
    return -np.log(np.einsum("bhn,bhn->bh", R, W)).sum(-1) + c * np.abs(D).sum((-1, -2)), D


def pdhg(wp, R, c, tau, fstar, dtype, weight, max_iter=20000, restart=True):
    """Returns the iteration counts at which the kernel bar / the SCS-like bar first hold for every
    window (None if not within max_iter)."""
    B, H, N = R.shape
    R = R.astype(dtype)
    wp = wp.astype(dtype)
    # restricted (simplex tangent) curvature of f: ||m_t - mean m_t||^2 / (R.w)^2, (R.w) >= min R
    m = R - R.mean(-1, keepdims=True)
    L = ((m * m).sum(-1) / (R.min(-1) ** 2)).max(-1)                       # [B]
    nK2 = 4.0
    # Condat-Vu step rule s (L / 2 + r ||K||^2) <= 1 with r = s / weight^2 (0.99 of the bound)
    a = nK2 / weight ** 2
    s = 0.99 * (-L / 2 + np.sqrt(L * L / 4 + 4 * a)) / (2 * a)
    r = s / weight ** 2
    s = s.astype(dtype)[:, None, None]
    r = r.astype(dtype)[:, None, None]
    W = np.repeat(wp[:, None], H, 1)
    Y = np.zeros_like(W)
    bar = 1e-6 + 1e-5 * np.abs(fstar)
    hit_k = hit_s = None
    Wavg, Yavg, navg = np.zeros_like(W), np.zeros_like(Y), 0
    last_err = None
    for k in range(1, max_iter + 1):
        Rw = np.einsum("bhn,bhn->bh", R, W)
        grad = -R / Rw[..., None]
        KtY = Y - np.concatenate([Y[:, 1:], np.zeros_like(Y[:, :1])], 1)          # K^T Y
        Wn = proj_simplex(W - s * (grad + KtY))
        X = 2 * Wn - W
        KX = np.diff(np.concatenate([wp[:, None], X], 1), axis=1)
        V = Y + r * KX
        Yn = V - r * prox_l1_cap(V / r, c / r, tau)
        W, Y = Wn, Yn
        Wavg += W
        Yavg += Y
        navg += 1
        if k % 10 == 0:
            f, D = objective(W.astype(np.float64), wp.astype(np.float64), R.astype(np.float64), c)
            viol = np.maximum(np.abs(D).sum(-1) - tau, 0).max(-1)
            err = np.abs(f - fstar)
            if os.environ.get("PDHG_TRACE") and k in (10, 100, 300, 1000, 3000, 10000):
                print(k, "err p50/max", np.median(err), err.max(), "viol max", viol.max(), "rel", (err / np.abs(fstar)).max(), flush=True)
            if hit_s is None and ((err <= 1e-4 * np.maximum(1, np.abs(fstar))) & (viol <= 1e-4)).all():
                hit_s = k
            if hit_k is None and ((err <= bar) & (viol <= 1e-6)).all():
                hit_k = k
                break
            if restart and k % restart == 0:
                # restart to the running average (the averaged iterate of PDHG converges at O(1/k)
                # and restarting it is what makes restarted PDHG linear on sharp problems)
                W, Y = (Wavg / navg).astype(dtype), (Yavg / navg).astype(dtype)
                Wavg[:], Yavg[:], navg = 0, 0, 0
    f, D = objective(W.astype(np.float64), wp.astype(np.float64), R.astype(np.float64), c)
    viol = np.maximum(np.abs(D).sum(-1) - tau, 0).max(-1)
    final = {"max_err_over_bar": float((np.abs(f - fstar) / bar).max()),
             "median_err_over_bar": float(np.median(np.abs(f - fstar) / bar)), "max_violation": float(viol.max())}
    return hit_k, hit_s, final


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    import f32phase_probe as fp
    import bench
    from oracle import solver as osolver
    c, tau = 1e-3, 0.2
    wp, y = fp.windows(B)
    R = np.exp(y).astype(np.float64)          # np.exp on float32 (mpc.py:55)
    Wl, stl, objl, itl = osolver.solve_batch(wp, y, c, tau, False, precision="ld", tol=1e-9)
    fstar = -objl                              # minimisation form
    ipm_iters = float(itl.mean())
    ipm_flops = bench.solve_flop_model(100, 10)["per_iteration"] * ipm_iters
    # PDHG FLOPs per iteration (per window): gradient 3 HN, K^T Y 1, projection step 2, simplex
    # projection (sort ~ N log2 N compares counted as flops + 4 HN), K X 2, dual step 2, L1 prox
    # (soft 3 + ball sort on the capped periods ~ N log2 N + 4 HN), objective checks not counted
    HN = 10 * 100
    per_it = HN * (3 + 1 + 2 + 4 + 2 + 2 + 3 + 4) + 2 * 10 * 100 * np.log2(100)
    print(f"windows {B}; interior point (oracle): {ipm_iters:.2f} iterations, {ipm_flops / 1e6:.2f} MFLOP/window; "
          f"PDHG ~{per_it / 1e3:.1f} kFLOP/iteration/window", flush=True)
    for dtype in (np.float64, np.float32):
        for weight in (1.0, 3.0, 10.0):
            for restart in (0, 500):
                t0 = time.time()
                hk, hs, final = pdhg(wp, R, c, tau, fstar, dtype, weight, max_iter, restart)
                row = {"dtype": np.dtype(dtype).name, "primal_weight": weight, "restart": restart,
                       "iters_kernel_bar": hk, "iters_scs_eps_1e-4": hs,
                       "mflop_kernel_bar": None if hk is None else hk * per_it / 1e6,
                       "mflop_scs_eps": None if hs is None else hs * per_it / 1e6,
                       "at_max_iter": final, "sec": round(time.time() - t0, 1)}
                print(row, flush=True)


if __name__ == "__main__":
    main()
