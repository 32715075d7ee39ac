"""Generate tests/golden/mv_*.npz: mean-variance MPC problems (mpc.py:119-184) and Markowitz
windows (baselines.py:48-106) with the float64 oracle optimum (oracle/mv_ref.py).

The reference's own mean-variance solve needs cvxpy (not installed, no network), so the expected
outputs come from the oracle, which tests/test_mv_cpu.py pins against scipy SLSQP and closed forms.
Inputs are synthetic and seeded. Data only (no code) is stored.

    python tests/golden/make_mv_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import mv_ref  # noqa: E402


def problems(seed, B, N, H, gamma, cost, short):
    rng = np.random.default_rng(seed)
    wp = rng.dirichlet(np.ones(N), B)
    mu = rng.normal(5e-4, 0.01, (B, H, N))
    X = rng.normal(5e-4, 0.015, (B, 60, N))
    S = np.stack([np.cov(x, rowvar=False) + 1e-6 * np.eye(N) for x in X])
    W = np.zeros((B, H, N))
    obj = np.zeros(B)
    st = np.zeros(B, np.int32)
    for b in range(B):
        Wb, s = mv_ref.mv_dense_ipm(wp[b], mu[b], S[b], gamma, cost, short)
        W[b] = Wb
        st[b] = 0 if s == "optimal" else 4
        obj[b] = mv_ref.mv_objective(Wb, wp[b], mu[b], S[b], gamma, cost)
    return dict(w_prev=wp, mu=mu, sigma=S, W=W, obj=obj, status=st,
                gamma=gamma, cost=cost, allow_short=int(short))


def markowitz(seed, T, N, ts):
    """Rolling windows over a float32 return panel: moments + H=1 optimum (gamma 1, cost 1e-3)."""
    rng = np.random.default_rng(seed)
    z = rng.normal(0, 1, (T, N)).astype(np.float32)
    mean = rng.normal(5e-4, 1e-4, N).astype(np.float32)
    std = rng.uniform(0.01, 0.02, N).astype(np.float32)
    R = z * std + mean                      # float32 destandardize (data_finance.py:740-742)
    wp = rng.dirichlet(np.ones(N), len(ts))
    out_mu = np.zeros((len(ts), N))
    out_S = np.zeros((len(ts), N, N))
    W0 = np.zeros((len(ts), N))
    valid = np.zeros(len(ts), np.int32)
    for b, t in enumerate(ts):
        m = mv_ref.rolling_moments(R[:t + 1])
        if m is None:
            W0[b] = wp[b]
            continue
        valid[b] = 1
        out_mu[b], out_S[b] = m
        W, info = mv_ref.solve_mpc_mean_variance_ref(wp[b], m[0].reshape(1, -1), m[1], 1.0, 1e-3)
        W0[b] = W[0]
    return dict(z=z, mean=mean, std=std, ts=np.asarray(ts, np.int32), w_prev=wp, mu=out_mu,
                sigma=out_S, valid=valid, W0=W0)


if __name__ == "__main__":
    cases = {
        "mv_N20_H1_g1_c1e-3": (1, 32, 20, 1, 1.0, 1e-3, False),
        "mv_N5_H3_g10_c1e-2": (2, 32, 5, 3, 10.0, 1e-2, False),
        "mv_N8_H2_g0.5_c0": (3, 32, 8, 2, 0.5, 0.0, False),
        "mv_short_N6_H2_g2_c1e-3": (4, 32, 6, 2, 2.0, 1e-3, True),
        "mv_N100_H1_g1_c1e-3": (5, 8, 100, 1, 1.0, 1e-3, False),
    }
    for name, args in cases.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **problems(*args))
        print("wrote", name)
    np.savez_compressed(os.path.join(HERE, "markowitz_N10.npz"),
                        **markowitz(7, 120, 10, [0, 3, 4, 5, 30, 59, 60, 61, 119]))
    print("wrote markowitz_N10")
