"""Mean-variance oracle (oracle/mv_ref.py, the checker of kmpc_solve_mv) pinned without a GPU:
scipy SLSQP agreement, closed forms, the reference's tests/test_baselines.py cases restated, and the
committed golden fixtures (tests/golden/make_mv_golden.py)."""
import glob
import os

import numpy as np
import pytest

from oracle import mv_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("seed", range(6))
def test_dense_ipm_matches_slsqp(seed):
    rng = np.random.default_rng(100 + seed)
    N, H = int(rng.integers(2, 6)), int(rng.integers(1, 4))
    gamma, cost, short = [(1.0, 1e-3, False), (10.0, 1e-2, False), (0.5, 0.0, False),
                          (2.0, 1e-3, True), (0.0, 1e-3, False), (5.0, 0.0, True)][seed]
    X = rng.normal(5e-4, 0.015, (60, N))
    S = np.cov(X, rowvar=False) + 1e-6 * np.eye(N)
    mu = rng.normal(5e-4, 0.01, (H, N))
    wp = rng.dirichlet(np.ones(N))
    W, st = mv_ref.mv_dense_ipm(wp, mu, S, gamma, cost, short)
    W2, ok = mv_ref.mv_slsqp(wp, mu, S, gamma, cost, short)
    assert st == "optimal" and ok
    f1 = mv_ref.mv_objective(W, wp, mu, S, gamma, cost)
    f2 = mv_ref.mv_objective(W2, wp, mu, S, gamma, cost)
    assert f1 >= f2 - 1e-10 * max(1.0, abs(f2))        # the oracle is never worse than SLSQP
    assert np.allclose(W.sum(1), 1.0, atol=1e-10)
    if not short:
        assert W.min() > -1e-10


def test_water_filling_closed_form():
    """Sigma = s2 I, c = 0, no short, H = 1: w_i = max((mu_i - lam) / (2 gamma s2), 0)."""
    mu = np.array([[0.03, 0.02, 0.01, -0.01]])
    s2, gamma = 1e-2, 1.0
    W, st = mv_ref.mv_dense_ipm(np.full(4, 0.25), mu, s2 * np.eye(4), gamma, 0.0)
    # active set {0, 1}: sum (mu_i - lam) / (2 gamma s2) = 1 -> lam = (0.05 - 0.02) / 2 = 0.015
    # (asset 2 would need mu_2 > lam)
    lam = (mu[0, :2].sum() - 2 * gamma * s2) / 2
    expect = np.maximum((mu[0] - lam) / (2 * gamma * s2), 0.0)
    assert np.allclose(expect, [0.75, 0.25, 0.0, 0.0])
    assert st == "optimal"
    assert np.allclose(W[0], expect, atol=1e-9)


def test_reference_markowitz_cases():
    """tests/test_baselines.py:29-61 of the reference: fewer than 5 rows -> hold; asset 0 with
    constant return 0.1 (Sigma = 1e-6 I after the regularisation) -> all weight on asset 0."""
    R = np.zeros((11, 2), np.float32)
    R[:, 0] = 0.1
    assert mv_ref.rolling_moments(R[:3]) is None
    mu, S = mv_ref.rolling_moments(R)
    assert np.allclose(S, 1e-6 * np.eye(2))
    W, info = mv_ref.solve_mpc_mean_variance_ref(np.array([0.5, 0.5]), mu.reshape(1, -1), S, 1.0, 1e-3)
    assert info["status"] == "optimal"
    assert np.allclose(W[0], [1.0, 0.0], atol=1e-9)


def test_rolling_moments_restate_numpy():
    rng = np.random.default_rng(0)
    R = rng.normal(0, 0.01, (100, 4)).astype(np.float32)
    mu, S = mv_ref.rolling_moments(R[:71])
    win = R[71 - 60:71]
    assert mu.dtype == np.float32 and np.array_equal(mu, np.mean(win, axis=0))
    assert np.allclose(S, np.cov(win.astype(np.float64), rowvar=False) + 1e-6 * np.eye(4), rtol=0, atol=1e-18)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "mv_*.npz"))))
def test_goldens_are_optimal_and_feasible(path):
    d = np.load(path)
    assert (d["status"] == 0).all()
    W = d["W"]
    assert np.abs(W.sum(-1) - 1).max() < 1e-9
    if not int(d["allow_short"]):
        assert W.min() > -1e-9
    for b in range(min(4, len(W))):   # the stored objective is problem.value at W
        f = mv_ref.mv_objective(W[b], d["w_prev"][b], d["mu"][b], d["sigma"][b], float(d["gamma"]), float(d["cost"]))
        assert abs(f - d["obj"][b]) < 1e-14
