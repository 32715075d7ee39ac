"""Mean-variance MPC (kmpc_solve_mv) and Markowitz (kmpc_rolling_moments) on the device, through
the C ABI, against the float64 oracle (oracle/mv_ref.py) and its golden fixtures.

Tolerances (float64 device arithmetic, interior point stopped at 1e-10 complementarity):
objective within 1e-9 + 1e-7 |f*|; W within 1e-5 (the program is strictly convex in w when
gamma > 0, so the optimum is unique); feasibility sum(w) = 1 +- 1e-9, w >= -1e-9 (no short).
"""
import glob
import os
from unittest.mock import MagicMock

import numpy as np
import pytest
import torch

from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_mean_variance, solve_mpc_mean_variance_batched
from koopman_mpc_portfolio_rebalancing_amd import _lib
from koopman_mpc_portfolio_rebalancing_amd.baselines import MarkowitzStrategy, rolling_moments
from oracle import mv_ref

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = torch.device("cuda", 0)


def _solve(d, full=True):
    cfg = MPCConfig(horizon=d["mu"].shape[1], gamma=float(d["gamma"]), cost_coeff=float(d["cost"]),
                    allow_short=bool(int(d["allow_short"])))
    W, st, val = solve_mpc_mean_variance_batched(torch.tensor(d["w_prev"], device=DEV), torch.tensor(d["mu"], device=DEV),
                                                 torch.tensor(d["sigma"], device=DEV), cfg, return_full=full)
    torch.cuda.synchronize()
    return W.cpu().numpy(), st.cpu().numpy(), val.cpu().numpy()


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "mv_*.npz"))))
def test_mv_matches_golden(path):
    d = np.load(path)
    W, st, val = _solve(d)
    assert (st == 0).all(), st
    assert np.abs(val - d["obj"]).max() <= 1e-9 + 1e-7 * np.abs(d["obj"]).max()
    assert np.abs(W - d["W"]).max() < 1e-5
    assert np.abs(W.sum(-1) - 1).max() < 1e-9
    if not int(d["allow_short"]):
        assert W.min() > -1e-9
    W0, st0, _ = _solve(d, full=False)              # W[0] output layout
    assert np.array_equal(W0, W[:, 0])


def test_shared_sigma_and_drop_in_api():
    d = np.load(os.path.join(GOLD, "mv_N20_H1_g1_c1e-3.npz"))
    S = d["sigma"][0]
    cfg = MPCConfig(horizon=1, gamma=1.0, cost_coeff=1e-3)
    W, info = solve_mpc_mean_variance(d["w_prev"][3], d["mu"][3], S, cfg)
    Wo, so = mv_ref.mv_dense_ipm(d["w_prev"][3], d["mu"][3], S, 1.0, 1e-3)
    assert info["status"] == "optimal" and W.shape == (1, 20) and W.dtype == np.float64
    assert np.abs(W - Wo).max() < 1e-5
    assert abs(info["value"] - mv_ref.mv_objective(Wo, d["w_prev"][3], d["mu"][3], S, 1.0, 1e-3)) < 1e-9
    # one [N, N] Sigma shared by the batch (sigma_stride 0)
    B = 8
    Wb, st, _ = solve_mpc_mean_variance_batched(torch.tensor(d["w_prev"][:B], device=DEV),
                                                torch.tensor(d["mu"][:B], device=DEV), torch.tensor(S, device=DEV), cfg)
    for b in range(B):
        Wo, _ = mv_ref.mv_dense_ipm(d["w_prev"][b], d["mu"][b], S, 1.0, 1e-3)
        assert np.abs(Wb[b].cpu().numpy() - Wo[0]).max() < 1e-5


@pytest.mark.parametrize("N,H,short", [(150, 1, False), (60, 3, False), (300, 2, False), (129, 1, True)])
def test_mv_workspace_path_matches_oracle(N, H, short):
    """H*N > 128: the Newton matrix no longer fits LDS and lives in a workspace slab (kmpc_mv.hip's
    global-M kernel, persistent grid); same program, same tolerances as the golden cases."""
    rng = np.random.default_rng(N * 10 + H)
    B = 6
    F = rng.standard_normal((B, N, 4)) * 0.02
    sigma = F @ F.transpose(0, 2, 1) + np.eye(N) * 1e-3
    mu = rng.standard_normal((B, H, N)) * 1e-2
    wp = rng.dirichlet(np.ones(N), size=B)
    cfg = MPCConfig(horizon=H, gamma=1.0, cost_coeff=1e-3, allow_short=short)
    W, st, val = solve_mpc_mean_variance_batched(torch.tensor(wp, device=DEV), torch.tensor(mu, device=DEV),
                                                 torch.tensor(sigma, device=DEV), cfg, return_full=True)
    torch.cuda.synchronize()
    W, st, val = W.cpu().numpy(), st.cpu().numpy(), val.cpu().numpy()
    assert (st == 0).all(), st
    for b in range(B):
        Wo, so = mv_ref.mv_dense_ipm(wp[b], mu[b], sigma[b], 1.0, 1e-3, allow_short=short)
        assert so == "optimal"
        fo = mv_ref.mv_objective(Wo, wp[b], mu[b], sigma[b], 1.0, 1e-3)
        assert abs(val[b] - fo) <= 1e-9 + 1e-7 * abs(fo)
        # the utility is gamma * lambda_min(Sigma)-strongly concave in W: a feasible W within df of
        # the optimum lies within sqrt(2 df / m) of W* (flat directions make 1e-5 too strict)
        m = np.linalg.eigvalsh(sigma[b])[0]
        df = abs(fo - mv_ref.mv_objective(W[b], wp[b], mu[b], sigma[b], 1.0, 1e-3)) + 1e-13
        assert np.abs(W[b] - Wo).max() < max(1e-5, 2 * np.sqrt(2 * df / m))
    assert np.abs(W.sum(-1) - 1).max() < 1e-9
    if not short:
        assert W.min() > -1e-9


def test_fallbacks():
    """Non-finite input -> solver_error + tile(w_prev) and no "value" (mpc.py:180-181);
    allow_short with gamma = 0, c = 0 and a return spread is an unbounded LP."""
    wp = np.array([0.3, 0.7])
    W, info = solve_mpc_mean_variance(wp, np.array([[np.nan, 0.0]]), np.eye(2), MPCConfig(horizon=1, gamma=1.0))
    assert info == {"status": "solver_error"} and np.array_equal(W, np.tile(wp, (1, 1)))
    W, info = solve_mpc_mean_variance(wp, np.array([[0.01, 0.0]]), np.eye(2) * 1e-4,
                                      MPCConfig(horizon=1, gamma=0.0, cost_coeff=0.0, allow_short=True))
    assert info["status"] == "unbounded" and np.array_equal(W, np.tile(wp, (1, 1)))
    with pytest.raises(_lib.KmpcError):
        solve_mpc_mean_variance(np.full(1025, 1 / 1025), np.zeros((1, 1025)), np.eye(1025), MPCConfig(horizon=1))


def test_rolling_moments_match_oracle():
    d = np.load(os.path.join(GOLD, "markowitz_N10.npz"))
    z = torch.tensor(d["z"], device=DEV)
    mu, S, valid = rolling_moments(z, d["ts"], 60, 10, d["mean"], d["std"])
    torch.cuda.synchronize()
    assert np.array_equal(valid.cpu().numpy(), d["valid"])
    v = d["valid"] == 1
    # mu: float32-rounded mean (the reference's float32 np.mean), within 2 float32 ulps of it
    assert np.abs(mu.cpu().numpy()[v] - d["mu"][v]).max() <= 2 * np.spacing(np.float32(np.abs(d["mu"]).max()))
    assert np.abs(S.cpu().numpy()[v] - d["sigma"][v]).max() < 1e-15


def test_markowitz_batch_matches_oracle():
    """Lock-free batch of Markowitz windows (baselines.py:48-106) against the per-window oracle."""
    d = np.load(os.path.join(GOLD, "markowitz_N10.npz"))
    env = MagicMock()
    env.n_assets = 10
    env.test_dataset.data = torch.tensor(d["z"])
    env.stats.mean, env.stats.std = d["mean"].astype(np.float64), d["std"].astype(np.float64)
    strat = MarkowitzStrategy(risk_aversion=1.0, cost_coeff=1e-3)
    W0 = strat.rebalance_batch(list(d["ts"]), d["w_prev"], env)
    assert np.abs(W0 - d["W0"]).max() < 1e-5
    hold = d["valid"] == 0
    assert np.array_equal(W0[hold], d["w_prev"][hold])


class _MockEnv:
    """tests/test_baselines.py:7-20 of the reference: MagicMock dataset, custom callables."""

    def __init__(self, data):
        self.n_assets = 2
        self.test_dataset = MagicMock()
        self.test_dataset.data = data
        self.extract_current_returns = lambda x: x[..., :2]
        self.destandardize_returns = lambda x: x


def test_reference_test_baselines_cases():
    env = _MockEnv(torch.randn(20, 5))
    strat = MarkowitzStrategy()
    w = strat.rebalance(t=2, current_weights=np.array([0.5, 0.5]), env=env)   # < 5 rows: hold
    assert np.allclose(w, [0.5, 0.5])
    data = torch.zeros(20, 5)
    data[:, 0] = 0.1
    env = _MockEnv(data)
    w = MarkowitzStrategy(risk_aversion=1.0).rebalance(t=10, current_weights=np.array([0.5, 0.5]), env=env)
    assert w[0] > 0.5 and w[1] < 0.5 and np.isclose(w.sum(), 1.0)
    assert np.allclose(w, [1.0, 0.0], atol=1e-6)      # the exact optimum (tests/test_mv_cpu.py)
