"""Backtest bookkeeping (package backtest.py and the oracle restatement) against the reference's
own run_backtest / calculate_metrics outputs. CPU only (no solver needed: recorded solver outputs
or buy-and-hold)."""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from koopman_mpc_portfolio_rebalancing_amd import (BacktestConfig, BuyAndHoldStrategy, Strategy,
                                                   calculate_metrics, run_backtest)
from oracle import backtest_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


class GoldenEnv:
    """Just the FinanceEnv surface run_backtest touches (data_finance.py:361-419, 700-742)."""

    class _DS:
        def __init__(self, data, dates, n):
            self.data = torch.from_numpy(data)
            self.dates = pd.to_datetime(dates)
            self._n = int(n)

        def __len__(self):
            return self._n

    class _Stats:
        def __init__(self, mean, std):
            self.mean, self.std = mean, std

    def __init__(self, g):
        self.test_dataset = self._DS(g["test_data"], g["dates"], g["test_len"])
        self.stats = self._Stats(g["mean"], g["std"])
        self.n_assets = int(g["mean"].shape[0])

    def extract_current_returns(self, x):
        return x[..., :self.n_assets]

    def destandardize_returns(self, x):
        mean = torch.from_numpy(self.stats.mean).float()
        std = torch.from_numpy(self.stats.std).float()
        return x * std + mean


class ReplayStrategy(Strategy):
    """Replays the W[0] the reference strategy applied at each call."""

    def __init__(self, W):
        self.W = W
        self.k = 0

    def rebalance(self, t, current_weights, env, lookback_window=60):
        w = self.W[self.k][0].copy()
        self.k += 1
        return w


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLD, "backtest_koopman_mpc.npz"))


def test_run_backtest_replay_matches_reference(golden):
    meta = json.loads(str(golden["meta"]))
    env = GoldenEnv(golden)
    cfg = BacktestConfig(**meta["backtest"])
    df = run_backtest(ReplayStrategy(golden["call_W"]), env, cfg, verbose=False)
    assert list(df.columns) == ["date", "portfolio_value", "return", "turnover", "cost"]
    assert len(df) == len(golden["df_value"]) == int(golden["test_len"]) - meta["H"]
    np.testing.assert_allclose(df["portfolio_value"].values, golden["df_value"], rtol=1e-12)
    np.testing.assert_allclose(df["return"].values, golden["df_return"], rtol=1e-10, atol=1e-15)
    np.testing.assert_allclose(df["turnover"].values, golden["df_turnover"], rtol=1e-10, atol=1e-15)
    np.testing.assert_allclose(df["cost"].values, golden["df_cost"], rtol=1e-10, atol=1e-15)
    assert [str(d.date()) for d in df["date"]] == list(golden["df_date"])
    m = calculate_metrics(df)
    for k, v in meta["metrics"].items():
        assert m[k] == pytest.approx(v, rel=1e-10, abs=1e-14)


def test_oracle_backtest_restatement_matches_reference(golden):
    meta = json.loads(str(golden["meta"]))
    N = meta["N"]
    realized = golden["test_data"][:, :N].astype(np.float32) * golden["std"].astype(np.float32) + \
        golden["mean"].astype(np.float32)
    W = golden["call_W"]
    k = {"i": 0}

    def reb(t, w):
        out = W[k["i"]][0]
        k["i"] += 1
        return out

    hist = backtest_ref.run_backtest(reb, realized, int(golden["test_len"]), meta["H"], N, 10000.0, 1, 1e-3)
    np.testing.assert_allclose([h["portfolio_value"] for h in hist], golden["df_value"], rtol=1e-12)


def test_buy_and_hold_matches_reference(golden):
    meta = json.loads(str(golden["meta"]))
    env = GoldenEnv(golden)
    df = run_backtest(BuyAndHoldStrategy(), env, BacktestConfig(**meta["backtest"]), verbose=False)
    np.testing.assert_allclose(df["portfolio_value"].values, golden["bh_value"], rtol=1e-12)
    np.testing.assert_allclose(df["turnover"].values, golden["bh_turnover"], rtol=1e-12, atol=1e-15)
    m = calculate_metrics(df)
    for k, v in meta["metrics_bh"].items():
        assert m[k] == pytest.approx(v, rel=1e-10, abs=1e-14)


def test_reference_mock_env_mechanics():
    """The reference's tests/test_backtest.py:15-38 (MockFinanceEnv, horizon=2 -> 8 rows)."""
    g = np.load(os.path.join(GOLD, "backtest_mock.npz"))

    class MockEnv:
        n_assets = 2

        def __init__(self):
            class DS:
                pass
            self.test_dataset = DS()
            self.test_dataset.dates = pd.date_range("2021-01-01", periods=10)
            self.test_dataset.data = torch.from_numpy(g["data"])
            self.test_dataset.__len__ = lambda: 10
            self.extract_current_returns = lambda x: x[..., :2]
            self.destandardize_returns = lambda x: x * 0.01

    env = MockEnv()
    type(env.test_dataset).__len__ = lambda self: 10
    df = run_backtest(BuyAndHoldStrategy(), env, BacktestConfig(horizon=2, initial_capital=1000.0), verbose=False)
    assert len(df) == 8
    assert df["portfolio_value"].iloc[-1] != 1000.0
    np.testing.assert_allclose(df["portfolio_value"].values, g["df_value"], rtol=1e-12)
    np.testing.assert_allclose(df["return"].values, g["df_return"], rtol=1e-10, atol=1e-15)


def test_calculate_metrics_reference_case():
    """The reference's tests/test_backtest.py:40-52 frame, compared to the reference's values."""
    g = np.load(os.path.join(GOLD, "backtest_mock.npz"))
    ref = json.loads(str(g["metrics"]))
    df = pd.DataFrame({"return": [0.01, -0.01, 0.02, 0.0], "turnover": [0.1, 0.0, 0.0, 0.0],
                       "portfolio_value": [1010, 999.9, 1019.9, 1019.9]})
    m = calculate_metrics(df)
    assert m["Max Drawdown"] < 0
    for k, v in ref.items():
        assert m[k] == pytest.approx(v, rel=1e-12)
    assert calculate_metrics(pd.DataFrame({"return": [], "turnover": [], "portfolio_value": []})) == {}


def test_rebalance_freq_quirk(golden):
    """rebalance_freq=2 skips intermediate days' returns exactly like backtest.py:173."""
    meta = json.loads(str(golden["meta"]))
    env = GoldenEnv(golden)
    cfg = BacktestConfig(initial_capital=10000.0, horizon=meta["H"], rebalance_freq=2, cost_coeff=1e-3)
    df = run_backtest(BuyAndHoldStrategy(), env, cfg, verbose=False)
    assert len(df) == len(range(0, int(golden["test_len"]) - meta["H"], 2))
