"""Backtest engine with the reference API (backtest.py:22-249), on the gfx950 window path.

``KoopmanMPCStrategy.rebalance`` keeps the reference signature and return contract
(backtest.py:80-131: a NEW float64 array W[0]; ``current_weights`` is never mutated) but runs the
whole window — encode, H x (z @ K, decode[:N], de-standardize), log-utility MPC solve — as one
fused device call (``kmpc_window``). ``rebalance_batch`` evaluates many independent windows in one
launch. ``run_backtest`` / ``calculate_metrics`` reproduce the reference bookkeeping exactly
(transaction cost, realized return, drift with the 1e-8 guard, the rebalance_freq quirk, population
std Sharpe, drawdown, total return relative to the first row).
"""
from __future__ import annotations

import ctypes
from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Any, Dict, Optional, Sequence

import numpy as np
import pandas as pd
import torch

from . import _lib
from .koopman import DeviceKoopman, KoopmanModelSpec
from .mpc import MPCConfig, _solve_desc, solve_mpc_log_utility_batched


@dataclass
class BacktestConfig:
    """Configuration for backtesting (backtest.py:22-30)."""
    initial_capital: float = 10000.0
    horizon: int = 5  # MPC prediction horizon
    rebalance_freq: int = 1  # Rebalance every N days
    cost_coeff: float = 0.001  # 10bps transaction cost
    risk_free_rate: float = 0.0  # Daily risk-free rate (unused, as in the reference)
    allow_short: bool = False  # unused, as in the reference


class Strategy(ABC):
    """Abstract base class for trading strategies (backtest.py:32-55)."""

    @abstractmethod
    def rebalance(self, t: int, current_weights: np.ndarray, env: Any, lookback_window: int = 60) -> np.ndarray:
        """Return new weights [n_assets] for test index t."""


class BuyAndHoldStrategy(Strategy):
    """Equal weight at t == 0, then hold (backtest.py:57-65)."""

    def rebalance(self, t, current_weights, env, lookback_window=60):
        if t == 0:
            n_assets = env.n_assets
            return np.ones(n_assets) / n_assets
        return current_weights


def _cache_key(data):
    """Key of a device copy of env data: the object itself (kept alive, so its identity cannot be
    reused by a new object) and, for tensors, the in-place version counter."""
    return (data, getattr(data, "_version", None))


def _cache_hit(key, data) -> bool:
    return key is not None and key[0] is data and key[1] == getattr(data, "_version", None)


def _env_stats(env) -> Optional[tuple]:
    stats = getattr(env, "stats", None)
    mean = getattr(stats, "mean", None)
    std = getattr(stats, "std", None)
    if mean is None or std is None:
        return None
    return np.asarray(mean, np.float64), np.asarray(std, np.float64)


class KoopmanMPCStrategy(Strategy):
    """Koopman-MPC strategy (backtest.py:67-131) on the device.

    Args:
        model: a reference KoopmanMachine (GenericKM / SparseKM / LISTAKM), a KoopmanModelSpec, a
            DeviceKoopman, or a train.py checkpoint dict ({'model_state_dict', 'config'}).
        mpc_config: MPCConfig (the reference's, or this package's).
        device: kept for signature compatibility. The hot path always runs on a HIP device; 'cpu'
            (the reference default) selects the current GPU.
    """

    def __init__(self, model: Any, mpc_config: MPCConfig, device: str = "cpu"):
        self.model = model
        self.mpc_config = mpc_config
        self.device = device
        self._dev = None
        self._km: Optional[DeviceKoopman] = None
        self._env_cache = (None, None)

    # -- device model -------------------------------------------------------------------------
    def _device(self) -> torch.device:
        if self._dev is None:
            if not torch.cuda.is_available():
                raise _lib.KmpcError("KoopmanMPCStrategy runs on the gfx950 kernels and needs a GPU")
            dev = torch.device(self.device) if str(self.device).startswith("cuda") else None
            self._dev = dev if dev is not None else torch.device("cuda", torch.cuda.current_device())
        return self._dev

    def device_model(self) -> DeviceKoopman:
        if self._km is None:
            m = self.model
            if isinstance(m, DeviceKoopman):
                self._km = m
            else:
                if isinstance(m, KoopmanModelSpec):
                    spec = m
                elif isinstance(m, dict) and "model_state_dict" in m:
                    spec = KoopmanModelSpec.from_checkpoint(m)
                else:
                    spec = KoopmanModelSpec.from_model(m)
                self._km = DeviceKoopman(spec, self._device())
        return self._km

    def _test_data(self, env) -> torch.Tensor:
        data = env.test_dataset.data
        if not _cache_hit(self._env_cache[0], data):
            self._env_cache = (_cache_key(data), torch.as_tensor(data).to(self._device(), torch.float32).contiguous())
        return self._env_cache[1]

    # -- windows --------------------------------------------------------------------------------
    def rebalance_batch(self, ts: Sequence[int], current_weights, env, return_info: bool = False):
        """Independent windows t in ts with their own current weights [B, N] -> W[0] [B, N] float64."""
        km = self.device_model()
        data = self._test_data(env)
        idx = torch.as_tensor(np.asarray(ts, np.int64), device=km.device)
        obs = data.index_select(0, idx)
        N = int(env.n_assets)
        wp = torch.as_tensor(np.asarray(current_weights, np.float64), device=km.device).reshape(len(ts), N)
        st = _env_stats(env)
        if st is not None:
            W0, status, value = km.window(obs, wp, st[0], st[1], N, self.mpc_config)
        else:
            # env with custom extract/destandardize callables: roll out in standardized space
            # (mean 0, std 1), apply the env's own destandardize_returns, then solve.
            y_std = km.rollout(obs, np.zeros(N), np.ones(N), int(self.mpc_config.horizon), N)
            yhat = torch.as_tensor(env.destandardize_returns(y_std), device=km.device, dtype=torch.float32)
            W0, status, value = solve_mpc_log_utility_batched(wp, yhat, self.mpc_config)
        W0 = W0.cpu().numpy()
        if return_info:
            return W0, status.cpu().numpy(), value.cpu().numpy()
        return W0

    def rebalance(self, t, current_weights, env, lookback_window=60):
        W0 = self.rebalance_batch([t], np.asarray(current_weights, np.float64).reshape(1, -1), env)
        return W0[0]


def run_backtest(strategy: Strategy, env: Any, config: BacktestConfig, verbose: bool = True) -> pd.DataFrame:
    """Sequential backtest loop with the reference semantics (backtest.py:133-219)."""
    n_steps = len(env.test_dataset) - config.horizon  # leave room for the horizon
    n_assets = env.n_assets
    portfolio_value = config.initial_capital
    history = []
    current_weights = np.ones(n_assets) / n_assets
    steps = range(0, n_steps, config.rebalance_freq)
    if verbose:
        from tqdm import tqdm
        steps = tqdm(steps, desc="Backtesting")
    data = env.test_dataset.data
    realized = env.destandardize_returns(env.extract_current_returns(data))
    all_returns = realized.cpu().numpy() if torch.is_tensor(realized) else np.asarray(realized)
    for t in steps:
        target_weights = strategy.rebalance(t, current_weights, env)
        turnover = np.sum(np.abs(target_weights - current_weights))
        cost = config.cost_coeff * turnover * portfolio_value
        current_weights = target_weights
        portfolio_value -= cost
        port_ret = 0.0
        if t + 1 < len(all_returns):
            realized_ret = np.exp(all_returns[t + 1]) - 1.0
            port_ret = np.sum(current_weights * realized_ret)
            portfolio_value *= (1.0 + port_ret)
            denom = 1.0 + port_ret
            if abs(denom) < 1e-8:
                denom = 1e-8
            current_weights = current_weights * (1.0 + realized_ret) / denom
        history.append({"date": env.test_dataset.dates[t], "portfolio_value": portfolio_value,
                        "return": port_ret, "turnover": turnover, "cost": cost})
    return pd.DataFrame(history)


def calculate_metrics(df: pd.DataFrame) -> Dict:
    """Sharpe, max drawdown, turnover, final value, total return (backtest.py:221-249)."""
    if len(df) == 0:
        return {}
    returns = df["return"].values
    mean_ret = np.mean(returns)
    std_ret = np.std(returns)
    sharpe = np.sqrt(252) * mean_ret / (std_ret + 1e-8)
    cum_returns = (1 + returns).cumprod()
    peak = np.maximum.accumulate(cum_returns)
    max_dd = np.min((cum_returns - peak) / peak)
    return {
        "Sharpe Ratio": sharpe,
        "Max Drawdown": max_dd,
        "Avg Turnover": df["turnover"].mean(),
        "Final Value": df["portfolio_value"].iloc[-1],
        "Total Return": (df["portfolio_value"].iloc[-1] / df["portfolio_value"].iloc[0]) - 1.0,
    }


METRIC_NAMES = ("Sharpe Ratio", "Max Drawdown", "Avg Turnover", "Final Value", "Total Return")


PREROLL_CHUNK = 65536   # windows per batched rollout of run_backtest_lockstep(prerollout=True)


# path groups on their own streams for latency-bound path counts (tools/lockstep_probe.py, C3
# model, ms per step, 1 / 2 / 3 groups): P = 64 1.144 / 1.111 / 1.084; P = 256 1.245 / 1.208 /
# 1.188; P = 1,024 2.393 / 1.923 / 1.904. Three: the process has four hardware queues
# (GPU_MAX_HW_QUEUES) and a fourth group's stream shared one of them with another group in the same
# measurement (2.10 ms at P = 64: two groups serialised)
LOCKSTEP_GROUPS = 3
LOCKSTEP_GROUPS_MAX_P = 1024


def run_backtest_lockstep(strategy: KoopmanMPCStrategy, obs, realized, config: BacktestConfig,
                          mean, std, n_rows: Optional[int] = None, graph: bool = False,
                          prerollout: bool = True, groups: Optional[int] = None,
                          persistent: Optional[bool] = None) -> Dict[str, Any]:
    """P independent backtests of the reference loop (backtest.py:133-219) run in lock step on the
    device: at every step one batched window launch (kmpc_window over the P
    paths) and one bookkeeping launch (kmpc_backtest_step); calculate_metrics per path at the end
    (kmpc_backtest_metrics). Path p reproduces run_backtest on an env whose test rows are obs[p] and
    whose de-standardized realized log-returns are realized[p].

    Args:
        obs: [P, T, obs] float32 standardized embeddings (env.test_dataset.data per path).
        realized: [P, T, N] float32 de-standardized log-returns (the reference's all_returns).
        mean, std: [N] de-standardisation of the rollout (env.stats).
        n_rows: len(env.test_dataset) (default T); n_steps = n_rows - config.horizon.
        graph: capture the whole step sequence in one HIP graph and replay it (no per-launch host
            overhead or inter-kernel gaps: the latency-bound small-P case); same launches, same
            results as the eager loop.
        prerollout: the forecasts depend on the observations only (not on the weights the steps
            carry), so every step's rollout runs up front as one batched kmpc_rollout over the
            S x P windows (PREROLL_CHUNK windows per launch) and each step launches only the solve
            (kmpc_solve); False: one fused kmpc_window per step. The rollout tiles differ with the
            batch size, so the two agree to fp32 summation order, not bit for bit.
        groups: the paths split into this many contiguous groups, each stepping on its own HIP
            stream (_lib.group_streams; default LOCKSTEP_GROUPS up to LOCKSTEP_GROUPS_MAX_P paths,
            with prerollout and without graph; else 1). A step's solve lasts as long as its slowest window, so
            independent groups wait only for their own slowest path: the small-P backtest runs at
            the groups' mean step time instead of the maximum over all paths. Every window is
            solved by the same kernel as in one group, so the results are bit-identical.
        persistent: run every step of a path in one launch (kmpc_backtest_run: one workgroup per
            path, the step's solve then its bookkeeping, back to back) — no lock step at all, so a
            path never waits for another path's window. Default: with prerollout, without graph or
            groups, wherever the C ABI has the kernel for the shape (the float64 constant-case
            kernels kmpc_solve would use for the per-step batch: the C3 shape, 32 < N <= 256 at
            H = 5 / 10, and the packed N <= 32 shapes at H = 2 / 5 / 10 — one path per lane group);
            bit-identical to the lock-step loop. Falls back to the loop where unsupported.
    Returns: dict of device tensors — portfolio_value / return / turnover / cost [P, S] (the
        reference DataFrame columns), weights [P, N] (after the last step), metrics {name: [P]}.
    """
    km = strategy.device_model()
    dev = km.device
    x = torch.as_tensor(obs).to(dev, torch.float32)
    r = torch.as_tensor(realized).to(dev, torch.float32).contiguous()
    if x.dim() != 3 or r.dim() != 3 or x.shape[:2] != r.shape[:2]:
        raise ValueError("obs must be [P, T, obs] and realized [P, T, N]")
    P, T, N = r.shape
    n_rows = T if n_rows is None else int(n_rows)
    steps = list(range(0, n_rows - config.horizon, config.rebalance_freq))
    S = len(steps)
    # per step the [P, obs] rows of test index t, contiguous ([T, P, obs]: one copy up front instead
    # of one gather per step), and the realized returns of t + 1
    xt = x.transpose(0, 1).contiguous()
    rt = r.transpose(0, 1).contiguous()
    m, sd = km._stats(mean, std, N)
    w = torch.full((P, N), 1.0 / N, dtype=torch.float64, device=dev)       # backtest.py:161
    value = torch.full((P,), float(config.initial_capital), dtype=torch.float64, device=dev)
    hist = torch.empty((P, max(S, 1), 4), dtype=torch.float64, device=dev)
    metrics = torch.empty((P, 5), dtype=torch.float64, device=dev)
    L = _lib.load()
    d = _lib.BacktestDesc(P, N, max(S, 1), float(config.cost_coeff))

    H = int(strategy.mpc_config.horizon)
    sc = max(1, PREROLL_CHUNK // P)          # steps per batched rollout
    steps_t = torch.as_tensor(steps, dtype=torch.long, device=dev)
    groups_arg = groups
    if groups is None:
        groups = LOCKSTEP_GROUPS if (prerollout and not graph and P <= LOCKSTEP_GROUPS_MAX_P) else 1
    groups = max(1, min(int(groups), P))
    if groups > 1 and (graph or not prerollout):
        raise ValueError("path groups need prerollout=True and graph=False")
    bounds = [(P * g) // groups for g in range(groups + 1)]
    explicit = persistent
    if persistent is None:
        persistent = prerollout and not graph and groups_arg is None
    if persistent and (graph or not prerollout):
        raise ValueError("persistent needs prerollout=True and graph=False")

    def run_persistent() -> bool:
        """Every step of every path in kmpc_backtest_run launches (one per rollout chunk of sc steps):
        False (nothing run) where the C ABI has no persistent kernel for this shape."""
        sdesc = _solve_desc(P, N, H, strategy.mpc_config, False)
        target = torch.empty((P, N), dtype=torch.float64, device=dev)
        status = torch.empty((P,), dtype=torch.int32, device=dev)
        objv = torch.empty((P,), dtype=torch.float64, device=dev)
        sh = _lib.stream_handle(dev)

        def call(k0, n, y, rr, n_real):
            return L.kmpc_backtest_run(ctypes.byref(d), ctypes.byref(sdesc), k0, n, y, rr, n_real, w.data_ptr(),
                                       value.data_ptr(), hist.data_ptr(), target.data_ptr(), status.data_ptr(),
                                       objv.data_ptr(), sh)

        rc = call(0, 0, None, None, 0)   # (shape check only)
        if rc == _lib.KMPC_ERR_UNSUPPORTED:
            if explicit:
                raise ValueError("persistent=True: no persistent backtest kernel for this shape")
            return False
        _lib.check(rc)
        for k0 in range(0, S, sc):
            n = min(sc, S - k0)
            y = km.rollout(xt[steps_t[k0:k0 + n]].reshape(n * P, -1), m, sd, H, N).contiguous()
            tn = steps_t[k0:k0 + n] + 1
            n_real = int((tn < T).sum().item())   # (steps increase: the rows with a t + 1 are a prefix)
            rr = rt[tn[:n_real]].contiguous() if n_real else None
            _lib.check(call(k0, n, y.data_ptr(), rr.data_ptr() if rr is not None else None, n_real))
        _lib.check(L.kmpc_backtest_metrics(ctypes.byref(d), hist.data_ptr(), metrics.data_ptr(), sh))
        return True

    def run_steps():
        y = None
        for k, t in enumerate(steps):
            if prerollout:
                if k % sc == 0:   # the forecasts of steps k .. k + sc - 1 in one launch
                    n = min(sc, S - k)
                    y = km.rollout(xt[steps_t[k:k + n]].reshape(n * P, -1), m, sd, H, N).reshape(n, P, H, N)
                W0, _, _ = solve_mpc_log_utility_batched(w, y[k % sc], strategy.mpc_config)
            else:
                W0, _, _ = km.window(xt[t], w, m, sd, N, strategy.mpc_config)
            rn = rt[t + 1] if t + 1 < T else None
            _lib.check(L.kmpc_backtest_step(ctypes.byref(d), k, W0.data_ptr(),
                                            rn.data_ptr() if rn is not None else None, w.data_ptr(),
                                            value.data_ptr(), hist.data_ptr(), _lib.stream_handle(dev)))
        if S:
            _lib.check(L.kmpc_backtest_metrics(ctypes.byref(d), hist.data_ptr(), metrics.data_ptr(),
                                               _lib.stream_handle(dev)))

    def run_groups():
        """The same per-step launches, path group g on stream g: group g's step k waits only for
        group g's step k - 1. The forecasts are rolled out on the calling stream, which every group
        stream waits for; the metrics launch waits for every group."""
        main = torch.cuda.current_stream(dev)
        streams = _lib.group_streams(groups, dev)   # (one hardware queue each; torch's pool may share)
        descs = [_lib.BacktestDesc(bounds[g + 1] - bounds[g], N, max(S, 1), float(config.cost_coeff))
                 for g in range(groups)]
        for st in streams:
            st.wait_stream(main)
        y = None
        for k, t in enumerate(steps):
            if k % sc == 0:
                n = min(sc, S - k)
                for st in streams:       # the previous chunk's readers before its memory is reused
                    main.wait_stream(st)
                y = km.rollout(xt[steps_t[k:k + n]].reshape(n * P, -1), m, sd, H, N).reshape(n, P, H, N)
                for st in streams:
                    st.wait_stream(main)
            rn = rt[t + 1] if t + 1 < T else None
            for g, st in enumerate(streams):
                g0, g1 = bounds[g], bounds[g + 1]
                with torch.cuda.stream(st):
                    W0, _, _ = solve_mpc_log_utility_batched(w[g0:g1], y[k % sc][g0:g1], strategy.mpc_config)
                    _lib.check(L.kmpc_backtest_step(
                        ctypes.byref(descs[g]), k, W0.data_ptr(), rn[g0:g1].data_ptr() if rn is not None else None,
                        w[g0:g1].data_ptr(), value[g0:g1].data_ptr(), hist[g0:g1].data_ptr(), _lib.stream_handle(dev)))
        for st in streams:
            main.wait_stream(st)
        if S:
            _lib.check(L.kmpc_backtest_metrics(ctypes.byref(d), hist.data_ptr(), metrics.data_ptr(),
                                               _lib.stream_handle(dev)))

    with torch.cuda.device(dev):
        if persistent and S and run_persistent():
            pass
        elif groups > 1 and S:
            run_groups()
        elif graph and S:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                run_steps()
            g.replay()
            torch.cuda.current_stream(dev).synchronize()   # (before the graph and its pool go)
        else:
            run_steps()
    hist = hist[:, :S]
    return {"portfolio_value": hist[..., 0], "return": hist[..., 1], "turnover": hist[..., 2],
            "cost": hist[..., 3], "weights": w,
            "metrics": {name: metrics[:, j] for j, name in enumerate(METRIC_NAMES)} if S else {}}
