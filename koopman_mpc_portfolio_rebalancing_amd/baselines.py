"""Baselines on the device: DMD and Markowitz.

Mirrors ``DMDStrategy`` of the reference (baselines.py:127-187): the operator A of x_{t+1} = A x_t
is fitted once on the host exactly as the reference does (``X' @ scipy.linalg.pinv(X)`` on the
float32 training embeddings, baselines.py:145-166 — a one-off fit, not on the path); the rollout
x <- A x over the horizon, the extraction of the first N entries, the de-standardisation and the
log-utility MPC solve run on the device. The rollout is the Koopman kernel chain with an identity
encoder / decoder and the latent operator A^T (row-vector convention, z <- z @ A^T), so DMD shares
``kmpc_window`` with the Koopman strategy.

Mirrors ``MarkowitzStrategy`` (baselines.py:24-106): the rolling 60-row mean / covariance of the
de-standardized current returns (kmpc_rolling_moments) and the H = 1 mean-variance solve
(kmpc_solve_mv, mpc.py:119-184) run on the device, for one window (``rebalance``) or many
(``rebalance_batch``).
"""
from __future__ import annotations

from typing import Any, Sequence

import numpy as np
import torch

from . import _lib
from .backtest import KoopmanMPCStrategy, Strategy, _cache_hit, _cache_key, _env_stats
from .koopman import KoopmanModelSpec
from .mpc import MPCConfig, solve_mpc_mean_variance_batched


def fit_dmd(train_data) -> np.ndarray:
    """A = X' pinv(X) with X = data[:-1]^T, X' = data[1:]^T (baselines.py:145-166), float32 in,
    computed by scipy.linalg.pinv as in the reference."""
    from scipy.linalg import pinv
    data = train_data.cpu().numpy() if torch.is_tensor(train_data) else np.asarray(train_data)
    X = data[:-1].T
    X_prime = data[1:].T
    return X_prime @ pinv(X)


def dmd_model_spec(A: np.ndarray) -> KoopmanModelSpec:
    """The DMD rollout as a Koopman model: identity encoder, latent operator A^T, identity decoder."""
    n = A.shape[0]
    eye = torch.eye(n, dtype=torch.float32)
    return KoopmanModelSpec(kind="generic", encoder=[(eye, None)], kmat=torch.as_tensor(A, dtype=torch.float32).t().contiguous(),
                            decoder=[(eye, None)], enc_act="relu", enc_last_relu=False, norm_fn="id")


class DMDStrategy(KoopmanMPCStrategy):
    """Dynamic Mode Decomposition strategy (baselines.py:127-187) on the device window path.

    Args:
        train_data: [samples, obs_size] training embeddings (env.train_dataset.data).
        mpc_config: MPCConfig for the log-utility solve.
        device: as KoopmanMPCStrategy ('cpu' selects the current GPU; there is no CPU path).
    """

    def __init__(self, train_data: Any, mpc_config: MPCConfig, device: str = "cpu"):
        self.K = fit_dmd(train_data)
        self.n_assets = None
        super().__init__(dmd_model_spec(self.K), mpc_config, device)


def rolling_moments(z: torch.Tensor, ts, lookback: int, n_assets: int, mean=None, std=None):
    """Markowitz moments on the device (baselines.py:70-88) for the windows t in ``ts``.

    Args:
        z: [T, >= N] float32 device tensor of standardized test rows (the first N columns are the
            current returns, data_finance.py:717-729).
        ts: test indices; window t uses rows max(0, t + 1 - lookback) .. t.
        mean, std: [N] de-standardization (data_finance.py:740-742); None -> identity.

    Returns:
        mu [B, N] float64 (float32-rounded mean), sigma [B, N, N] float64 (np.cov + 1e-6 I),
        valid [B] int32 (t + 1 >= 5).
    """
    _lib.require_gpu(z)
    dev = z.device
    N = int(n_assets)
    z = z.to(torch.float32)
    if z.dim() != 2 or z.shape[1] < N or z.stride(1) != 1:
        z = z.reshape(z.shape[0], -1).contiguous()
    T = int(z.shape[0])
    m = torch.zeros(N, dtype=torch.float32, device=dev) if mean is None else \
        torch.as_tensor(np.asarray(mean, np.float64).astype(np.float32), device=dev)
    sd = torch.ones(N, dtype=torch.float32, device=dev) if std is None else \
        torch.as_tensor(np.asarray(std, np.float64).astype(np.float32), device=dev)
    tt = torch.as_tensor(np.asarray(ts, np.int64).astype(np.int32), device=dev)
    B = int(tt.numel())
    mu = torch.empty((B, N), dtype=torch.float64, device=dev)
    sigma = torch.empty((B, N, N), dtype=torch.float64, device=dev)
    valid = torch.empty(B, dtype=torch.int32, device=dev)
    L = _lib.load()
    with torch.cuda.device(dev):
        rc = L.kmpc_rolling_moments(B, T, N, int(lookback), z.data_ptr(), int(z.stride(0)), m.data_ptr(),
                                    sd.data_ptr(), tt.data_ptr(), mu.data_ptr(), sigma.data_ptr(),
                                    valid.data_ptr(), _lib.stream_handle(dev))
    _lib.check(rc)
    return mu, sigma, valid


class MarkowitzStrategy(Strategy):
    """Classic mean-variance strategy (baselines.py:24-106) on the device.

    Same constructor and ``mpc_config`` (H = 1, gamma = risk_aversion, baselines.py:39-45);
    ``rebalance`` follows baselines.py:48-106 (hold when fewer than 5 past rows, rolling moments
    of the last ``lookback_window`` rows, W[0] of the mean-variance solve).
    """

    def __init__(self, risk_aversion: float = 1.0, cost_coeff: float = 0.001, allow_short: bool = False):
        self.risk_aversion = risk_aversion
        self.cost_coeff = cost_coeff
        self.allow_short = allow_short
        self.mpc_config = MPCConfig(horizon=1, gamma=risk_aversion, cost_coeff=cost_coeff,
                                    allow_short=allow_short, solver="ECOS")
        self._dev = None
        self._cache = (None, None)

    def _device(self) -> torch.device:
        if self._dev is None:
            if not torch.cuda.is_available():
                raise _lib.KmpcError("MarkowitzStrategy runs on the gfx950 kernels and needs a GPU")
            self._dev = torch.device("cuda", torch.cuda.current_device())
        return self._dev

    def _returns(self, env):
        """(rows [T, >= N] float32 on the device, mean, std, N): the env's test rows with its stats,
        or — for envs with custom extract / destandardize callables — the de-standardized
        current returns computed by those callables (baselines.py:71-73)."""
        data = env.test_dataset.data
        if not _cache_hit(self._cache[0], data):
            dev = self._device()
            st = _env_stats(env)
            n = getattr(env, "n_assets", None)
            if st is not None and n is not None:
                entry = (torch.as_tensor(data).to(dev, torch.float32).contiguous(), st[0], st[1], int(n))
            else:
                r = env.destandardize_returns(env.extract_current_returns(torch.as_tensor(data)))
                r = torch.as_tensor(r).to(dev, torch.float32).contiguous()
                entry = (r, None, None, int(r.shape[-1]))
            self._cache = (_cache_key(data), entry)
        return self._cache[1]

    def rebalance_batch(self, ts: Sequence[int], current_weights, env, lookback_window: int = 60,
                        return_info: bool = False):
        """Independent windows t in ts with their own current weights [B, N] -> W[0] [B, N] float64."""
        self._device()   # no GPU -> KmpcError (there is no CPU path)
        z, mean, std, N = self._returns(env)
        dev = z.device
        wp = torch.as_tensor(np.asarray(current_weights, np.float64), device=dev).reshape(len(ts), N)
        mu, sigma, valid = rolling_moments(z, ts, lookback_window, N, mean, std)
        W0, status, value = solve_mpc_mean_variance_batched(wp, mu.unsqueeze(1), sigma, self.mpc_config)
        hold = valid == 0   # fewer than 5 past rows: keep the current weights (baselines.py:76-78)
        W0 = torch.where(hold.unsqueeze(1), wp, W0)
        W0 = W0.cpu().numpy()
        if return_info:
            return W0, status.cpu().numpy(), value.cpu().numpy(), valid.cpu().numpy()
        return W0

    def rebalance(self, t, current_weights, env, lookback_window: int = 60) -> np.ndarray:
        W0 = self.rebalance_batch([t], np.asarray(current_weights, np.float64).reshape(1, -1), env,
                                  lookback_window)
        return W0[0]


__all__: Sequence[str] = ("DMDStrategy", "MarkowitzStrategy", "fit_dmd", "dmd_model_spec",
                          "rolling_moments", "Strategy")
