"""MPC solve — the reference's ``mpc.py`` API on the gfx950 solver kernel.

Mirrors ``MPCConfig`` (mpc.py:17-25) field for field and ``solve_mpc_log_utility``
(mpc.py:27-117) signature, return shapes/dtypes and failure semantics: solver failure is never
raised; a status outside {"optimal", "optimal_inaccurate"} returns ``tile(current_weights)`` and
``{"status": s, "value": None}`` (mpc.py:113-115).

``solve_mpc_log_utility_batched`` is the batched entry point (torch device tensors in and out)
that the strategies and the benchmark use. ``solve_mpc_mean_variance`` (mpc.py:119-184) and its
batched form run the mean-variance QP kernel (kmpc_solve_mv) with the same conventions.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Tuple

import numpy as np
import torch

from . import _lib


@dataclass
class MPCConfig:
    """Configuration for MPC solver (mpc.py:17-25)."""
    horizon: int = 5
    gamma: float = 0.0  # Risk aversion (0.0 = log utility maximization); unused by log utility
    cost_coeff: float = 0.001  # Transaction cost coefficient (e.g. 10bps)
    max_turnover: float = 0.2  # Maximum turnover per step
    allow_short: bool = False
    solver: str = "ECOS"  # accepted for compatibility; the gfx950 interior-point kernel solves
    # extra (defaulted) knobs of the device solver
    max_iter: int = 80
    tol: float = 1e-9
    n_refine: int = 0  # 0 -> kernel default
    solver_path: int = 0  # kmpc_solve_desc.path: 0 by shape, 1 register IPM (no presolve), 2 large-window IPM, 3 register IPM without lane-group packing
    precision: str = "auto"  # kmpc_solve_desc.precision: "mixed" (float32 warm-start phase + float64 finish where available), "f64", or "auto" (mixed from 2,048 windows per call, else f64)
    mu_handoff: float = 0.0  # float32 -> float64 handoff at mu <= mu_handoff (0 -> kernel default 3e-5)


def _solve_desc(B: int, N: int, H: int, config: MPCConfig, full: bool) -> _lib.SolveDesc:
    d = _lib.SolveDesc()
    d.B, d.N, d.H = int(B), int(N), int(H)
    d.cost_coeff = float(config.cost_coeff)
    d.max_turnover = float(config.max_turnover)
    d.allow_short = int(bool(config.allow_short))
    d.max_iter = int(getattr(config, "max_iter", 80))
    d.tol = float(getattr(config, "tol", 1e-9))
    d.return_full_W = int(bool(full))
    d.n_refine = int(getattr(config, "n_refine", 0))
    d.path = int(getattr(config, "solver_path", 0))
    prec = getattr(config, "precision", "auto")
    if prec not in ("auto", "f64", "mixed"):
        raise ValueError(f"precision must be 'auto', 'f64' or 'mixed' (got {prec!r})")
    d.precision = {"auto": _lib.PRECISION_AUTO, "f64": _lib.PRECISION_F64, "mixed": _lib.PRECISION_MIXED}[prec]
    d.mu_handoff = float(getattr(config, "mu_handoff", 0.0))
    if d.cost_coeff < 0:
        # -c ||dw||_1 with c < 0 is not concave: the reference's cvxpy problem fails DCP and raises
        raise ValueError(f"cost_coeff must be >= 0 (got {config.cost_coeff}): the problem is not convex")
    return d


def _workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """A device buffer of at least nbytes for one call, from torch's caching allocator on the
    current stream: the block returns to the pool when the caller drops it and is handed out again
    only in stream order, so concurrent streams never share scratch and nothing is held between calls."""
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def solve_mpc_log_utility_batched(
    current_weights: torch.Tensor,
    predicted_log_returns: torch.Tensor,
    config: MPCConfig,
    return_full: bool = False,
    with_iters: bool = False,
):
    """Batched solve on the device.

    Args:
        current_weights: [B, N] (float64; other dtypes are converted) device tensor.
        predicted_log_returns: [B, H, N] float32 device tensor (the reference feeds float32 yhat).
        config: MPCConfig.
        return_full: return W [B, H, N] instead of W[:, 0] [B, N].

    Returns:
        (W, status, value[, iters]): W float64, status int32 [B] (see _lib.STATUS_NAMES),
        value float64 [B] (NaN where the fallback was applied).
    """
    y = predicted_log_returns
    _lib.require_gpu(y)
    if y.dim() != 3:
        raise ValueError("predicted_log_returns must be [B, H, N]")
    B, H, N = y.shape
    y = y.to(torch.float32).contiguous()
    wp = current_weights.to(device=y.device, dtype=torch.float64).contiguous()
    if wp.shape != (B, N):
        raise ValueError(f"current_weights must be [{B}, {N}], got {tuple(wp.shape)}")
    if H > _lib.KMPC_MAX_H or N > _lib.KMPC_MAX_N:
        raise _lib.KmpcError(f"shape H={H}, N={N} exceeds the kernel limits "
                             f"(H <= {_lib.KMPC_MAX_H}, N <= {_lib.KMPC_MAX_N})")
    W = torch.empty((B, H, N) if return_full else (B, N), dtype=torch.float64, device=y.device)
    status = torch.empty(B, dtype=torch.int32, device=y.device)
    value = torch.empty(B, dtype=torch.float64, device=y.device)
    iters = torch.empty(B, dtype=torch.int32, device=y.device)
    d = _solve_desc(B, N, H, config, return_full)
    L = _lib.load()
    with torch.cuda.device(y.device):
        nws = int(L.kmpc_workspace_bytes(None, ctypes.byref(d)))
        ws = _workspace(y.device, nws) if nws else None
        rc = L.kmpc_solve(ctypes.byref(d), y.data_ptr(), wp.data_ptr(), W.data_ptr(),
                          status.data_ptr(), value.data_ptr(), iters.data_ptr(),
                          ws.data_ptr() if ws is not None else None, nws, _lib.stream_handle(y.device))
    _lib.check(rc)
    if with_iters:
        return W, status, value, iters
    return W, status, value


def gross_returns(predicted_log_returns: torch.Tensor) -> torch.Tensor:
    """R = np.exp(yhat) on the float32 yhat (mpc.py:55), bit for bit as numpy evaluates it
    (kmpc_gross_returns), as a float32 device tensor of the same shape."""
    y = predicted_log_returns
    _lib.require_gpu(y)
    y = y.to(torch.float32).contiguous()
    R = torch.empty_like(y)
    L = _lib.load()
    with torch.cuda.device(y.device):
        rc = L.kmpc_gross_returns(y.numel(), y.data_ptr(), R.data_ptr(), _lib.stream_handle(y.device))
    _lib.check(rc)
    return R


def log_utility_value_batched(W: torch.Tensor, current_weights: torch.Tensor,
                              predicted_log_returns: torch.Tensor, cost_coeff: float) -> torch.Tensor:
    """problem.value of the reference program (mpc.py:66-103) at given weights: for each window,
    sum_t log(R_t . w_t) - c sum_t ||w_t - w_{t-1}||_1 (w_{-1} = current_weights), R = np.exp(yhat)
    in float32, sums in float64. W [B, H, N], current_weights [B, N], yhat [B, H, N] -> [B] float64.
    Evaluates any W (e.g. a decision taken on another forecast) in the program of `yhat`."""
    R = gross_returns(predicted_log_returns).double()
    W = W.to(torch.float64)
    wp = current_weights.to(device=W.device, dtype=torch.float64)
    D = torch.diff(torch.cat([wp[:, None, :], W], 1), dim=1)
    return torch.log((R * W).sum(-1)).sum(-1) - cost_coeff * D.abs().sum((-1, -2))


def _default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise _lib.KmpcError("solve_mpc_log_utility runs on the gfx950 kernel and needs a GPU")
    return torch.device("cuda", torch.cuda.current_device())


def solve_mpc_log_utility(
    current_weights: np.ndarray,
    predicted_log_returns: np.ndarray,
    config: MPCConfig,
) -> Tuple[np.ndarray, Dict]:
    """Drop-in for mpc.py:27-117: returns (W [H, N] float64, {"status", "value"})."""
    y = np.asarray(predicted_log_returns)
    H, N = y.shape
    dev = _default_device()
    yt = torch.as_tensor(np.ascontiguousarray(y, dtype=np.float32), device=dev).reshape(1, H, N)
    wt = torch.as_tensor(np.asarray(current_weights, dtype=np.float64), device=dev).reshape(1, N)
    W, status, value = solve_mpc_log_utility_batched(wt, yt, config, return_full=True)
    st = _lib.STATUS_NAMES.get(int(status.item()), "solver_error")
    W_np = W[0].cpu().numpy()
    if st not in ("optimal", "optimal_inaccurate"):
        return np.tile(np.asarray(current_weights, dtype=np.float64), (H, 1)), {"status": st, "value": None}
    return W_np, {"status": st, "value": float(value.item())}


# ---- mean-variance MPC (mpc.py:119-184) ------------------------------------------------------

def solve_mpc_mean_variance_batched(
    current_weights: torch.Tensor,
    mu: torch.Tensor,
    cov_matrix: torch.Tensor,
    config: MPCConfig,
    return_full: bool = False,
    with_iters: bool = False,
):
    """Batched mean-variance solve on the device (kmpc_solve_mv).

    Args:
        current_weights: [B, N] device tensor (float64; other dtypes are converted).
        mu: [B, H, N] expected returns (the reference passes predicted log-returns / the rolling
            mean as mu, mpc.py:150-155); computed in float64.
        cov_matrix: [B, N, N] per-window covariance, or one shared [N, N] (mpc.py:123).
        config: MPCConfig (gamma, cost_coeff, allow_short; max_turnover is not part of this
            program in the reference either).
        return_full: return W [B, H, N] instead of W[:, 0].

    Returns:
        (W, status, value[, iters]) as solve_mpc_log_utility_batched; value is problem.value
        (mpc.py:172, maximize form), NaN where the fallback was applied.
    """
    _lib.require_gpu(mu)
    if mu.dim() != 3:
        raise ValueError("mu must be [B, H, N]")
    B, H, N = mu.shape
    dev = mu.device
    mu64 = mu.to(torch.float64).contiguous()
    wp = current_weights.to(device=dev, dtype=torch.float64).contiguous()
    if wp.shape != (B, N):
        raise ValueError(f"current_weights must be [{B}, {N}], got {tuple(wp.shape)}")
    S = torch.as_tensor(cov_matrix).to(device=dev, dtype=torch.float64).contiguous()
    if S.dim() == 2:
        if S.shape != (N, N):
            raise ValueError(f"cov_matrix must be [{N}, {N}] or [{B}, {N}, {N}]")
        stride = 0
    elif S.shape == (B, N, N):
        stride = N * N
    else:
        raise ValueError(f"cov_matrix must be [{N}, {N}] or [{B}, {N}, {N}], got {tuple(S.shape)}")
    if H > _lib.KMPC_MV_MAX_H or H * N > _lib.KMPC_MV_MAX_HN:
        raise _lib.KmpcError(f"mean-variance shape H={H}, N={N} exceeds the kernel limits "
                             f"(H <= {_lib.KMPC_MV_MAX_H}, H*N <= {_lib.KMPC_MV_MAX_HN})")
    W = torch.empty((B, H, N) if return_full else (B, N), dtype=torch.float64, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    value = torch.empty(B, dtype=torch.float64, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    d = _lib.MvDesc()
    d.B, d.N, d.H = int(B), int(N), int(H)
    d.gamma = float(config.gamma)
    d.cost_coeff = float(config.cost_coeff)
    d.allow_short = int(bool(config.allow_short))
    d.max_iter = int(getattr(config, "mv_max_iter", 100))
    d.tol = float(getattr(config, "mv_tol", 1e-10))
    d.return_full_W = int(bool(return_full))
    L = _lib.load()
    with torch.cuda.device(dev):
        nws = int(L.kmpc_mv_workspace_bytes(ctypes.byref(d)))
        ws = _workspace(dev, nws) if nws else None
        rc = L.kmpc_solve_mv_ws(ctypes.byref(d), mu64.data_ptr(), S.data_ptr(), stride, wp.data_ptr(),
                                W.data_ptr(), status.data_ptr(), value.data_ptr(), iters.data_ptr(),
                                ws.data_ptr() if ws is not None else None, nws, _lib.stream_handle(dev))
    _lib.check(rc)
    if with_iters:
        return W, status, value, iters
    return W, status, value


def solve_mpc_mean_variance(
    current_weights: np.ndarray,
    predicted_log_returns: np.ndarray,
    cov_matrix: np.ndarray,
    config: MPCConfig,
) -> Tuple[np.ndarray, Dict]:
    """Drop-in for mpc.py:119-184: returns (W [H, N] float64, info). On a non-optimal status the
    reference returns tile(current_weights) and {"status": s} without a "value" key (mpc.py:180-181)."""
    y = np.asarray(predicted_log_returns)
    H, N = y.shape
    dev = _default_device()
    mu = torch.as_tensor(np.ascontiguousarray(y, dtype=np.float64), device=dev).reshape(1, H, N)
    wt = torch.as_tensor(np.asarray(current_weights, dtype=np.float64), device=dev).reshape(1, N)
    S = torch.as_tensor(np.asarray(cov_matrix, dtype=np.float64), device=dev)
    W, status, value = solve_mpc_mean_variance_batched(wt, mu, S, config, return_full=True)
    st = _lib.STATUS_NAMES.get(int(status.item()), "solver_error")
    if st not in ("optimal", "optimal_inaccurate"):
        return np.tile(np.asarray(current_weights, dtype=np.float64), (H, 1)), {"status": st}
    return W[0].cpu().numpy(), {"status": st, "value": float(value.item())}
