"""ctypes binding of libkmpc.so (the C ABI declared in include/kmpc.h).

The library is built in-tree (``python -m koopman_mpc_portfolio_rebalancing_amd.build`` or
``__graft_entry__.build()``). There is no CPU fallback: if the library or a GPU is missing, the
product path raises :class:`KmpcError`.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first so libkmpc.so binds to the same one)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkmpc.so")

KMPC_OK = 0
KMPC_ERR_UNSUPPORTED = -2   # shape outside what the kernels were built for
KMPC_MAX_LAYERS = 8
KMPC_MAX_N = 1024
KMPC_MAX_H = 21          # the Schur system (3H rows) is factored by one 64-lane wavefront

MODEL_GENERIC, MODEL_LISTA = 0, 1
ACT = {"relu": 0, "tanh": 1, "gelu": 2}
NORM = {"id": 0, "ball": 1}
DTYPE = {"fp32": 0, "bf16": 1, "fp32_f32mfma": 2}
LATENT_FORM = {"auto": 0, "unfused": 1, "sequential": 2}   # kmpc_rollout_desc.latent_unfused (KMPC_LATENT_*)

STATUS_NAMES = {0: "optimal", 1: "optimal_inaccurate", 2: "infeasible", 3: "unbounded",
                4: "solver_error"}

KMPC_MV_MAX_HN = 1024    # mean-variance solve: H * N per workgroup (> 128: workspace-resident matrix)
KMPC_MV_MAX_H = 16

EXPORTED_SYMBOLS = ("kmpc_solve", "kmpc_rollout", "kmpc_window", "kmpc_workspace_bytes",
                    "kmpc_backtest_step", "kmpc_backtest_metrics", "kmpc_standardize", "kmpc_strerror",
                    "kmpc_version", "kmpc_solve_mv", "kmpc_rolling_moments", "kmpc_solve_mv_ws",
                    "kmpc_mv_workspace_bytes", "kmpc_gross_returns", "kmpc_backtest_run")

PATH_AUTO, PATH_REGISTER, PATH_LARGE, PATH_REGISTER_UNPACKED = 0, 1, 2, 3   # kmpc_solve_desc.path
PRECISION_AUTO, PRECISION_F64, PRECISION_MIXED = 0, 1, 2   # kmpc_solve_desc.precision
MIXED_MIN_B = 2048   # KMPC_MIXED_MIN_B: AUTO runs the mixed pair from this many windows per call
PACK_MIN_B = 512     # KMPC_PACK_MIN_B: AUTO packs N <= 32 windows 2-4 per wave from this many (H > 2)

# ABI of the structs below (include/kmpc.h); 0.2.0 appended kmpc_solve_desc.path and
# kmpc_rollout_desc.latent_unfused, 0.3.0 kmpc_solve_desc.precision and .mu_handoff, so an older
# library would read them past its structs' end; 0.4.0 added enum values only (KMPC_PRECISION_MIXED,
# KMPC_DTYPE_F32_F32MFMA), no layout change; 0.5.0 added kmpc_backtest_run;
# 0.6.0 enum values only (KMPC_LATENT_SEQUENTIAL)
ABI_VERSION = "0.6.0"


class KmpcError(RuntimeError):
    pass


class SolveDesc(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("N", ctypes.c_int), ("H", ctypes.c_int),
                ("cost_coeff", ctypes.c_double), ("max_turnover", ctypes.c_double),
                ("allow_short", ctypes.c_int), ("max_iter", ctypes.c_int),
                ("tol", ctypes.c_double), ("return_full_W", ctypes.c_int), ("n_refine", ctypes.c_int),
                ("path", ctypes.c_int), ("precision", ctypes.c_int), ("mu_handoff", ctypes.c_double)]


class MvDesc(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("N", ctypes.c_int), ("H", ctypes.c_int),
                ("gamma", ctypes.c_double), ("cost_coeff", ctypes.c_double),
                ("allow_short", ctypes.c_int), ("max_iter", ctypes.c_int),
                ("tol", ctypes.c_double), ("return_full_W", ctypes.c_int)]


class Mlp(ctypes.Structure):
    _fields_ = [("n_layers", ctypes.c_int), ("dims", ctypes.c_int * (KMPC_MAX_LAYERS + 1)),
                ("act", ctypes.c_int), ("last_relu", ctypes.c_int),
                ("weight", ctypes.c_void_p * KMPC_MAX_LAYERS),
                ("bias", ctypes.c_void_p * KMPC_MAX_LAYERS)]


class RolloutDesc(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("N", ctypes.c_int), ("H", ctypes.c_int), ("L", ctypes.c_int),
                ("obs", ctypes.c_int), ("model_kind", ctypes.c_int), ("norm_fn", ctypes.c_int),
                ("encoder", Mlp), ("lista_S", ctypes.c_void_p), ("lista_loops", ctypes.c_int),
                ("lista_thresh", ctypes.c_float), ("kmat", ctypes.c_void_p), ("decoder", Mlp),
                ("mean", ctypes.c_void_p), ("std", ctypes.c_void_p), ("obs_ld", ctypes.c_int),
                ("dtype", ctypes.c_int), ("latent_unfused", ctypes.c_int)]


class BacktestDesc(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int), ("N", ctypes.c_int), ("S", ctypes.c_int),
                ("cost_coeff", ctypes.c_double)]


_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libkmpc.so (raises KmpcError if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise KmpcError(f"{p} not found: build it with `python -m koopman_mpc_portfolio_rebalancing_amd.build`")
    L = ctypes.CDLL(p)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.kmpc_solve.argtypes = [ctypes.POINTER(SolveDesc), vp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.kmpc_solve.restype = ctypes.c_int
    L.kmpc_rollout.argtypes = [ctypes.POINTER(RolloutDesc), vp, vp, vp, sz, vp]
    L.kmpc_rollout.restype = ctypes.c_int
    L.kmpc_window.argtypes = [ctypes.POINTER(RolloutDesc), ctypes.POINTER(SolveDesc), vp, vp, vp, vp,
                              vp, vp, vp, vp, sz, vp]
    L.kmpc_window.restype = ctypes.c_int
    L.kmpc_backtest_step.argtypes = [ctypes.POINTER(BacktestDesc), ctypes.c_int, vp, vp, vp, vp, vp, vp]
    L.kmpc_backtest_step.restype = ctypes.c_int
    L.kmpc_backtest_run.argtypes = [ctypes.POINTER(BacktestDesc), ctypes.POINTER(SolveDesc), ctypes.c_int,
                                    ctypes.c_int, vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp]
    L.kmpc_backtest_run.restype = ctypes.c_int
    L.kmpc_backtest_metrics.argtypes = [ctypes.POINTER(BacktestDesc), vp, vp, vp]
    L.kmpc_backtest_metrics.restype = ctypes.c_int
    L.kmpc_standardize.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp]
    L.kmpc_standardize.restype = ctypes.c_int
    L.kmpc_solve_mv.argtypes = [ctypes.POINTER(MvDesc), vp, vp, sz, vp, vp, vp, vp, vp, vp]
    L.kmpc_solve_mv.restype = ctypes.c_int
    L.kmpc_solve_mv_ws.argtypes = [ctypes.POINTER(MvDesc), vp, vp, sz, vp, vp, vp, vp, vp, vp, sz, vp]
    L.kmpc_solve_mv_ws.restype = ctypes.c_int
    L.kmpc_mv_workspace_bytes.argtypes = [ctypes.POINTER(MvDesc)]
    L.kmpc_mv_workspace_bytes.restype = ctypes.c_size_t
    ci = ctypes.c_int
    L.kmpc_rolling_moments.argtypes = [ci, ci, ci, ci, vp, ci, vp, vp, vp, vp, vp, vp, vp]
    L.kmpc_rolling_moments.restype = ctypes.c_int
    L.kmpc_workspace_bytes.argtypes = [ctypes.POINTER(RolloutDesc), ctypes.POINTER(SolveDesc)]
    L.kmpc_workspace_bytes.restype = ctypes.c_size_t
    L.kmpc_gross_returns.argtypes = [sz, vp, vp, vp]
    L.kmpc_gross_returns.restype = ctypes.c_int
    L.kmpc_strerror.argtypes = [ctypes.c_int]
    L.kmpc_strerror.restype = ctypes.c_char_p
    L.kmpc_version.argtypes = []
    L.kmpc_version.restype = ctypes.c_char_p
    ver = L.kmpc_version().decode()
    if ver.split()[1:2] != [ABI_VERSION]:
        raise KmpcError(f"{p} reports {ver!r}; these bindings need ABI {ABI_VERSION}: rebuild the library")
    if path is None:
        _lib = L
    return L


def check(rc: int) -> None:
    if rc != KMPC_OK:
        msg = load().kmpc_strerror(rc).decode()
        raise KmpcError(f"libkmpc call failed: {msg} ({rc})")


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


_STREAMS: dict = {}


def group_streams(n: int, device: torch.device) -> list:
    """n HIP streams of their own for concurrent launch sequences (the lock-step path groups),
    created back to back once per process and device. HIP hands the process's GPU_MAX_HW_QUEUES
    hardware queues to streams round-robin in creation order, so n consecutive creations land on n
    different queues (measured: tools/queue_probe.py); streams from torch's pool may share one,
    and two streams on one queue run their kernels one after the other."""
    import ctypes
    key = torch.device(device).index or 0
    if key not in _STREAMS or len(_STREAMS[key]) < n:
        hip = ctypes.CDLL("libamdhip64.so")
        made = []
        with torch.cuda.device(key):
            for _ in range(max(n, 4)):
                h = ctypes.c_void_p()
                if hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) != 0:   # hipStreamNonBlocking
                    raise KmpcError("hipStreamCreateWithFlags failed")
                made.append(torch.cuda.ExternalStream(h.value, device=torch.device("cuda", key)))
        _STREAMS[key] = made
    return _STREAMS[key][:n]


def require_gpu(t: torch.Tensor) -> None:
    if not t.is_cuda:
        raise KmpcError("libkmpc kernels need device (HIP) tensors; got a CPU tensor")
