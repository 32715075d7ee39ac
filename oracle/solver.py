"""ctypes binding of the float64 C oracle (oracle/kmpc_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATHS = {"d": os.path.join(_HERE, "_build", "libkmpc_oracle.so"),
              "ld": os.path.join(_HERE, "_build", "libkmpc_oracle_ld.so")}
_libs = {}

STATUS_NAMES = {0: "optimal", 1: "optimal_inaccurate", 2: "infeasible", 3: "unbounded",
                4: "solver_error"}


def build(force: bool = False) -> None:
    """Compile the C oracle with the Makefile in this directory (gcc, no reference sources)."""
    src = os.path.join(_HERE, "kmpc_oracle.c")
    stale = [p for p in _LIB_PATHS.values()
             if not os.path.exists(p) or os.path.getmtime(p) < os.path.getmtime(src)]
    if force or stale:
        subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib(precision: str = "ld"):
    """precision 'ld' (long double, the parity reference) or 'd' (float64, the CPU baseline)."""
    if precision not in _libs:
        build()
        sfx = "_ld" if precision == "ld" else ""
        L = ctypes.CDLL(_LIB_PATHS[precision])
        dp = ctypes.POINTER(ctypes.c_double)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int)
        solve_f = getattr(L, "kmpc_oracle_solve" + sfx)
        batch_f = getattr(L, "kmpc_oracle_solve_batch" + sfx)
        obj_f = getattr(L, "kmpc_oracle_objective" + sfx)
        solve_f.argtypes = [ctypes.c_int, ctypes.c_int, dp, fp, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_double, dp, dp, ip]
        solve_f.restype = ctypes.c_int
        batch_f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, fp,
                                              ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_double, dp, dp, ip, ip]
        batch_f.restype = ctypes.c_int
        obj_f.argtypes = [ctypes.c_int, ctypes.c_int, dp, fp, ctypes.c_double, dp]
        obj_f.restype = ctypes.c_double
        gr_f = L.kmpc_oracle_gross_returns
        gr_f.argtypes = [ctypes.c_long, fp, fp]
        gr_f.restype = None
        _libs[precision] = (solve_f, batch_f, obj_f, gr_f)
    return _libs[precision]


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def solve(w_prev, yhat, cost_coeff=1e-3, max_turnover=0.2, allow_short=False, max_iter=0, tol=0.0,
          precision="ld"):
    """One window. Returns (W [H,N] float64, status int, obj float, iters int)."""
    wp = np.ascontiguousarray(w_prev, dtype=np.float64)
    y = np.ascontiguousarray(yhat, dtype=np.float32)
    H, N = y.shape
    W = np.empty((H, N), np.float64)
    obj = np.zeros(1, np.float64)
    it = np.zeros(1, np.int32)
    st = lib(precision)[0](N, H, _p(wp, ctypes.c_double), _p(y, ctypes.c_float),
                                 float(cost_coeff), float(max_turnover), int(bool(allow_short)),
                                 int(max_iter), float(tol), _p(W, ctypes.c_double),
                                 _p(obj, ctypes.c_double), _p(it, ctypes.c_int))
    return W, int(st), float(obj[0]), int(it[0])


def solve_batch(w_prev, yhat, cost_coeff=1e-3, max_turnover=0.2, allow_short=False, max_iter=0,
                tol=0.0, precision="ld"):
    """B windows (OpenMP over windows). Returns (W [B,H,N], status [B], obj [B], iters [B])."""
    wp = np.ascontiguousarray(w_prev, dtype=np.float64)
    y = np.ascontiguousarray(yhat, dtype=np.float32)
    B, H, N = y.shape
    W = np.empty((B, H, N), np.float64)
    obj = np.empty(B, np.float64)
    st = np.empty(B, np.int32)
    it = np.empty(B, np.int32)
    lib(precision)[1](B, N, H, _p(wp, ctypes.c_double), _p(y, ctypes.c_float),
                                  float(cost_coeff), float(max_turnover), int(bool(allow_short)),
                                  int(max_iter), float(tol), _p(W, ctypes.c_double),
                                  _p(obj, ctypes.c_double), _p(st, ctypes.c_int),
                                  _p(it, ctypes.c_int))
    return W, st, obj, it


def objective(W, w_prev, yhat, cost_coeff):
    W = np.ascontiguousarray(W, np.float64)
    wp = np.ascontiguousarray(w_prev, np.float64)
    y = np.ascontiguousarray(yhat, np.float32)
    H, N = y.shape
    return float(lib()[2](N, H, _p(wp, ctypes.c_double), _p(y, ctypes.c_float),
                                             float(cost_coeff), _p(W, ctypes.c_double)))


def gross_returns(yhat):
    """R = np.exp(yhat) in float32 by the oracle's restatement of numpy's float32 exp."""
    y = np.ascontiguousarray(yhat, np.float32)
    R = np.empty_like(y)
    lib("d")[3](y.size, _p(y, ctypes.c_float), _p(R, ctypes.c_float))
    return R
