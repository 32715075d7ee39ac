#!/usr/bin/env python3
"""Dev measurement (CPU only): does a float32 interior-point phase followed by
a float64 finish keep the oracle's iteration count and optimum on the bench's own windows?

For 1,024 C3 windows (the bench model's torch-CPU rollout of window_inputs(0, 1024), c = 1e-3,
tau = 0.2, no short) it runs
  * the float64 oracle iteration from scratch (tools/dev/f32phase.c with mu_stop = 0), and
  * for each mu_s: the same iteration in float32 until mu <= mu_s (or a float breakdown /
    stagnation), then the float64 iteration from that state,
and reports iteration counts, statuses, the objective against the long-double oracle and, on a
subsample, the weak-duality certificate gap (oracle/certificate.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BUILD = os.path.join(ROOT, "tools", "dev", "_build")


def build():
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(ROOT, "tools", "dev", "f32phase.c")
    for name, flag in (("f32phase_f.so", "-DKMPC_REAL_FLOAT"), ("f32phase_d.so", "")):
        cmd = f"gcc -O2 -fPIC -fopenmp -ffp-contract=off -shared {flag} -o {BUILD}/{name} {src} -lm"
        subprocess.run(cmd, shell=True, check=True)
    libs = {}
    dp, fp, ip = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
    for k, name, sym in (("f", "f32phase_f.so", "kmpc_phase_f"), ("d", "f32phase_d.so", "kmpc_phase")):
        L = ctypes.CDLL(os.path.join(BUILD, name))
        fn = getattr(L, sym)
        fn.argtypes = [ctypes.c_int, ctypes.c_int, dp, fp, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                       ctypes.c_double, ctypes.c_double, dp, dp, ip, dp, dp, dp]
        fn.restype = ctypes.c_int
        libs[k] = fn
    return libs


def P(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t)) if a is not None else None


def phase(fn, wp, y, c, tau, mu_stop, st_in=None, max_iter=80, tol=1e-9):
    H, N = y.shape
    st_out = np.zeros(5 * H * N + 3 * H)
    it = np.zeros(1, np.int32)
    mu = np.zeros(1)
    W = np.zeros((H, N))
    obj = np.zeros(1)
    s = fn(N, H, P(wp, ctypes.c_double), P(y, ctypes.c_float), c, tau, max_iter, tol, mu_stop,
           P(st_in, ctypes.c_double), P(st_out, ctypes.c_double), P(it, ctypes.c_int), P(mu, ctypes.c_double),
           P(W, ctypes.c_double), P(obj, ctypes.c_double))
    return s, int(it[0]), st_out, W, float(obj[0]), float(mu[0])


def windows(B=1024):
    import bench
    N, L, H, hidden = 100, 256, 10, 1024
    obs = N * 20
    sd = bench.make_state_dict(obs, L, hidden, seed=0)
    x, wp = bench.window_inputs(0, B, N, obs, seed=0, device=torch.device("cpu"))
    y = bench.torch_cpu_rollout(sd, x, H, N, torch.full((N,), 5e-4), torch.full((N,), 0.015)).numpy()
    return wp.numpy(), np.ascontiguousarray(y, np.float32)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n_cert = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    c, tau = 1e-3, 0.2
    libs = build()
    wp, y = windows(B)
    from oracle import solver as osolver, certificate as cert
    Wl, stl, objl, itl = osolver.solve_batch(wp, y, c, tau, False, precision="ld", tol=1e-9)
    print(f"long-double oracle: mean iters {itl.mean():.2f}, optimal {int((stl == 0).sum())}/{B}")
    rows = []
    for mu_s in [float(v) for v in os.environ.get("MUS", "0,1e-1,1e-2,1e-3,1e-4,1e-5,1e-6").split(",")]:
        t0 = time.time()
        n32, n64, st, dobj, dW0, gaps, kinds = [], [], [], [], [], [], {1: 0, 2: 0, "done": 0}
        for b in range(B):
            if mu_s == 0:
                s, it64, _, W, ob, _ = phase(libs["d"], wp[b], y[b], c, tau, 0.0)
                it32 = 0
            else:
                s1, it32, state, W, ob, _ = phase(libs["f"], wp[b], y[b], c, tau, mu_s)
                if s1 == 100:
                    s, it64, _, W, ob, _ = phase(libs["d"], wp[b], y[b], c, tau, 0.0, st_in=state)
                else:
                    s, it64 = s1, 0
            n32.append(it32)
            n64.append(it64)
            st.append(s)
            dobj.append(abs(ob - objl[b]) if s <= 1 else np.inf)
            dW0.append(np.abs(W[0] - Wl[b, 0]).max() if s <= 1 else np.inf)
            if b < n_cert and s <= 1:
                r = cert.certify(W, wp[b], y[b], c, tau)
                gaps.append(r["gap"] / (1 + abs(r["f"])))
        n32, n64, st = np.array(n32), np.array(n64), np.array(st)
        row = {"mu_s": mu_s, "f32_iters": n32.mean(), "f64_iters": n64.mean(),
               "f64_iters_p90": float(np.percentile(n64, 90)), "f64_iters_max": int(n64.max()),
               "optimal": int((st == 0).sum()), "inaccurate": int((st == 1).sum()),
               "max_dobj": float(np.max(dobj)), "max_dW0": float(np.max(dW0)),
               "max_cert_gap_rel": float(np.max(gaps)) if gaps else None, "sec": time.time() - t0}
        rows.append(row)
        print(row, flush=True)
    return rows


if __name__ == "__main__":
    main()
