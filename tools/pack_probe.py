"""Dev probe: small windows packed on lane groups (path 0/1) vs one window per wave
(KMPC_PATH_REGISTER_UNPACKED) on the same inputs: throughput, iterations, status, objective gap.
usage: python tools/pack_probe.py [NxH[:case] ...]   case: c (cost+cap, default), n (no-short only), s (short+cost)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):   # a variant library (csrc/Makefile pvar)
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
ONLY = os.environ.get("PACKED_ONLY") == "1"

CASES = {"c": dict(cost_coeff=1e-3, max_turnover=0.2), "n": dict(cost_coeff=0.0, max_turnover=0.0),
         "s": dict(cost_coeff=1e-3, max_turnover=0.0, allow_short=True)}


def run(B, N, H, case, path, reps=3):
    rng = np.random.default_rng(1)
    wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
    cfg = MPCConfig(horizon=H, solver_path=path, **CASES[case])
    out = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(reps):
        out = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize()
    dt = (time.time() - t) / reps
    W, st, v, it = (x.cpu().numpy() for x in out)
    return B / dt, W, st, v, it


args = sys.argv[1:] or ["10x5", "16x5", "30x5", "32x5", "10x10", "30x10", "8x2", "10x5:n", "10x5:s", "20x7"]
for a in args:
    shape, _, case = a.partition(":")
    case = case or "c"
    N, H = (int(x) for x in shape.split("x"))
    B = 262144 if N * H <= 100 else 131072
    p = 1 if case == "n" else 0
    r1, W1, s1, v1, i1 = run(B, N, H, case, p)
    if ONLY:
        print(f"N={N:3d} H={H:2d} {case}: packed {r1 / 1e6:6.2f} M/s ({i1.mean():5.2f} it, {(s1 == 0).mean():.4f} opt)",
              flush=True)
        continue
    r0, W0, s0, v0, i0 = run(B, N, H, case, _lib.PATH_REGISTER_UNPACKED)
    ok = (s1 <= 1) & (s0 <= 1)
    print(f"N={N:3d} H={H:2d} {case}: packed {r1 / 1e6:6.2f} M/s ({i1.mean():5.2f} it, {(s1 == 0).mean():.4f} opt)  "
          f"unpacked {r0 / 1e6:6.2f} M/s ({i0.mean():5.2f} it, {(s0 == 0).mean():.4f} opt)  x{r1 / r0:4.2f}  "
          f"max|dobj| {np.max(np.abs(v1[ok] - v0[ok])):.1e}  max|dW| {np.max(np.abs(W1[ok] - W0[ok])):.1e}", flush=True)
