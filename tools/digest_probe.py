"""Dev probe (GPU): digests of the solve's outputs (W0, objective, status, iterations) over a batch
of windows per variant library, so that an A/B can show two builds bit-identical.
    KMPC_DEV_LIB=libkmpc_x.so python tools/digest_probe.py"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, _lib, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))

rng = np.random.default_rng(3)
for (B, N, H, prec) in [(16384, 100, 10, "f64"), (16384, 100, 10, "auto"), (8192, 64, 10, "f64"),
                        (8192, 200, 10, "f64"), (16384, 30, 5, "f64"), (16384, 10, 5, "f64"), (4096, 90, 7, "f64")]:
    wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
    cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, precision=prec)
    W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    h = hashlib.sha256()
    for t in (W, v, st, it):
        h.update(t.cpu().numpy().tobytes())
    print(f"B={B} N={N} H={H} {prec}: {h.hexdigest()[:16]} iters {it.float().mean().item():.3f} "
          f"status {np.bincount(st.cpu().numpy(), minlength=5)}", flush=True)
