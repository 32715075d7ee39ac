"""Dev probe (GPU): solve-only time per call at small batches (the lock-step backtest's regime) —
float64-only vs mixed precision, C3 shape, bench yhat distribution (random N(5e-4, 0.015))."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, _lib, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
N, H = 100, 10
rng = np.random.default_rng(0)
for B in (1, 64, 256, 1024, 8192):
    wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
    for prec in ("f64", "auto"):
        cfg = MPCConfig(horizon=H, precision=prec)
        solve_mpc_log_utility_batched(wp, y, cfg)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            e0.record()
            W, s, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"B={B} {prec}: {min(ts) * 1e3:.0f} us per call, iters {it.float().mean().item():.2f}, "
              f"{min(ts) * 1e3 / it.float().mean().item():.1f} us per iteration", flush=True)
