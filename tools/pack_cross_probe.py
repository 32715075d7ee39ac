"""Dev probe (GPU): solve time of the packed (lane-group) and one-window-per-wave register kernels
by batch size at N <= 32 shapes — where does packing start to pay?"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility_batched

for (N, H) in [(10, 5), (16, 5), (30, 5), (20, 10), (8, 2)]:
    rng = np.random.default_rng(0)
    for B in (64, 256, 1024, 2048, 4096, 8192, 16384, 65536):
        wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
        y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
        t = {}
        for path in (0, 3):
            cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, solver_path=path)
            solve_mpc_log_utility_batched(wp, y, cfg)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(5):
                s = time.perf_counter()
                solve_mpc_log_utility_batched(wp, y, cfg)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - s)
            t[path] = best * 1e3
        print(f"N={N} H={H} B={B}: packed {t[0]:.3f} ms, unpacked {t[3]:.3f} ms ({t[0] / t[3]:.2f}x)", flush=True)
