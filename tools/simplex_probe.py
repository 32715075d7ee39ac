"""Dev probe: the configs[1] presolve alone (4,096 windows, N = 30, H = 5, c = tau = 0)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility_batched
B, N, H = 4096, 30, 5
rng = np.random.default_rng(0)
wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
cfg = MPCConfig(horizon=H, cost_coeff=0.0, max_turnover=0.0)
for _ in range(3):
    W, s, v = solve_mpc_log_utility_batched(wp, y, cfg)
torch.cuda.synchronize()
print("ok", int((s == 0).sum()))
