"""Quick device timing of the solve kernel (dev probe, not the benchmark)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility_batched
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N, H = 100, 10
rng = np.random.default_rng(0)
wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
cfg = MPCConfig(horizon=H)
W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
torch.cuda.synchronize()
for rep in range(3):
    t = time.time()
    W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize()
    dt = time.time() - t
    print(f"B={B} {dt*1e3:.1f} ms  {B/dt:.0f} windows/s  status={np.bincount(st.cpu().numpy(), minlength=5)} iters {it.float().mean().item():.1f}", flush=True)
