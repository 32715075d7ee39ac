"""Dev probe: solve throughput vs asset count N at H=10 (and the C5 shape) — where the window's
per-asset cost and the per-workgroup overheads (barriers, idle lanes) show."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))

def run(B, N, H, cost=1e-3, tau=0.2):
    rng = np.random.default_rng(0)
    wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
    cfg = MPCConfig(horizon=H, cost_coeff=cost, max_turnover=tau)
    solve_mpc_log_utility_batched(wp[:64], y[:64], cfg); torch.cuda.synchronize()
    t = time.time()
    W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize(); dt = time.time() - t
    print(f"B={B} N={N} H={H} {dt*1e3:.1f} ms {B/dt:.0f} windows/s {B*N/dt/1e6:.1f} M asset-windows/s "
          f"iters {it.float().mean().item():.1f} status {np.bincount(st.cpu().numpy(), minlength=5)}", flush=True)

for N in [32, 64, 100, 128, 192, 256]:
    run(16384, N, 10)
for H in [5, 10, 20]:
    run(2048 if H == 20 else 4096, 500, H)
