"""Quick device timing/accuracy of the solve kernel vs n_refine (dev probe, not the benchmark)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility_batched
from oracle import solver as oracle
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N, H = 100, 10
rng = np.random.default_rng(0)
wpn = rng.dirichlet(np.ones(N), B)
yn = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
wp = torch.tensor(wpn, device="cuda")
y = torch.tensor(yn, device="cuda")
nchk = 48
Wo, sto, vo, _ = oracle.solve_batch(wpn[:nchk], yn[:nchk], 1e-3, 0.2, precision="ld")
for nref in [int(x) for x in os.environ.get("REFINE", "1,2,6").split(",")]:
    cfg = MPCConfig(horizon=H, n_refine=nref if nref > 0 else -1)
    W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize()
    for rep in range(2):
        t = time.time()
        W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
        torch.cuda.synchronize()
        dt = time.time() - t
    Wn, vn = W.cpu().numpy(), v.cpu().numpy()
    print(f"refine={nref} B={B} {dt*1e3:.1f} ms {B/dt:.0f} windows/s status={np.bincount(st.cpu().numpy(), minlength=5)} "
          f"iters {it.float().mean().item():.1f}  dobj {np.abs(vn[:nchk]-vo).max():.2e} dW0 {np.abs(Wn[:nchk]-Wo[:, 0]).max():.2e}",
          flush=True)
