"""Dev probe: one C5-shaped solve launch (N=500, H=20; BASELINE configs[4]) for rocprofv3 passes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N, H = int(os.environ.get("PN", "500")), int(os.environ.get("PH", "20"))
rng = np.random.default_rng(0)
wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
cfg = MPCConfig(horizon=H)
for rep in range(int(os.environ.get("REPS", "2"))):
    torch.cuda.synchronize(); t = time.time()
    W, s, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize(); dt = time.time() - t
    print(f"N={N} H={H} B={B} {dt*1e3:.1f} ms {B/dt:.0f} win/s iters {it.float().mean().item():.2f}", flush=True)
NCHK = int(os.environ.get("NCHK", "0"))   # > 0: the first NCHK windows against the long-double oracle
print("status", np.bincount(s.cpu().numpy(), minlength=5), flush=True)
if NCHK:
    from oracle import solver as oracle
    Wo, sto, vo, _ = oracle.solve_batch(wp[:NCHK].cpu().numpy(), y[:NCHK].cpu().numpy(), cfg.cost_coeff,
                                        cfg.max_turnover, precision="ld")
    print(f"oracle[{NCHK}]: status {np.bincount(sto, minlength=5)} max|dobj| "
          f"{np.abs(v[:NCHK].cpu().numpy() - vo).max():.2e} max|dW0| {np.abs(W[:NCHK].cpu().numpy() - Wo[:, 0]).max():.2e}",
          flush=True)
