"""Dev probe: one C3-size solve launch (for rocprofv3 counter passes). Uses libkmpc_dev_*.so if
KMPC_DEV_LIB is set, else the product library."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N, H = 100, 10
rng = np.random.default_rng(0)
wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
cfg = MPCConfig(horizon=H)
for rep in range(int(os.environ.get("REPS", "2"))):
    torch.cuda.synchronize(); t = time.time()
    W, s, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize(); dt = time.time() - t
    print(f"{dt*1e3:.1f} ms {B/dt:.0f} win/s iters {it.float().mean().item():.2f} status {np.bincount(s.cpu().numpy(), minlength=5)}"
          f" sum(obj) {v.double().sum().item():.12e} sum|W0| {W.double().abs().sum().item():.12e}", flush=True)
