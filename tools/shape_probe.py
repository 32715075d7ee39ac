"""Dev probe: solve-kernel throughput at the BASELINE config shapes (not the benchmark).
usage: python tools/shape_probe.py [B_C5]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
if os.environ.get("KMPC_DEV_LIB"):   # A/B of variant libraries built next to libkmpc.so
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))

def run(name, B, N, H, cost, tau, reps=2):
    rng = np.random.default_rng(0)
    wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
    cfg = MPCConfig(horizon=H, cost_coeff=cost, max_turnover=tau)
    solve_mpc_log_utility_batched(wp[:64], y[:64], cfg); torch.cuda.synchronize()
    for _ in range(reps):
        t = time.time()
        W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
        torch.cuda.synchronize(); dt = time.time() - t
    print(f"{name}: B={B} N={N} H={H} {dt*1e3:.1f} ms {B/dt:.0f} windows/s iters {it.float().mean().item():.1f} "
          f"status {np.bincount(st.cpu().numpy(), minlength=5)}", flush=True)

SHAPES = os.environ.get("SHAPES", "")
_run = run
def run(name, *a, **k):
    if not SHAPES or name in SHAPES.split("|"):
        _run(name, *a, **k)

run("C2", 65536, 30, 5, 0.0, 0.0)
run("N=64,H=10", 65536, 64, 10, 1e-3, 0.2)
run("N=30,H=5,cost", 65536, 30, 5, 1e-3, 0.2)
run("C1-shape", 65536, 10, 5, 1e-3, 0.2)
run("C3", 65536, 100, 10, 1e-3, 0.2)
run("N=120,H=10", 65536, 120, 10, 1e-3, 0.2)
run("N=90,H=7", 65536, 90, 7, 1e-3, 0.2)
run("N=200,H=10", 16384, 200, 10, 1e-3, 0.2)
run("N=250,H=10", 8192, 250, 10, 1e-3, 0.2)
run("N=500,H=10", 4096, 500, 10, 1e-3, 0.2)
run("N=100,H=20", 8192, 100, 20, 1e-3, 0.2)
run("N=1000,H=5", 2048, 1000, 5, 1e-3, 0.2)
run("C5", int(sys.argv[1]) if len(sys.argv) > 1 else 2048, 500, 20, 1e-3, 0.2, reps=2)
