"""Dev probe: register kernels (path 1) vs the large-window kernel (path 2) on the same shapes,
through the per-call kmpc_solve_desc.path — the data behind kmpc_solve.hip's dispatch rule."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
L = _lib.load()

def run(B, N, H, path):
    rng = np.random.default_rng(0)
    wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
    cfg = MPCConfig(horizon=H, solver_path=path)
    solve_mpc_log_utility_batched(wp[:64], y[:64], cfg); torch.cuda.synchronize()
    t = time.time()
    W, st, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize(); dt = time.time() - t
    return B / dt, v.cpu().numpy(), int((st.cpu().numpy() <= 1).sum())

shapes = [(int(a), int(b)) for a, b in (s.split("x") for s in sys.argv[1:])] if len(sys.argv) > 1 else \
    [(64, 20), (100, 15), (100, 20), (128, 21), (160, 10), (192, 10), (256, 10), (256, 5), (320, 10), (400, 5), (500, 5), (500, 10)]
for N, H in shapes:
    B = max(1024, min(16384, 4_000_000 // (N * H)))
    try:
        r1, v1, ok1 = run(B, N, H, 1)
    except _lib.KmpcError as e:   # no register kernel for this shape
        print(f"N={N:4d} H={H:2d}: register path unsupported ({e})", flush=True)
        continue
    r2, v2, ok2 = run(B, N, H, 2)
    print(f"N={N:4d} H={H:2d} B={B:5d} register {r1:9.0f} win/s  big {r2:9.0f} win/s  ratio {r2 / r1:5.2f}  "
          f"ok {ok1}/{ok2}  max|dobj| {np.nanmax(np.abs(v1 - v2)):.1e}", flush=True)
