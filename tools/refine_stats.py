"""Dev probe: solve time / accuracy / refinement steps per Newton solve for dev builds
(libkmpc_dev_*.so, built by `make -C koopman_mpc_portfolio_rebalancing_amd/csrc dev ...`)."""
import ctypes, glob, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched
from oracle import solver as oracle


def read_stats(L, reset=1):
    """Sum of the dev counters of every solve translation unit that exports a reader."""
    tot = [0] * 18
    for fn in ("kmpc_debug_stats", "kmpc_debug_stats_case", "kmpc_debug_stats_c3"):
        if hasattr(L, fn):
            f = getattr(L, fn)
            f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
            st = (ctypes.c_ulonglong * 18)()
            f(st, reset)
            tot = [a + b for a, b in zip(tot, st)]
    return tot
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N, H = 100, 10
rng = np.random.default_rng(0)
wpn = rng.dirichlet(np.ones(N), B)
yn = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
wp = torch.tensor(wpn, device="cuda"); y = torch.tensor(yn, device="cuda")
nchk = 64
Wo, sto, vo, _ = oracle.solve_batch(wpn[:nchk], yn[:nchk], 1e-3, 0.2, precision="ld")
libs = sorted(glob.glob(os.path.join(os.path.dirname(_lib.LIB_PATH), "libkmpc_dev*.so")))
for path in libs:
    L = _lib.load(path)
    _lib._lib = L
    for nref in [int(x) for x in os.environ.get("REFINE", "1,2,3,6").split(",")]:
        cfg = MPCConfig(horizon=H, n_refine=nref if nref > 0 else -1)
        solve_mpc_log_utility_batched(wp, y, cfg); torch.cuda.synchronize()
        read_stats(L)
        t = time.time()
        W, s, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
        torch.cuda.synchronize(); dt = time.time() - t
        st = read_stats(L)
        Wn, vn = W.cpu().numpy(), v.cpu().numpy()
        print(f"{os.path.basename(path)} max_refine={nref} {dt*1e3:.1f} ms {B/dt:.0f} win/s "
              f"refines/solve {st[0]/max(st[1],1):.3f} iters {it.float().mean().item():.2f} "
              f"status={np.bincount(s.cpu().numpy(), minlength=5)} dobj {np.abs(vn[:nchk]-vo).max():.2e} "
              f"dW0 {np.abs(Wn[:nchk]-Wo[:, 0]).max():.2e}", flush=True)
