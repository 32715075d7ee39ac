"""Dev probe: per-phase s_memtime cycles of the solve kernel (dev builds with -DKMPC_STATS)."""
import ctypes, glob, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib, MPCConfig, solve_mpc_log_utility_batched


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
wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
if os.environ.get("BENCH_Y", "1") == "1":
    # the benchmark's own yhat: bench.py's seeded finance_sparse model rolled out on its inputs
    import bench
    from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec
    sd = bench.make_state_dict(N * 20, 256, 1024, seed=0)
    km = DeviceKoopman(KoopmanModelSpec.from_state_dict(sd, bench.MODEL_CFG), torch.device("cuda", 0))
    x, _ = bench.window_inputs(0, B, N, N * 20, 0, torch.device("cuda", 0))
    y = km.rollout(x, np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32), H, N)
else:
    y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
from oracle import solver as oracle
nchk = 64
Wo, sto, vo, _ = oracle.solve_batch(wp[:nchk].cpu().numpy(), y[:nchk].cpu().numpy(), 1e-3, 0.2, precision="ld")
names = ["residual+best", "factor:prep", "factor:gram", "factor:chol", "newton", "step+corr", "update", "(lsolve)",
         "ls:rhs+sinv", "ls:qsolve+bs", "ls:trisolve", "ls:back+sinv", "nt:setup+bn", "nt:lsolve+acc", "nt:resid+max", "nt:tail"]
libs = sys.argv[2:] or sorted(os.path.basename(p) for p in glob.glob(os.path.join(os.path.dirname(_lib.LIB_PATH), "libkmpc_dev*.so")))
for name in libs:
    L = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), name))
    _lib._lib = L
    cfg = MPCConfig(horizon=H, precision=os.environ.get("PRECISION", "auto"))
    solve_mpc_log_utility_batched(wp, y, cfg); torch.cuda.synchronize()
    read_stats(L)
    t = time.time()
    W, s, v, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
    torch.cuda.synchronize(); dt = time.time() - t
    st = read_stats(L)
    nb = (B + 255) // 256
    iters = it.float().mean().item()
    tot = sum(st[2 + k] for k in range(7))
    print(f"{name}: {dt*1e3:.1f} ms {B/dt:.0f} win/s iters {iters:.2f} refines/solve {st[0]/max(st[1],1):.3f} "
          f"status {np.bincount(s.cpu().numpy(), minlength=5)} dobj {np.abs(v[:nchk].cpu().numpy() - vo).max():.2e} "
          f"dW0 {np.abs(W[:nchk].cpu().numpy() - Wo[:, 0]).max():.2e}")
    for k in range(16):
        c = st[2 + k] / nb / iters
        print(f"   {names[k]:14s} {c:10.0f} cycles/iter  {st[2 + k] / nb:12.0f} cycles/window  {100*st[2+k]/max(tot,1):5.1f}%")
