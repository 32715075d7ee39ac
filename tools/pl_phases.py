"""Dev probe: per-phase s_memtime cycles of the period-lane kernel (libkmpc_plprof.so, make plprof)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib
L = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), "libkmpc_plprof.so"))
L.kmpc_debug_pl_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
names = ["update->resid", "residuals", "factor elem+owner", "gens+vv", "MFMA gram", "schur LDLT",
         "A (rhs, px)", "B (g, owner Qinv)", "C (Z^T x)", "schur solve", "D (owner Qinv)", "E (ds, sums, refine)",
         "step+corrector", "", "", ""]
N, H = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "100x10").split("x")]
B = 4096
rng = np.random.default_rng(0)
wp = torch.tensor(rng.dirichlet(np.ones(N), B), device="cuda")
y = torch.tensor(rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32), device="cuda")
d = _lib.SolveDesc(); d.B, d.N, d.H = B, N, H; d.cost_coeff, d.max_turnover = 1e-3, 0.2; d.path = 3
W = torch.empty(B, N, dtype=torch.float64, device="cuda"); st = torch.empty(B, dtype=torch.int32, device="cuda")
v = torch.empty(B, dtype=torch.float64, device="cuda"); it = torch.empty(B, dtype=torch.int32, device="cuda")
def run():
    _lib.check(L.kmpc_solve(ctypes.byref(d), y.data_ptr(), wp.data_ptr(), W.data_ptr(), st.data_ptr(), v.data_ptr(),
                            it.data_ptr(), None, 0, None)); torch.cuda.synchronize()
run()
buf = (ctypes.c_ulonglong * 16)()
L.kmpc_debug_pl_phases(buf, 1)
run()
L.kmpc_debug_pl_phases(buf, 1)
nblk = (B + 63) // 64
iters = it.float().mean().item()
tot = sum(buf)
print(f"N={N} H={H}: {iters:.1f} iterations, {tot / nblk / iters:,.0f} cycles per iteration (block 0 of every 64)")
for k in range(16):
    if buf[k]:
        print(f"  {k:2d} {names[k]:22s} {buf[k] / nblk / iters:10,.0f}  {100 * buf[k] / tot:5.1f}%")
