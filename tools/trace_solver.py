"""Dev probe: per-iteration trace of problem 0 on the device vs the oracle (KMPC_ORACLE_TRACE)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import _lib
from koopman_mpc_portfolio_rebalancing_amd.mpc import MPCConfig, _solve_desc
N, H, c, tau = [int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4])] if len(sys.argv) > 4 else (10, 5, 1e-3, 0.2)
rng = np.random.default_rng(0)
wp = rng.dirichlet(np.ones(N), 1); y = rng.normal(5e-4, 0.015, (1, H, N)).astype(np.float32)
L = _lib.load()
L.kmpc_solve_trace.argtypes = [ctypes.POINTER(_lib.SolveDesc)] + [ctypes.c_void_p] * 8 + [ctypes.c_size_t, ctypes.c_void_p]
d = _solve_desc(1, N, H, MPCConfig(horizon=H, cost_coeff=c, max_turnover=tau), True)
yt = torch.tensor(y, device="cuda"); wt = torch.tensor(wp, device="cuda")
W = torch.empty((1, H, N), dtype=torch.float64, device="cuda"); st = torch.empty(1, dtype=torch.int32, device="cuda")
ob = torch.empty(1, dtype=torch.float64, device="cuda"); it = torch.empty(1, dtype=torch.int32, device="cuda")
tr = torch.full((4 * 100,), float("nan"), dtype=torch.float64, device="cuda")
nws = int(L.kmpc_workspace_bytes(None, ctypes.byref(d)))
ws = torch.empty(max(nws, 8), dtype=torch.uint8, device="cuda")
rc = L.kmpc_solve_trace(ctypes.byref(d), yt.data_ptr(), wt.data_ptr(), W.data_ptr(), st.data_ptr(), ob.data_ptr(), it.data_ptr(), tr.data_ptr(), ws.data_ptr(), nws, None)
torch.cuda.synchronize()
print("rc", rc, "status", st.item(), "iters", it.item(), "obj", ob.item())
t = tr.cpu().numpy().reshape(-1, 4)
for k in range(it.item() + 1):
    print("gpu it %d mu %.3e rd %.3e pr %.3e step %.3f" % (k, *t[k]))
from oracle import solver
os.environ["KMPC_ORACLE_TRACE"] = "1"
Wo, sto, obo, ito = solver.solve(wp[0], y[0], c, tau, precision="d")
print("oracle status", sto, "iters", ito, "obj", obo, "max|dW|", np.abs(W[0].cpu().numpy() - Wo).max())
