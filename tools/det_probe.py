"""Dev probe: run-to-run determinism of the solve kernel per block-size variant (not a test)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility_batched
from oracle import solver as oracle
from koopman_mpc_portfolio_rebalancing_amd import _lib

libs = sys.argv[1:] or [None]
CASES = [(100, 10), (300, 7), (500, 20), (700, 3), (1000, 2)] if libs == [None] else \
        [(100, 10), (300, 10), (520, 10), (600, 10), (700, 10), (1000, 10)]

for lib, (N, H) in [(l, c) for l in libs for c in CASES]:
    if lib: _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), lib))
    rng = np.random.default_rng(N * 31 + H)
    B = 6
    wp = rng.dirichlet(np.ones(N), B)
    y = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
    cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.3)
    outs = []
    for r in range(4):
        W, st, v, it = solve_mpc_log_utility_batched(torch.tensor(wp, device="cuda"), torch.tensor(y, device="cuda"),
                                                     cfg, return_full=True, with_iters=True)
        outs.append((W.cpu().numpy(), st.cpu().numpy(), v.cpu().numpy(), it.cpu().numpy()))
    Wo, sto, valo, ito = oracle.solve_batch(wp, y, 1e-3, 0.3)
    same = all(np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][2], o[2]) for o in outs[1:])
    print(f"{lib} N={N} H={H} deterministic={same} status={[np.bincount(o[1], minlength=5).tolist() for o in outs]} iters={[o[3].tolist() for o in outs]} "
          f"oracle iters={ito.tolist()} dobj={[float(np.abs(o[2]-valo).max()) for o in outs]}", flush=True)
