"""Dev probe: GPU run_backtest engine (run_backtest_lockstep) throughput —
P lock-stepped backtest paths of the C3 model (100 assets, latent 256, H = 10, c = 1e-3, tau = 0.2)
over T test rows; path-steps/s = P x steps / wall time (one window launch + one bookkeeping
launch per step)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from koopman_mpc_portfolio_rebalancing_amd import (BacktestConfig, DeviceKoopman, KoopmanModelSpec, KoopmanMPCStrategy,
                                                   MPCConfig)
from koopman_mpc_portfolio_rebalancing_amd.backtest import run_backtest_lockstep
from koopman_mpc_portfolio_rebalancing_amd import _lib
if os.environ.get("KMPC_DEV_LIB"):   # a variant library built by csrc/Makefile (tvar / var)
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))

dev = torch.device("cuda", 0)
N, L, H = 100, 256, 10
obs = N * 20
spec = KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs, L, 1024, seed=0), bench.MODEL_CFG)
# MU: the solve's precision / float32 handoff per run ("f64" = float64 only; a number = mu_handoff)
MUS = os.environ.get("MU", "5e-5").split(",")
strats = {mu: KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2,
                                                 **({"precision": "f64"} if mu == "f64" else
                                                    {"precision": "mixed"} if mu == "mixed" else {"mu_handoff": float(mu)})),
                                 device="cuda") for mu in MUS}
CASES = [tuple(int(v) for v in c.split('x')) for c in os.environ.get('CASES', '64x260,1024x260,8192x60').split(',')]
for P, T in CASES:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(P, T, obs, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    cfg = BacktestConfig(horizon=H)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    for graph, pre, mu in [(g_ == '1', p_ == '1', mu) for g_ in os.environ.get('GRAPH', '0,1').split(',')
                           for p_ in os.environ.get('PRE', '1,0').split(',') for mu in MUS]:
        strat = strats[mu]
        for grp in [None if v == "d" else int(v) for v in os.environ.get("PATH_GROUPS", "d").split(",")]:
            if grp is not None and grp > 1 and (graph or not pre):
                continue
            out = run_backtest_lockstep(strat, x[:, :H + 2], r[:, :H + 2], cfg, mean, std, graph=graph,
                                        prerollout=pre, groups=grp)   # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = run_backtest_lockstep(strat, x, r, cfg, mean, std, graph=graph, prerollout=pre, groups=grp)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            S = out["return"].shape[1]
            print(f"P={P} T={T} graph={graph} prerollout={pre} mu={mu} groups={grp}: {S} steps in {dt*1e3:.1f} ms -> {P*S/dt:.0f} path-steps/s, "
                  f"{dt/S*1e3:.3f} ms/step, final value mean {out['portfolio_value'][:, -1].mean().item():.1f}", flush=True)
