"""Lock-step backtest engine on the device: the bookkeeping kernel against
the numpy restatement of run_backtest (oracle/backtest_ref.py, backtest.py:133-219), the metrics
kernel against calculate_metrics (backtest.py:221-249), and whole lock-step runs against the
sequential run_backtest and the reference's recorded run.

Tolerance: the reference computes realized returns as float32 `np.exp(r) - 1`; the device
evaluates numpy's own float32 exp (kmpc_npexp.h), so the float32 returns are bit-identical and
the float64 bookkeeping differs only in the summation order of the block-reduced dot products
(w . r, |dw|_1): returns at atol 1e-15, values / turnovers / costs at rtol 1e-12. Runs whose target
weights come from the solver (device vs oracle, ~1e-6 apart) keep rtol 1e-6.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from koopman_mpc_portfolio_rebalancing_amd import (BacktestConfig, KoopmanModelSpec, KoopmanMPCStrategy,
                                                   MPCConfig, run_backtest, run_backtest_lockstep, _lib)
from koopman_mpc_portfolio_rebalancing_amd.backtest import METRIC_NAMES
from oracle import backtest_ref

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def device_replay(targets, realized, cost, capital):
    """kmpc_backtest_step over P paths replaying targets [P, S, N]; realized [P, T, N] (f32)."""
    P, S, N = targets.shape
    T = realized.shape[1]
    L = _lib.load()
    w = torch.full((P, N), 1.0 / N, dtype=torch.float64, device="cuda")
    value = torch.full((P,), capital, dtype=torch.float64, device="cuda")
    hist = torch.empty((P, S, 4), dtype=torch.float64, device="cuda")
    met = torch.empty((P, 5), dtype=torch.float64, device="cuda")
    d = _lib.BacktestDesc(P, N, S, cost)
    r = torch.tensor(realized, device="cuda")
    tg = torch.tensor(targets, device="cuda")
    for k in range(S):
        t = k
        rn = r[:, t + 1].contiguous() if t + 1 < T else None
        tk = tg[:, k].contiguous()
        _lib.check(L.kmpc_backtest_step(ctypes.byref(d), k, tk.data_ptr(), rn.data_ptr() if rn is not None else None,
                                        w.data_ptr(), value.data_ptr(), hist.data_ptr(), None))
    _lib.check(L.kmpc_backtest_metrics(ctypes.byref(d), hist.data_ptr(), met.data_ptr(), None))
    torch.cuda.synchronize()
    return hist.cpu().numpy(), met.cpu().numpy()


@pytest.mark.parametrize("N,S,tail", [(7, 11, True), (1, 6, False), (300, 8, True)])
def test_step_kernel_replays_reference_bookkeeping(N, S, tail):
    """tail: the last step has no t+1 return row (no market move, backtest.py:191)."""
    rng = np.random.default_rng(N + S)
    P, capital, cost = 5, 10000.0, 1e-3
    realized = rng.normal(5e-4, 0.02, (P, S if tail else S + 1, N)).astype(np.float32)
    targets = rng.dirichlet(np.ones(N), (P, S)) if N > 1 else np.ones((P, S, 1))
    hist, met = device_replay(targets, realized, cost, capital)
    for p in range(P):
        it = iter(targets[p])
        rows = backtest_ref.run_backtest(lambda t, w: next(it), realized[p], S + 1, 1, N, capital, 1, cost)
        ref = np.array([[h["portfolio_value"], h["return"], h["turnover"], h["cost"]] for h in rows])
        np.testing.assert_allclose(hist[p][:, 0], ref[:, 0], rtol=1e-12)
        np.testing.assert_allclose(hist[p][:, 1], ref[:, 1], rtol=0, atol=1e-15)
        np.testing.assert_allclose(hist[p][:, 2], ref[:, 2], rtol=1e-12, atol=1e-15)
        assert hist[p][0, 2] == pytest.approx(ref[0, 2], rel=1e-14)   # before any drift: float64 only
        np.testing.assert_allclose(hist[p][:, 3], ref[:, 3], rtol=1e-12, atol=1e-15)
        m = backtest_ref.calculate_metrics(ref[:, 1], ref[:, 2], ref[:, 0])
        for j, name in enumerate(METRIC_NAMES):
            assert met[p, j] == pytest.approx(m[name], rel=1e-4, abs=1e-6), name


def test_metrics_kernel_matches_calculate_metrics():
    rng = np.random.default_rng(3)
    P, S = 9, 40
    hist = np.empty((P, S, 4))
    hist[..., 1] = rng.normal(3e-4, 0.01, (P, S))
    hist[..., 2] = rng.uniform(0, 0.4, (P, S))
    hist[..., 0] = 1e4 * np.cumprod(1 + hist[..., 1], axis=1)
    hist[..., 3] = 0.0
    d = _lib.BacktestDesc(P, 4, S, 1e-3)
    h = torch.tensor(hist, device="cuda")
    met = torch.empty((P, 5), dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().kmpc_backtest_metrics(ctypes.byref(d), h.data_ptr(), met.data_ptr(), None))
    met = met.cpu().numpy()
    for p in range(P):
        m = backtest_ref.calculate_metrics(hist[p, :, 1], hist[p, :, 2], hist[p, :, 0])
        for j, name in enumerate(METRIC_NAMES):
            assert met[p, j] == pytest.approx(m[name], rel=1e-12, abs=1e-15), name


def test_lockstep_paths_match_sequential_and_reference_runs():
    from test_backtest_cpu import GoldenEnv
    g = np.load(os.path.join(GOLD, "backtest_koopman_mpc.npz"))
    meta = json.loads(str(g["meta"]))
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}
    spec = KoopmanModelSpec.from_state_dict(sd, meta["config"])
    env = GoldenEnv(g)
    strat = KoopmanMPCStrategy(spec, MPCConfig(**meta["mpc"]))
    bcfg = BacktestConfig(**meta["backtest"])
    data = torch.from_numpy(g["test_data"])
    realized = env.destandardize_returns(env.extract_current_returns(data))
    # three paths: the golden env, a time-shuffled copy and a scaled copy of its rows
    rng = np.random.default_rng(0)
    perm = torch.from_numpy(rng.permutation(data.shape[0]))
    obs = torch.stack([data, data[perm], data * 0.5])
    rets = torch.stack([env.destandardize_returns(env.extract_current_returns(o)) for o in obs])
    out = run_backtest_lockstep(strat, obs, rets, bcfg, g["mean"], g["std"], n_rows=int(g["test_len"]))
    val = out["portfolio_value"].cpu().numpy()
    # path 0 vs the reference's recorded run
    np.testing.assert_allclose(val[0], g["df_value"], rtol=1e-6)
    np.testing.assert_allclose(out["turnover"][0].cpu().numpy(), g["df_turnover"], atol=1e-4)
    assert out["metrics"]["Final Value"][0].item() == pytest.approx(meta["metrics"]["Final Value"], rel=1e-6)
    # every path vs the sequential run_backtest on an env holding that path's rows
    for p in range(3):
        e = GoldenEnv(g)
        e.test_dataset.data = obs[p].clone()
        df = run_backtest(strat, e, bcfg, verbose=False)
        np.testing.assert_allclose(val[p], df["portfolio_value"].values, rtol=1e-6)
        np.testing.assert_allclose(out["return"][p].cpu().numpy(), df["return"].values, rtol=0, atol=3e-7)
        # (a turnover of 1e-12 is solver noise around w_prev: absolute floor 1e-6)
        np.testing.assert_allclose(out["turnover"][p].cpu().numpy(), df["turnover"].values, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("prerollout", [True, False])
def test_lockstep_graph_replay_equals_eager_loop(prerollout):
    """run_backtest_lockstep(graph=True): the whole step sequence (window + bookkeeping launches of
    every step, then the metrics) captured in one HIP graph and replayed gives the eager loop's
    histories, weights and metrics bit for bit (C3-shaped model, 64 paths)."""
    import bench
    dev = torch.device("cuda")
    N, L, H, P, T = 100, 256, 10, 64, 24
    obs_n = N * 20
    spec = KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs_n, L, 1024, seed=0), bench.MODEL_CFG)
    strat = KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2), device="cuda")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(P, T, obs_n, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    cfg = BacktestConfig(horizon=H)
    eager = run_backtest_lockstep(strat, x, r, cfg, mean, std, prerollout=prerollout)
    graph = run_backtest_lockstep(strat, x, r, cfg, mean, std, graph=True, prerollout=prerollout)
    for k in ("portfolio_value", "return", "turnover", "cost", "weights"):
        assert torch.equal(eager[k], graph[k]), k
    for k, v in eager["metrics"].items():
        assert torch.equal(v, graph["metrics"][k]), k


def test_lockstep_prerollout_matches_per_step_windows(monkeypatch):
    """prerollout=True (every step's forecasts from batched kmpc_rollout launches up front, then one
    kmpc_solve per step) against one fused kmpc_window per step: the same program; the rollout's
    GEMM tiles depend on the batch size, so the forecasts agree to fp32 summation order and the
    histories to 1e-6. PREROLL_CHUNK = 128 windows: 2 steps per rollout launch (chunk edges)."""
    import bench
    from koopman_mpc_portfolio_rebalancing_amd import backtest as bt
    dev = torch.device("cuda")
    N, L, H, P, T = 100, 256, 10, 64, 19
    obs_n = N * 20
    spec = KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs_n, L, 1024, seed=0), bench.MODEL_CFG)
    strat = KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2), device="cuda")
    g = torch.Generator().manual_seed(2)
    x = torch.randn(P, T, obs_n, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    cfg = BacktestConfig(horizon=H)
    ref = run_backtest_lockstep(strat, x, r, cfg, mean, std, prerollout=False)
    monkeypatch.setattr(bt, "PREROLL_CHUNK", 128)
    pre = run_backtest_lockstep(strat, x, r, cfg, mean, std)
    assert pre["return"].shape == ref["return"].shape == (P, T - H)
    np.testing.assert_allclose(pre["portfolio_value"].cpu().numpy(), ref["portfolio_value"].cpu().numpy(), rtol=1e-6)
    np.testing.assert_allclose(pre["turnover"].cpu().numpy(), ref["turnover"].cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(pre["weights"].cpu().numpy(), ref["weights"].cpu().numpy(), atol=1e-5)


@pytest.mark.parametrize("P,groups", [(64, 4), (61, 3)])
def test_lockstep_path_groups_on_streams_equal_one_group(P, groups):
    """run_backtest_lockstep(groups=G): the paths in G contiguous groups, each stepping on its own
    HIP stream, against one group: every window goes through the same solve kernel, so histories,
    weights and metrics are bit-identical (uneven groups at P = 61)."""
    import bench
    dev = torch.device("cuda")
    N, L, H, T = 100, 256, 10, 22
    obs_n = N * 20
    spec = KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs_n, L, 1024, seed=0), bench.MODEL_CFG)
    strat = KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2), device="cuda")
    g = torch.Generator().manual_seed(3)
    x = torch.randn(P, T, obs_n, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    cfg = BacktestConfig(horizon=H)
    one = run_backtest_lockstep(strat, x, r, cfg, mean, std, groups=1)
    grp = run_backtest_lockstep(strat, x, r, cfg, mean, std, groups=groups)
    for k in ("portfolio_value", "return", "turnover", "cost", "weights"):
        assert torch.equal(one[k], grp[k]), k
    for k, v in one["metrics"].items():
        assert torch.equal(v, grp["metrics"][k]), k


@pytest.mark.parametrize("P,T,chunk,N,H,path", [(64, 22, None, 100, 10, 0), (61, 19, 128, 100, 10, 0),
                                                  (24, 14, None, 100, 5, 0), (20, 15, None, 50, 10, 0),
                                                  (16, 14, None, 150, 10, 0), (12, 12, None, 200, 5, 0),
                                                  # packed (N <= 32; KMPC_PATH_REGISTER packs at any batch
                                                  # size): one path per lane group
                                                  (64, 30, None, 10, 5, 1), (61, 14, 80, 10, 5, 1),
                                                  (22, 13, None, 16, 5, 1), (21, 13, None, 30, 5, 1),
                                                  (19, 16, None, 20, 10, 1), (9, 10, None, 8, 2, 0),
                                                  # N <= 32 under AUTO below KMPC_PACK_MIN_B paths: one per wave
                                                  (64, 20, None, 10, 5, 0), (19, 16, None, 20, 10, 0)])
def test_persistent_backtest_equals_lockstep_loop(P, T, chunk, N, H, path, monkeypatch):
    """run_backtest_lockstep(persistent=True): every step of every path in kmpc_backtest_run launches
    (one workgroup per path: the step's solve, then its bookkeeping, back to back) against the
    lock-step loop (one kmpc_solve over the P windows + one kmpc_backtest_step per step): the same
    window solve and bookkeeping code, so histories, weights and metrics are bit-identical. P = 61
    with 2 steps per rollout chunk: several launches, each resuming the paths' state. The other
    shapes: the constant-case kernels' persistent forms (64-, 128- and 256-thread windows, H = 5),
    the packed kernels' (N <= 32: 16-lane groups with 11 or 16 cold slots, 32-lane groups, H = 2 /
    5 / 10; one path per lane group, the bookkeeping's sums as group butterflies — the lock-step
    kernel's order — with ragged last blocks: P = 61, 22, 21, 19, 9), and N <= 32 under AUTO below
    KMPC_PACK_MIN_B paths (one window per wave, as kmpc_solve then runs the step's batch)."""
    import bench
    from koopman_mpc_portfolio_rebalancing_amd import backtest as bt
    dev = torch.device("cuda")
    L = 256
    obs_n = N * 20
    spec = KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs_n, L, 1024, seed=0), bench.MODEL_CFG)
    strat = KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, solver_path=path),
                               device="cuda")
    g = torch.Generator().manual_seed(4)
    x = torch.randn(P, T, obs_n, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    cfg = BacktestConfig(horizon=H)
    if chunk:
        monkeypatch.setattr(bt, "PREROLL_CHUNK", chunk)
    loop = run_backtest_lockstep(strat, x, r, cfg, mean, std, persistent=False, groups=1)
    per = run_backtest_lockstep(strat, x, r, cfg, mean, std, persistent=True)
    assert per["return"].shape == (P, T - H)
    for k in ("portfolio_value", "return", "turnover", "cost", "weights"):
        assert torch.equal(loop[k], per[k]), k
    for k, v in loop["metrics"].items():
        assert torch.equal(v, per["metrics"][k]), k
    assert run_backtest_lockstep(strat, x, r, cfg, mean, std)["portfolio_value"].equal(per["portfolio_value"])


def test_persistent_backtest_unsupported_shape():
    """persistent=True on a shape without a persistent kernel (N = 20, H = 3: the packed kernel of a
    ragged horizon, the generic constraint case) raises; the default falls back to the lock-step loop."""
    import bench
    dev = torch.device("cuda")
    N, L, H, P, T = 20, 256, 3, 8, 9
    obs_n = N * 20
    spec = KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs_n, L, 1024, seed=0), bench.MODEL_CFG)
    strat = KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2), device="cuda")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(P, T, obs_n, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    cfg = BacktestConfig(horizon=H)
    with pytest.raises(ValueError):
        run_backtest_lockstep(strat, x, r, cfg, mean, std, persistent=True)
    a = run_backtest_lockstep(strat, x, r, cfg, mean, std)
    b = run_backtest_lockstep(strat, x, r, cfg, mean, std, persistent=False, groups=1)
    assert torch.equal(a["portfolio_value"], b["portfolio_value"])
