"""Generate the golden fixtures in tests/golden/ from the reference implementation.

Run in the build container only (the reference lives at /root/reference and never ships):

    python tests/golden/make_golden.py

What it records (all float data, no code):
  rollout_*.npz   reference model.py weights (seeded init), observations, stats, and the yhat the
                  reference KoopmanMPCStrategy.rebalance loop computes (backtest.py:99-121) using the
                  reference's own model / FinanceEnv methods.
  mpc_*.npz       MPC problems (w_prev, yhat, numpy's float32 R = np.exp(yhat), config) with the
                  long-double oracle optimum
                  (oracle/kmpc_oracle.c), plus SLSQP / dense-IPM cross-checks where small enough.
  headline_*.npz  the bench's models (weights regenerated from their seed by the test) run through
                  the reference's GenericKM / LISTAKM and rebalance op order on 64 (c5: 16) windows:
                  obs, stats, yhat (c5: and the same model in float64).
  backtest_*.npz  reference run_backtest + calculate_metrics (backtest.py:133-249) on a synthetic
                  FinanceEnv built with the reference's data_finance functions; the MPC solve inside
                  KoopmanMPCStrategy is routed to the oracle (cvxpy is not installed here), and every
                  solver call's inputs/outputs are recorded.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import pandas as pd
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("KMPC_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

# cvxpy is not installed: an in-memory stub lets mpc.py / backtest.py import (the solve is replaced).
_cvx = types.ModuleType("cvxpy")


class _SolverError(Exception):
    pass


_cvx.SolverError = _SolverError
sys.modules.setdefault("cvxpy", _cvx)

import config as ref_config  # noqa: E402
import model as ref_model  # noqa: E402
import data_finance as ref_data  # noqa: E402
import backtest as ref_backtest  # noqa: E402
import mpc as ref_mpc  # noqa: E402

from oracle import dense_ipm, solver as oracle_solver  # noqa: E402


def oracle_solve(current_weights, predicted_log_returns, config):
    """Stand-in for mpc.solve_mpc_log_utility with its return contract (mpc.py:113-117)."""
    H, N = predicted_log_returns.shape
    W, st, obj, _ = oracle_solver.solve(current_weights, predicted_log_returns, config.cost_coeff,
                                        config.max_turnover, config.allow_short)
    name = oracle_solver.STATUS_NAMES[st]
    if name not in ("optimal", "optimal_inaccurate"):
        return np.tile(current_weights, (H, 1)), {"status": name, "value": None}
    return W, {"status": name, "value": obj}


def state_arrays(model):
    return {f"w:{k}": v.detach().cpu().numpy().astype(np.float32) for k, v in model.state_dict().items()}


def make_env(n_assets, emb, n_rows, seed, seq_len):
    """Synthetic FinanceEnv through the reference's own data_finance functions."""
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range("2015-01-01", periods=n_rows)
    lr = pd.DataFrame(rng.normal(4e-4, 0.012, (n_rows, n_assets)), index=dates,
                      columns=[f"A{i}" for i in range(n_assets)])
    train_end = str(dates[int(n_rows * 0.5)].date())
    val_end = str(dates[int(n_rows * 0.6)].date())
    stats = ref_data.compute_standardization_stats(lr, train_end)
    tr, trd, va, vad, te, ted = ref_data.create_finance_splits(lr, stats, train_end, val_end, emb)
    meta = {"n_assets": n_assets, "embedding_dim": emb}
    env = ref_data.FinanceEnv(ref_data.FinanceDataset(tr, trd, seq_len), ref_data.FinanceDataset(va, vad, seq_len),
                              ref_data.FinanceDataset(te, ted, seq_len), stats, meta)
    return env


def reference_yhat(model, env, obs, H):
    """The exact op sequence of KoopmanMPCStrategy.rebalance (backtest.py:85-121), per window."""
    out = []
    with torch.no_grad():
        model.eval()
        for b in range(obs.shape[0]):
            z = model.encode(torch.from_numpy(obs[b]).unsqueeze(0))
            preds = []
            for _ in range(H):
                z = model.step_latent(z)
                p = model.decode(z)
                y = env.destandardize_returns(env.extract_current_returns(p))
                preds.append(y.cpu().numpy().flatten())
            out.append(np.array(preds))
    return np.stack(out).astype(np.float32)


def orthogonal(L, scale, seed):
    g = torch.Generator().manual_seed(seed)
    q, _ = torch.linalg.qr(torch.randn(L, L, generator=g))
    return (q * scale).float()


def rollout_cases():
    cases = []
    # (name, preset, overrides)
    cases.append(("generic_finance", "finance_sparse", dict(TARGET_SIZE=16, LAYERS=[32, 32])))
    cases.append(("generic_ball_tanh", "finance_sparse",
                  dict(TARGET_SIZE=12, LAYERS=[24], NORM_FN="ball", ACTIVATION="tanh", DEC_LAYERS=[10],
                       DEC_BIAS=True)))
    cases.append(("generic_gelu_lastrelu", "finance_sparse",
                  dict(TARGET_SIZE=16, LAYERS=[20, 20], ACTIVATION="gelu", LAST_RELU=True)))
    cases.append(("lista_linear", "lista", dict(TARGET_SIZE=24, LINEAR=True, LOOPS=10, ALPHA=5e-3)))
    cases.append(("lista_mlp", "lista_nonlinear", dict(TARGET_SIZE=20, LINEAR=False, LAYERS=[32], LOOPS=4,
                                                       ALPHA=5e-3)))
    return cases


def build_model(preset, ov, obs_size, seed):
    cfg = ref_config.get_config(preset)
    cfg.MODEL.TARGET_SIZE = ov["TARGET_SIZE"]
    if "LAYERS" in ov:
        cfg.MODEL.ENCODER.LAYERS = list(ov["LAYERS"])
    if "NORM_FN" in ov:
        cfg.MODEL.NORM_FN = ov["NORM_FN"]
    if "ACTIVATION" in ov:
        cfg.MODEL.ENCODER.ACTIVATION = ov["ACTIVATION"]
        cfg.MODEL.DECODER.ACTIVATION = ov["ACTIVATION"]
    if "LAST_RELU" in ov:
        cfg.MODEL.ENCODER.LAST_RELU = ov["LAST_RELU"]
    if "DEC_LAYERS" in ov:
        cfg.MODEL.DECODER.LAYERS = list(ov["DEC_LAYERS"])
    if "DEC_BIAS" in ov:
        cfg.MODEL.DECODER.USE_BIAS = ov["DEC_BIAS"]
    if "LINEAR" in ov:
        cfg.MODEL.ENCODER.LISTA.LINEAR_ENCODER = ov["LINEAR"]
        cfg.MODEL.ENCODER.LISTA.NUM_LOOPS = ov["LOOPS"]
        cfg.MODEL.ENCODER.LISTA.ALPHA = ov["ALPHA"]
    torch.manual_seed(seed)
    if cfg.MODEL.MODEL_NAME == "LISTAKM":
        # contractive LISTA: L = 1.1 * ||W_d||_2^2 of the init dictionary
        torch.manual_seed(seed)
        wd = torch.randn(obs_size, cfg.MODEL.TARGET_SIZE) * 0.01
        cfg.MODEL.ENCODER.LISTA.L = float(1.1 * torch.linalg.matrix_norm(wd, ord=2) ** 2)
        torch.manual_seed(seed)
    model = ref_model.make_model(cfg, obs_size)
    with torch.no_grad():
        model.kmat.copy_(orthogonal(cfg.MODEL.TARGET_SIZE, 0.95, seed + 1))
        if cfg.MODEL.MODEL_NAME == "LISTAKM":
            # spread the dictionary so the decode is not ~0 (the reference init is 0.01 * randn)
            model.dict.mul_(50.0)
    model.eval()
    return cfg, model


def make_rollout_goldens():
    N, d, H, B = 5, 4, 3, 12
    obs_size = N * d
    for ci, (name, preset, ov) in enumerate(rollout_cases()):
        cfg, model = build_model(preset, ov, obs_size, seed=100 + ci)
        env = make_env(N, d, 120, seed=7 + ci, seq_len=1)
        rng = np.random.default_rng(ci)
        obs = rng.normal(0, 1, (B, obs_size)).astype(np.float32)
        yhat = reference_yhat(model, env, obs, H)
        meta = {"model_name": cfg.MODEL.MODEL_NAME, "norm_fn": cfg.MODEL.NORM_FN,
                "enc_layers": list(cfg.MODEL.ENCODER.LAYERS), "enc_act": cfg.MODEL.ENCODER.ACTIVATION,
                "enc_bias": cfg.MODEL.ENCODER.USE_BIAS, "enc_last_relu": cfg.MODEL.ENCODER.LAST_RELU,
                "dec_layers": list(cfg.MODEL.DECODER.LAYERS), "dec_act": cfg.MODEL.DECODER.ACTIVATION,
                "dec_bias": cfg.MODEL.DECODER.USE_BIAS, "target_size": cfg.MODEL.TARGET_SIZE,
                "lista_loops": cfg.MODEL.ENCODER.LISTA.NUM_LOOPS, "lista_alpha": cfg.MODEL.ENCODER.LISTA.ALPHA,
                "lista_L": cfg.MODEL.ENCODER.LISTA.L, "lista_linear": cfg.MODEL.ENCODER.LISTA.LINEAR_ENCODER,
                "N": N, "H": H, "obs": obs_size, "config": cfg.to_dict()}
        np.savez_compressed(os.path.join(HERE, f"rollout_{name}.npz"), obs=obs, yhat=yhat,
                            mean=env.stats.mean.astype(np.float64), std=env.stats.std.astype(np.float64),
                            meta=json.dumps(meta), **state_arrays(model))
        print("rollout", name, yhat.shape, float(np.abs(yhat).max()))


HEADLINE_CASES = [  # name, N, emb, latent, hidden, H, weight seed, obs seed (bench.py's models)
    ("c3", 100, 20, 256, 1024, 10, 0, 0),    # BASELINE configs[2]: the bench's headline model
    ("c2", 30, 20, 128, 1024, 5, 1, 100),    # configs[1] (bench.secondary_c2)
    ("c1", 10, 20, 128, 1024, 5, 10, 10),    # configs[0] (bench.secondary_c1 / cpu_baseline_c1)
]
HEADLINE_WINDOWS = 64


def state_checksums(sd):
    """float64 sum and sum of squares per tensor: binds a golden to the weights the test regenerates."""
    return {k: [float(v.double().sum()), float((v.double() ** 2).sum())] for k, v in sd.items()}


def make_headline_goldens():
    """The bench's own models (bench.make_state_dict, finance_sparse GenericKM layout) loaded into the
    reference's GenericKM (model.py:701-797, strict load_state_dict), rolled out by the reference's
    rebalance op order (backtest.py:99-121: encode, then H x step_latent / decode / extract /
    destandardize, batch 1 per window) on 64 windows of the bench's input stream. Only the
    observations, the de-standardisation stats, the yhat and weight checksums are stored: the test
    regenerates the weights from the seed and tiles the 64 rows to the batch sizes whose kernels it
    pins (the latent-powers GEMM path from 8,192 windows, the fused latent loops below)."""
    import bench
    for name, N, emb, L, hidden, H, wseed, xseed in HEADLINE_CASES:
        obs_n = N * emb
        cfg = ref_config.get_config("finance_sparse")
        cfg.MODEL.TARGET_SIZE = L
        cfg.MODEL.ENCODER.LAYERS = [hidden, hidden]
        model = ref_model.make_model(cfg, obs_n)
        sd = bench.make_state_dict(obs_n, L, hidden, seed=wseed)
        model.load_state_dict(sd, strict=True)
        model.eval()
        # per-asset stats (not constants), through the reference's own FinanceEnv methods
        mean = np.linspace(-8e-4, 1.2e-3, N)
        std = np.linspace(0.01, 0.025, N)
        env = types.SimpleNamespace(n_assets=N, stats=ref_data.FinanceStats(mean, std, [f"A{i}" for i in range(N)]))
        env.extract_current_returns = types.MethodType(ref_data.FinanceEnv.extract_current_returns, env)
        env.destandardize_returns = types.MethodType(ref_data.FinanceEnv.destandardize_returns, env)
        x, _ = bench.window_inputs(0, HEADLINE_WINDOWS, N, obs_n, seed=xseed, device=torch.device("cpu"))
        obs = x.numpy().astype(np.float32)
        yhat = reference_yhat(model, env, obs, H)
        meta = {"N": N, "emb": emb, "L": L, "hidden": hidden, "H": H, "weight_seed": wseed, "obs_seed": xseed,
                "checksums": state_checksums(sd), "torch": torch.__version__,
                "generator": "tests/golden/make_golden.py make_headline_goldens"}
        np.savez_compressed(os.path.join(HERE, f"headline_{name}.npz"), obs=obs, yhat=yhat, mean=mean, std=std,
                            meta=json.dumps(meta))
        print("headline", name, yhat.shape, float(np.abs(yhat).max()))


def make_headline_c5():
    """BASELINE configs[4]'s model (bench.make_lista_state_dict: LISTAKM, linear We, 10 loops,
    latent 512, obs 10,000, N = 500, H = 20) loaded strictly into the reference's LISTAKM
    (model.py:804-850, the 'lista' config), 16 windows of bench.secondary_c5's input stream, the
    reference's rebalance op order in fp32 — and the same model in float64 (the reference modules
    cast with .double()), the yardstick of both fp32 rollouts at this depth (10 shrink loops, 20
    latent steps, K = 10,000 dot products: the reference's own fp32 result is ~1e-6 from it)."""
    import copy
    import bench
    N, L, H, emb, xseed = 500, 512, 20, 20, 200
    obs_n = N * emb
    sd, lc = bench.make_lista_state_dict(obs_n, L, seed=2)
    cfg = ref_config.get_config("lista")
    cfg.MODEL.TARGET_SIZE = L
    cfg.MODEL.ENCODER.LISTA.L = lc
    cfg.MODEL.ENCODER.LISTA.NUM_LOOPS = 10
    cfg.MODEL.ENCODER.LISTA.ALPHA = 5e-3
    cfg.MODEL.ENCODER.LISTA.LINEAR_ENCODER = True
    model = ref_model.make_model(cfg, obs_n)
    model.load_state_dict(sd, strict=True)
    model.eval()
    mean = np.linspace(-8e-4, 1.2e-3, N)
    std = np.linspace(0.01, 0.025, N)
    env = types.SimpleNamespace(n_assets=N, stats=ref_data.FinanceStats(mean, std, [f"A{i}" for i in range(N)]))
    env.extract_current_returns = types.MethodType(ref_data.FinanceEnv.extract_current_returns, env)
    env.destandardize_returns = types.MethodType(ref_data.FinanceEnv.destandardize_returns, env)
    x, _ = bench.window_inputs(0, 16, N, obs_n, seed=xseed, device=torch.device("cpu"))
    obs = x.numpy().astype(np.float32)
    yhat = reference_yhat(model, env, obs, H)
    md = copy.deepcopy(model).double()
    y64 = []
    with torch.no_grad():
        for b in range(obs.shape[0]):
            z = md.encode(torch.from_numpy(obs[b]).double().unsqueeze(0))
            ps = []
            for _ in range(H):
                z = md.step_latent(z)
                p = md.decode(z)[..., :N]
                ps.append((p * torch.from_numpy(std) + torch.from_numpy(mean)).numpy().ravel())
            y64.append(np.array(ps))
    y64 = np.stack(y64)
    meta = {"N": N, "emb": emb, "L": L, "H": H, "weight_seed": 2, "obs_seed": xseed, "lista_L": lc,
            "checksums": state_checksums(sd), "torch": torch.__version__,
            "generator": "tests/golden/make_golden.py make_headline_c5"}
    np.savez_compressed(os.path.join(HERE, "headline_c5.npz"), obs=obs, yhat=yhat, yhat_f64=y64, mean=mean, std=std,
                        meta=json.dumps(meta))
    print("headline c5", yhat.shape, float(np.abs(yhat).max()), float(np.abs(yhat - y64).max() / np.abs(yhat).max()))


def make_mpc_goldens():
    rng = np.random.default_rng(2024)
    # reference test_mpc cases with their exact optima (tests/test_mpc.py:6-55 of the reference)
    kat = {
        "pref_wp": np.array([0.5, 0.5]), "pref_y": np.array([[0.1, 0.0]], np.float32), "pref_W": np.array([[0.6, 0.4]]),
        "cost_wp": np.array([1.0, 0.0]), "cost_y": np.array([[0.0, 0.01]], np.float32), "cost_W": np.array([[1.0, 0.0]]),
        "feas_wp": np.ones(5) / 5, "feas_y": np.zeros((3, 5), np.float32),
    }
    np.savez_compressed(os.path.join(HERE, "mpc_kat.npz"), **kat)
    shapes = [  # name, B, N, H, c, tau, allow_short, loc, scale, xcheck
        ("small_c1e-3_t0.2", 24, 6, 3, 1e-3, 0.2, False, 5e-4, 0.02, True),
        ("small_c1e-2_t0.5", 24, 5, 2, 1e-2, 0.5, False, 5e-4, 0.02, True),
        ("small_c0_t0.2", 24, 7, 2, 0.0, 0.2, False, 5e-4, 0.02, True),
        ("small_c1e-3_t0", 24, 6, 3, 1e-3, 0.0, False, 5e-4, 0.02, True),
        ("small_short_c1e-2_t0.5", 16, 4, 2, 1e-2, 0.5, True, 5e-4, 0.02, True),
        ("cfg1_N10_H5", 32, 10, 5, 1e-3, 0.5, False, 5e-4, 0.015, False),
        ("cfg2_N30_H5_simplex", 32, 30, 5, 0.0, 0.0, False, 5e-4, 0.015, False),
        ("cfg3_N100_H10", 16, 100, 10, 1e-3, 0.2, False, 5e-4, 0.015, False),
        ("cfg5_N500_H20", 2, 500, 20, 1e-3, 0.2, False, 5e-4, 0.015, False),
    ]
    for name, B, N, H, c, tau, short, loc, scale, xcheck in shapes:
        wp = rng.dirichlet(np.ones(N), B)
        y = rng.normal(loc, scale, (B, H, N)).astype(np.float32)
        W, st, obj, it = oracle_solver.solve_batch(wp, y, c, tau, short)
        extra = {}
        if xcheck:
            Wd = np.stack([dense_ipm.dense_ipm(wp[b], y[b], c, tau, short)[0] for b in range(B)])
            Ws = np.stack([dense_ipm.slsqp(wp[b], y[b], c, tau, short)[0] for b in range(B)])
            extra = {"W_dense": Wd, "W_slsqp": Ws}
        # R: the gross returns exactly as the reference forms them (np.exp on the float32 yhat,
        # mpc.py:55) — what cvxpy receives, after promotion to float64
        np.savez_compressed(os.path.join(HERE, f"mpc_{name}.npz"), w_prev=wp, yhat=y, R=np.exp(y), W=W, status=st,
                            obj=obj, iters=it, config=np.array([c, tau, float(short)]), **extra)
        print("mpc", name, np.bincount(st, minlength=5), int(it.max()))


def make_backtest_goldens():
    N, d, H = 5, 4, 3
    obs_size = N * d
    cfg, model = build_model("finance_sparse", dict(TARGET_SIZE=16, LAYERS=[32, 32]), obs_size, seed=11)
    env = make_env(N, d, 200, seed=3, seq_len=10)
    calls = []

    def recording_solve(current_weights, predicted_log_returns, config):
        W, info = oracle_solve(current_weights, predicted_log_returns, config)
        calls.append((np.array(current_weights, np.float64), np.array(predicted_log_returns, np.float32),
                      np.array(W, np.float64), info["status"]))
        return W, info

    ref_backtest.solve_mpc_log_utility = recording_solve
    mcfg = ref_mpc.MPCConfig(horizon=H, gamma=0.0, cost_coeff=1e-3, max_turnover=0.5)
    bcfg = ref_backtest.BacktestConfig(initial_capital=10000.0, horizon=H, rebalance_freq=1, cost_coeff=1e-3)
    strat = ref_backtest.KoopmanMPCStrategy(model, mcfg)
    df = ref_backtest.run_backtest(strat, env, bcfg, verbose=False)
    met = ref_backtest.calculate_metrics(df)
    df_bh = ref_backtest.run_backtest(ref_backtest.BuyAndHoldStrategy(), env, bcfg, verbose=False)
    met_bh = ref_backtest.calculate_metrics(df_bh)
    # rebalance_freq = 2 quirk (intermediate returns skipped, backtest.py:173)
    bcfg2 = ref_backtest.BacktestConfig(initial_capital=10000.0, horizon=H, rebalance_freq=2, cost_coeff=1e-3)
    n_before = len(calls)
    df2 = ref_backtest.run_backtest(strat, env, bcfg2, verbose=False)
    calls2 = calls[n_before:]
    del calls[n_before:]
    meta = {"N": N, "d": d, "H": H, "mpc": {"horizon": H, "cost_coeff": 1e-3, "max_turnover": 0.5},
            "backtest": {"initial_capital": 10000.0, "horizon": H, "rebalance_freq": 1, "cost_coeff": 1e-3},
            "metrics": {k: float(v) for k, v in met.items()},
            "metrics_bh": {k: float(v) for k, v in met_bh.items()},
            "statuses": [c[3] for c in calls], "config": cfg.to_dict()}
    np.savez_compressed(
        os.path.join(HERE, "backtest_koopman_mpc.npz"),
        test_data=env.test_dataset.data.numpy(), test_len=len(env.test_dataset),
        dates=np.array([str(x.date()) for x in env.test_dataset.dates]),
        mean=env.stats.mean.astype(np.float64), std=env.stats.std.astype(np.float64),
        df_value=df["portfolio_value"].values, df_return=df["return"].values, df_turnover=df["turnover"].values,
        df_cost=df["cost"].values, df_date=np.array([str(x.date()) for x in df["date"]]),
        bh_value=df_bh["portfolio_value"].values, bh_return=df_bh["return"].values,
        bh_turnover=df_bh["turnover"].values, bh_cost=df_bh["cost"].values,
        f2_value=df2["portfolio_value"].values, f2_turnover=df2["turnover"].values,
        call_wprev=np.stack([c[0] for c in calls]), call_yhat=np.stack([c[1] for c in calls]),
        call_W=np.stack([c[2] for c in calls]), meta=json.dumps(meta), **state_arrays(model))
    print("backtest", len(df), len(calls), met)

    # the reference's tests/test_backtest.py MockFinanceEnv mechanics (data = torch.randn(10, 10))
    torch.manual_seed(0)

    class MockEnv:
        n_assets = 2

        def __init__(self):
            from unittest.mock import MagicMock
            self.test_dataset = MagicMock()
            self.test_dataset.dates = pd.date_range("2021-01-01", periods=10)
            self.test_dataset.data = torch.randn(10, 10)
            self.test_dataset.__len__.return_value = 10
            self.extract_current_returns = lambda x: x[..., :2]
            self.destandardize_returns = lambda x: x * 0.01

    env_m = MockEnv()
    dfm = ref_backtest.run_backtest(ref_backtest.BuyAndHoldStrategy(), env_m,
                                    ref_backtest.BacktestConfig(horizon=2, initial_capital=1000.0), verbose=False)
    metm = ref_backtest.calculate_metrics(pd.DataFrame({"return": [0.01, -0.01, 0.02, 0.0],
                                                        "turnover": [0.1, 0.0, 0.0, 0.0],
                                                        "portfolio_value": [1010, 999.9, 1019.9, 1019.9]}))
    np.savez_compressed(os.path.join(HERE, "backtest_mock.npz"), data=env_m.test_dataset.data.numpy(),
                        df_value=dfm["portfolio_value"].values, df_return=dfm["return"].values,
                        df_turnover=dfm["turnover"].values, df_cost=dfm["cost"].values,
                        metrics=json.dumps({k: float(v) for k, v in metm.items()}))
    print("mock", len(dfm))


def make_dmd_goldens():
    """reference DMDStrategy (baselines.py:127-187): fitted operator and the predicted log-returns
    it hands to the solver at each call (the solve routed to the oracle, recorded)."""
    import baselines as ref_baselines
    N, d, H = 5, 4, 3
    env = make_env(N, d, 160, seed=5, seq_len=10)
    calls = []

    def recording_solve(current_weights, predicted_log_returns, config):
        W, info = oracle_solve(current_weights, predicted_log_returns, config)
        calls.append((np.array(current_weights, np.float64), np.array(predicted_log_returns, np.float32),
                      np.array(W, np.float64)))
        return W, info

    ref_baselines.solve_mpc_log_utility = recording_solve
    mcfg = ref_mpc.MPCConfig(horizon=H, gamma=0.0, cost_coeff=1e-3, max_turnover=0.3)
    strat = ref_baselines.DMDStrategy(env.train_dataset.data, mcfg)
    w = np.ones(N) / N
    for t in range(12):
        w = strat.rebalance(t, w, env)
    np.savez_compressed(os.path.join(HERE, "dmd.npz"), K=strat.K, train_data=env.train_dataset.data.numpy(),
                        test_data=env.test_dataset.data.numpy(), mean=env.stats.mean, std=env.stats.std,
                        call_wprev=np.stack([c[0] for c in calls]), call_yhat=np.stack([c[1] for c in calls]),
                        call_W=np.stack([c[2] for c in calls]), meta=json.dumps({"N": N, "d": d, "H": H,
                        "mpc": {"horizon": H, "cost_coeff": 1e-3, "max_turnover": 0.3}}))
    print("dmd", strat.K.shape, len(calls))


def make_embedding_goldens():
    """reference standardize_returns + time_delay_embedding (data_finance.py:243-300, 331)."""
    rng = np.random.default_rng(77)
    T, N, d = 40, 6, 4
    y = rng.normal(4e-4, 0.02, (T, N))
    df = pd.DataFrame(y, columns=[f"A{i}" for i in range(N)],
                      index=pd.date_range("2020-01-01", periods=T))
    stats = ref_data.compute_standardization_stats(df, "2020-01-25")
    z = ref_data.standardize_returns(df, stats).values.astype(np.float32)
    emb = ref_data.time_delay_embedding(z, d)
    np.savez_compressed(os.path.join(HERE, "embedding.npz"), log_returns=y, mean=stats.mean, std=stats.std,
                        standardized=z, embedded=emb, emb_dim=d)
    print("embedding", emb.shape)


if __name__ == "__main__":
    which = sys.argv[1:] or ["rollout", "mpc", "backtest", "embedding", "dmd", "headline"]
    if "headline" in which:
        make_headline_goldens()
    if "headline" in which or "headline_c5" in which:
        make_headline_c5()
    if "dmd" in which:
        make_dmd_goldens()
    if "embedding" in which:
        make_embedding_goldens()
    if "rollout" in which:
        make_rollout_goldens()
    if "mpc" in which:
        make_mpc_goldens()
    if "backtest" in which:
        make_backtest_goldens()
