"""The train.py checkpoint contract (reference train.py:475-491): a torch.save'd dict
{step, epoch, model_state_dict, optimizer_state_dict, config (cfg.to_dict()), metrics,
finance_metadata} loads with the weights-only unpickler and drives KoopmanMPCStrategy exactly like
the state dict it holds (KoopmanModelSpec.from_checkpoint, koopman.py; run_experiment.py:70-79 is
the reference consumer)."""
import json
import os

import numpy as np
import pytest
import torch

from koopman_mpc_portfolio_rebalancing_amd import KoopmanModelSpec, KoopmanMPCStrategy, MPCConfig

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _golden():
    g = np.load(os.path.join(GOLD, "backtest_koopman_mpc.npz"))
    meta = json.loads(str(g["meta"]))
    sd = {k[2:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith("w:")}
    return g, meta, sd


def _write_checkpoint(path, sd, cfg_dict):
    """The dict train.py:475-483 writes, with an AdamW-shaped optimizer state."""
    params = list(sd.values())
    opt_state = {"state": {i: {"step": torch.tensor(500.0), "exp_avg": torch.zeros_like(p),
                               "exp_avg_sq": torch.zeros_like(p)} for i, p in enumerate(params)},
                 "param_groups": [{"lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 1e-4,
                                   "amsgrad": False, "params": list(range(len(params)))}]}
    ckpt = {"step": 500, "epoch": 3, "model_state_dict": sd, "optimizer_state_dict": opt_state,
            "config": cfg_dict, "metrics": {"val/loss": 0.123, "train/loss": 0.2},
            "finance_metadata": {"n_assets": 5, "embedding_dim": 4, "tickers": ["A0", "A1", "A2", "A3", "A4"]}}
    torch.save(ckpt, path)


def _specs_equal(a, b):
    assert a.kind == b.kind and a.norm_fn == b.norm_fn and a.enc_act == b.enc_act
    assert torch.equal(a.kmat, b.kmat)
    for (Wa, ba), (Wb, bb) in zip(a.encoder + a.decoder, b.encoder + b.decoder):
        assert torch.equal(Wa, Wb) and ((ba is None and bb is None) or torch.equal(ba, bb))


def test_checkpoint_loads_weights_only_and_matches_state_dict(tmp_path):
    g, meta, sd = _golden()
    p = tmp_path / "checkpoint.pt"
    _write_checkpoint(p, sd, meta["config"])
    ckpt = torch.load(p, map_location="cpu", weights_only=True)        # nothing executed from the file
    assert set(ckpt) >= {"model_state_dict", "config", "optimizer_state_dict"}
    _specs_equal(KoopmanModelSpec.from_checkpoint(ckpt), KoopmanModelSpec.from_state_dict(sd, meta["config"]))


@pytest.mark.gpu
def test_strategy_from_checkpoint_matches_state_dict_bit_for_bit(tmp_path):
    from test_backtest_cpu import GoldenEnv
    g, meta, sd = _golden()
    p = tmp_path / "checkpoint.pt"
    _write_checkpoint(p, sd, meta["config"])
    ckpt = torch.load(p, map_location="cpu", weights_only=True)
    cfg = MPCConfig(**meta["mpc"])
    env = GoldenEnv(g)
    a = KoopmanMPCStrategy(ckpt, cfg)
    b = KoopmanMPCStrategy(KoopmanModelSpec.from_state_dict(sd, meta["config"]), cfg)
    ts = list(range(0, 40, 3))
    wp = np.tile(np.ones(5) / 5, (len(ts), 1))
    Wa, sa, va = a.rebalance_batch(ts, wp, env, return_info=True)
    Wb, sb, vb = b.rebalance_batch(ts, wp, env, return_info=True)
    assert np.array_equal(Wa, Wb) and np.array_equal(sa, sb) and np.array_equal(va, vb, equal_nan=True)
    assert np.array_equal(a.rebalance(7, np.ones(5) / 5, env), b.rebalance(7, np.ones(5) / 5, env))
