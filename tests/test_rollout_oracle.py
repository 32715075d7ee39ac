"""The numpy rollout restatement (oracle/rollout.py) against yhat computed by the reference's own
model.py / FinanceEnv code (tests/golden/make_golden.py). CPU only."""
import glob
import json
import os

import numpy as np
import pytest

from oracle import rollout as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def spec_from_golden(g):
    """Build an oracle spec from a golden's state_dict arrays (reference key names)."""
    meta = json.loads(str(g["meta"]))
    sd = {k[2:]: g[k] for k in g.files if k.startswith("w:")}

    def stack(prefix):
        idx = sorted({int(k[len(prefix) + 1:].split(".")[0]) for k in sd if k.startswith(prefix + ".")})
        return [sd[f"{prefix}.{i}.weight"] for i in idx], [sd.get(f"{prefix}.{i}.bias") for i in idx]

    if meta["model_name"] == "LISTAKM":
        if "lista.We.weight" in sd:
            ew, eb, last = [sd["lista.We.weight"]], [None], False
        else:
            ew, eb = stack("lista.We.network")
            last = meta["enc_last_relu"]
        return meta, {"kind": "lista", "enc_w": ew, "enc_b": eb, "enc_act": meta["enc_act"],
                      "enc_last_relu": last, "kmat": sd["kmat"], "dict": sd["dict"], "lista_S": sd["lista.S"],
                      "lista_loops": meta["lista_loops"],
                      "lista_thresh": meta["lista_alpha"] / meta["lista_L"]}
    ew, eb = stack("encoder.network")
    dw, db = stack("decoder.network")
    return meta, {"kind": "generic", "enc_w": ew, "enc_b": eb, "enc_act": meta["enc_act"],
                  "enc_last_relu": meta["enc_last_relu"], "kmat": sd["kmat"], "norm_fn": meta["norm_fn"],
                  "dec_w": dw, "dec_b": db, "dec_act": meta["dec_act"]}


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "rollout_*.npz"))))
def test_rollout_restatement_matches_reference(path):
    g = np.load(path)
    meta, spec = spec_from_golden(g)
    y = R.rollout(spec, g["obs"], meta["H"], meta["N"], g["mean"].astype(np.float32), g["std"].astype(np.float32))
    ref = g["yhat"]
    scale = np.abs(ref).max()
    assert y.shape == ref.shape
    # float32 path, different summation order only
    assert np.abs(y - ref).max() <= 2e-5 * max(scale, 1e-3)


def test_embedding_restatement_matches_reference():
    """oracle standardize + time_delay_embedding == the reference's (data_finance.py:243-300, 331), bit for bit."""
    g = np.load(os.path.join(GOLD, "embedding.npz"))
    z = R.standardize(g["log_returns"], g["mean"], g["std"])
    assert np.array_equal(z, g["standardized"])
    assert np.array_equal(R.time_delay_embedding(z, int(g["emb_dim"])), g["embedded"])
