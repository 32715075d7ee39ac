"""Float32 numpy restatement of the reference's Koopman rollout — TEST INFRASTRUCTURE ONLY.

Follows, op for op, what ``KoopmanMPCStrategy.rebalance`` computes before the solve
(backtest.py:99-121):

    z = model.encode(obs)                       GenericKM.encode  model.py:756-766
                                                LISTAKM.encode    model.py:828-837 -> LISTA.forward 190-209
    for _ in range(H):
        z = model.step_latent(z)                GenericKM.step_latent model.py:787-797 (z @ K, norm_fn)
                                                KoopmanMachine.step_latent model.py:311-321 (LISTAKM)
        p = model.decode(z)                     GenericKM.decode model.py:768-777 / LISTAKM.decode 839-850
        y = env.extract_current_returns(p)      data_finance.py:717-729  (p[..., :N])
        y = env.destandardize_returns(y)        data_finance.py:731-742  (y * std + mean, float32)

Weights use the reference's state_dict layout (nn.Linear weight = [out, in]). The arithmetic is
float32 like the reference's torch path; only the summation order of each dot product differs.
With ``bf16=True`` every matrix-product operand is first rounded to bfloat16 (round to nearest
even) and the products accumulate in float32 — the semantics of the device's bf16 MFMA rollout
(kmpc_rollout with KMPC_DTYPE_BF16, BASELINE configs[4]); it is not a reference code path.
"""
from __future__ import annotations

import math

import numpy as np


def _act(x, name):
    if name == "relu":
        return np.maximum(x, np.float32(0))
    if name == "tanh":
        return np.tanh(x)
    if name == "gelu":  # nn.GELU() default (erf form), model.py:54
        from scipy.special import erf
        return (np.float32(0.5) * x * (np.float32(1) + erf(x / np.float32(math.sqrt(2))))).astype(np.float32)
    raise ValueError(name)


def bf16_round(x):
    """float32 -> nearest-even bfloat16, returned as float32 (v_cvt_pk_bf16_f32 semantics)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32).view(np.float32)


def _mm(a, b, bf16=False):
    """a @ b in float32, operands rounded to bf16 first when bf16."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if bf16:
        a, b = bf16_round(a), bf16_round(b)
    return (a @ b).astype(np.float32)


def mlp(x, weights, biases, activation="relu", last_relu=False, bf16=False):
    """MLPCoder.forward (model.py:67-117): Linear, act, ..., Linear (+ReLU if last_relu)."""
    h = np.asarray(x, np.float32)
    n = len(weights)
    for k, (W, b) in enumerate(zip(weights, biases)):
        h = _mm(h, np.asarray(W, np.float32).T, bf16)
        if b is not None:
            h = h + np.asarray(b, np.float32)
        if k < n - 1:
            h = _act(h, activation)
        elif last_relu:
            h = np.maximum(h, np.float32(0))
    return h.astype(np.float32)


def shrink(x, thr):
    """model.py:30-40: sign(x) * max(|x| - thr, 0)."""
    return (np.sign(x) * np.maximum(np.abs(x) - np.float32(thr), np.float32(0))).astype(np.float32)


def norm_fn(z, name):
    """GenericKM._norm_fn (model.py:740-754)."""
    if name == "id":
        return z
    if name == "ball":
        return (z / np.linalg.norm(z, axis=-1, keepdims=True)).astype(np.float32)
    raise ValueError(name)


def lista_decoder_weight(dict_param):
    """LISTAKM.decode dictionary (model.py:846-850): dict / clamp(||dict row||, 1e-4), as [obs, L]."""
    d = np.asarray(dict_param, np.float32)                      # [L, obs]
    nrm = np.maximum(np.linalg.norm(d, axis=1, keepdims=True), np.float32(1e-4))
    return (d / nrm).T.astype(np.float32)                        # Linear weight layout [obs, L]


def rollout(spec, obs, H, n_assets, mean, std, bf16=False):
    """yhat [B, H, N] float32 for observations obs [B, obs] (bf16: see the module docstring).

    spec: dict with
      kind: 'generic' | 'lista'
      enc_w, enc_b: lists (encoder MLP, or LISTA We as a 1-layer list), enc_act, enc_last_relu
      kmat [L, L]; norm_fn ('id' | 'ball', generic only)
      dec_w, dec_b, dec_act (generic MLP decoder) | dict (lista, [L, obs])
      lista_S [L, L], lista_loops, lista_thresh (= alpha / L)
    """
    x = np.asarray(obs, np.float32)
    mean = np.asarray(mean, np.float32)
    std = np.asarray(std, np.float32)
    K = np.asarray(spec["kmat"], np.float32)
    if spec["kind"] == "generic":
        z = norm_fn(mlp(x, spec["enc_w"], spec["enc_b"], spec.get("enc_act", "relu"),
                        spec.get("enc_last_relu", False), bf16), spec.get("norm_fn", "id"))
    else:
        c = mlp(x, spec["enc_w"], spec["enc_b"], spec.get("enc_act", "relu"), spec.get("enc_last_relu", False),
                bf16)
        z = shrink(c, spec["lista_thresh"])
        S = np.asarray(spec["lista_S"], np.float32)
        for _ in range(int(spec["lista_loops"])):
            z = shrink(_mm(z, S, bf16) + c, spec["lista_thresh"])
    out = np.empty((x.shape[0], H, n_assets), np.float32)
    for k in range(H):
        z = _mm(z, K, bf16)
        if spec["kind"] == "generic":
            z = norm_fn(z, spec.get("norm_fn", "id"))
            p = mlp(z, spec["dec_w"], spec["dec_b"], spec.get("dec_act", "relu"), False, bf16)
        else:
            p = _mm(z, lista_decoder_weight(spec["dict"]).T, bf16)
        out[:, k, :] = p[:, :n_assets] * std + mean
    return out


def standardize(log_returns, mean, std):
    """data_finance.py:243-260 then .astype(np.float32) (data_finance.py:331): float64 arithmetic,
    one cast to float32."""
    y = np.asarray(log_returns, np.float64)
    return ((y - np.asarray(mean, np.float64)) / np.asarray(std, np.float64)).astype(np.float32)


def time_delay_embedding(data, embedding_dim):
    """data_finance.py:262-300: row i = [y_{i+d-1}, y_{i+d-2}, ..., y_i] (most recent first)."""
    data = np.asarray(data)
    T, n = data.shape
    if T < embedding_dim:
        raise ValueError("series shorter than the embedding")
    rows = T - embedding_dim + 1
    out = np.empty((rows, embedding_dim * n), data.dtype)
    for j in range(embedding_dim):
        out[:, j * n:(j + 1) * n] = data[embedding_dim - 1 - j: embedding_dim - 1 - j + rows]
    return out
