"""Koopman model inference subset on the device (the rollout half of the window hot path).

Mirrors what ``KoopmanMPCStrategy.rebalance`` uses of the reference model (backtest.py:99-121):
``encode`` (GenericKM model.py:756-766 / LISTAKM model.py:828-837), ``step_latent``
(model.py:311-321, 787-797), ``decode`` (model.py:768-777, 839-850), then the env's
``extract_current_returns`` (first N outputs, data_finance.py:729) and ``destandardize_returns``
(data_finance.py:740-742). Weights are read from the reference's ``state_dict`` layout (the
checkpoint written by train.py:475-491), or from a live reference model object.

All per-window arithmetic runs in libkmpc.so (fp32 MFMA GEMMs + fused epilogues); this module only
arranges weight pointers (and, once per model, normalises the LISTA dictionary).
"""
from __future__ import annotations

import ctypes
import re
from dataclasses import dataclass, field
from typing import Any, List, Optional, Tuple

import numpy as np
import torch

from . import _lib


def _cfg_get(cfg: Any, *path, default=None):
    """Read cfg.MODEL.ENCODER.LAYERS style paths from a Config object or its to_dict()."""
    cur = cfg
    for key in path:
        if cur is None:
            return default
        if isinstance(cur, dict):
            cur = cur.get(key, None)
        else:
            cur = getattr(cur, key, None)
    return default if cur is None else cur


def _linear_stack(sd: dict, prefix: str) -> List[Tuple[torch.Tensor, Optional[torch.Tensor]]]:
    """Collect nn.Sequential Linear layers '<prefix>.<idx>.weight/bias' in index order."""
    pat = re.compile(re.escape(prefix) + r"\.(\d+)\.weight$")
    idx = sorted(int(m.group(1)) for k in sd for m in [pat.match(k)] if m)
    return [(sd[f"{prefix}.{i}.weight"], sd.get(f"{prefix}.{i}.bias")) for i in idx]


@dataclass
class KoopmanModelSpec:
    """Inference description of a reference KoopmanMachine (weights as float32 tensors)."""
    kind: str                                   # 'generic' (GenericKM / SparseKM) | 'lista' (LISTAKM)
    encoder: List[Tuple[torch.Tensor, Optional[torch.Tensor]]]
    kmat: torch.Tensor
    decoder: List[Tuple[torch.Tensor, Optional[torch.Tensor]]]
    enc_act: str = "relu"
    enc_last_relu: bool = False
    dec_act: str = "relu"
    norm_fn: str = "id"
    lista_S: Optional[torch.Tensor] = None
    lista_loops: int = 0
    lista_thresh: float = 0.0

    @property
    def fuse_latent(self) -> bool:
        return self.latent_form != "unfused"

    @fuse_latent.setter
    def fuse_latent(self, v: bool) -> None:
        self.latent_form = "auto" if v else "unfused"

    @property
    def latent(self) -> int:
        return int(self.kmat.shape[0])

    @property
    def obs_size(self) -> int:
        return int(self.encoder[0][0].shape[1])

    @classmethod
    def from_state_dict(cls, sd: dict, cfg: Any) -> "KoopmanModelSpec":
        """sd: model_state_dict (train.py:478); cfg: Config or checkpoint['config'] dict."""
        sd = {k: (v if torch.is_tensor(v) else torch.as_tensor(np.asarray(v))) for k, v in sd.items()}
        name = _cfg_get(cfg, "MODEL", "MODEL_NAME", default="GenericKM")
        enc_act = _cfg_get(cfg, "MODEL", "ENCODER", "ACTIVATION", default="relu")
        enc_last_relu = bool(_cfg_get(cfg, "MODEL", "ENCODER", "LAST_RELU", default=False))
        if name == "LISTAKM":
            alpha = float(_cfg_get(cfg, "MODEL", "ENCODER", "LISTA", "ALPHA"))
            L = float(_cfg_get(cfg, "MODEL", "ENCODER", "LISTA", "L"))
            loops = int(_cfg_get(cfg, "MODEL", "ENCODER", "LISTA", "NUM_LOOPS"))
            if "lista.We.weight" in sd:          # LINEAR_ENCODER=True: nn.Linear(bias=False)
                enc = [(sd["lista.We.weight"], None)]
                enc_last = False
            else:
                enc = _linear_stack(sd, "lista.We.network")
                enc_last = enc_last_relu
            d = sd["dict"].float()                                      # [L, obs]
            wd = d / torch.linalg.norm(d, dim=1, keepdim=True).clamp(min=1e-4)   # model.py:846-850
            return cls(kind="lista", encoder=enc, kmat=sd["kmat"], decoder=[(wd.t().contiguous(), None)],
                       enc_act=enc_act, enc_last_relu=enc_last, lista_S=sd["lista.S"],
                       lista_loops=loops, lista_thresh=alpha / L)
        if name not in ("GenericKM", "SparseKM"):
            raise ValueError(f"unknown MODEL_NAME {name!r}")
        return cls(kind="generic", encoder=_linear_stack(sd, "encoder.network"), kmat=sd["kmat"],
                   decoder=_linear_stack(sd, "decoder.network"), enc_act=enc_act,
                   enc_last_relu=enc_last_relu,
                   dec_act=_cfg_get(cfg, "MODEL", "DECODER", "ACTIVATION", default="relu"),
                   norm_fn=_cfg_get(cfg, "MODEL", "NORM_FN", default="id"))

    @classmethod
    def from_model(cls, model: Any) -> "KoopmanModelSpec":
        """From a live reference KoopmanMachine (uses model.cfg + model.state_dict())."""
        return cls.from_state_dict(model.state_dict(), model.cfg)

    @classmethod
    def from_checkpoint(cls, checkpoint: dict) -> "KoopmanModelSpec":
        """From a train.py checkpoint dict: {'model_state_dict', 'config', ...} (train.py:475-491)."""
        return cls.from_state_dict(checkpoint["model_state_dict"], checkpoint["config"])


class DeviceKoopman:
    """A KoopmanModelSpec resident on one device, evaluated through kmpc_rollout / kmpc_window."""

    def __init__(self, spec: KoopmanModelSpec, device: Optional[torch.device] = None, dtype: str = "fp32",
                 fuse_latent: bool = True, latent_form: str = "auto"):
        """dtype: 'fp32' (the reference's arithmetic, default: GEMMs on the bf16 MFMA with every fp32
        operand split exactly into three bf16 planes — an fp32 GEMM in accuracy), 'fp32_f32mfma' (the
        same arithmetic on the f32-input MFMA) or 'bf16' (GEMM operands rounded to bf16 on the bf16
        MFMA, fp32 accumulation — BASELINE configs[4]). latent_form (kmpc_rollout_desc.latent_unfused)
        picks how the H-step latent loop runs: 'auto' (the library's choice: the latent-powers GEMM
        from 8,192 windows where the latent step is linear, else one fused launch), 'sequential' (the
        fused step-by-step loop at every batch size: latent_steps_x3_kernel at L = 256 on three bf16
        planes, the fp32 loops otherwise) or 'unfused' (one GEMM launch per step); fuse_latent=False
        is 'unfused'. All three are the same fp32 arithmetic up to summation order (A/B and tests)."""
        if latent_form not in _lib.LATENT_FORM:
            raise ValueError(f"latent_form must be one of {sorted(_lib.LATENT_FORM)}")
        self.latent_form = latent_form if fuse_latent else "unfused"
        if dtype not in _lib.DTYPE:
            raise ValueError(f"dtype must be one of {sorted(_lib.DTYPE)}")
        self.dtype = dtype
        if device is None:
            if not torch.cuda.is_available():
                raise _lib.KmpcError("DeviceKoopman needs a GPU (libkmpc.so has no CPU path)")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.KmpcError("DeviceKoopman needs a HIP device")
        self.spec = spec

        def up(t):
            return None if t is None else t.detach().to(self.device, torch.float32).contiguous()

        self.enc = [(up(W), up(b)) for W, b in spec.encoder]
        self.dec = [(up(W), up(b)) for W, b in spec.decoder]
        self.kmat = up(spec.kmat)
        self.S = up(spec.lista_S)
        if len(self.enc) > _lib.KMPC_MAX_LAYERS or len(self.dec) > _lib.KMPC_MAX_LAYERS:
            raise _lib.KmpcError("too many layers for kmpc_mlp")

    @property
    def fuse_latent(self) -> bool:
        return self.latent_form != "unfused"

    @fuse_latent.setter
    def fuse_latent(self, v: bool) -> None:
        self.latent_form = "auto" if v else "unfused"

    @property
    def latent(self) -> int:
        return self.spec.latent

    @property
    def obs_size(self) -> int:
        return self.spec.obs_size

    def _mlp(self, layers, act, last_relu) -> _lib.Mlp:
        m = _lib.Mlp()
        m.n_layers = len(layers)
        m.dims[0] = int(layers[0][0].shape[1])
        for k, (W, b) in enumerate(layers):
            m.dims[k + 1] = int(W.shape[0])
            m.weight[k] = W.data_ptr()
            m.bias[k] = b.data_ptr() if b is not None else None
        m.act = _lib.ACT[act]
        m.last_relu = int(bool(last_relu))
        return m

    def rollout_desc(self, B: int, H: int, N: int, mean: torch.Tensor, std: torch.Tensor,
                     enc=None, obs_ld: int = 0) -> _lib.RolloutDesc:
        d = _lib.RolloutDesc()
        d.B, d.N, d.H, d.L, d.obs = int(B), int(N), int(H), self.latent, self.obs_size
        s = self.spec
        d.model_kind = _lib.MODEL_LISTA if s.kind == "lista" else _lib.MODEL_GENERIC
        d.norm_fn = _lib.NORM[s.norm_fn]
        d.encoder = self._mlp(enc if enc is not None else self.enc, s.enc_act, s.enc_last_relu)
        d.obs_ld = int(obs_ld)
        d.dtype = _lib.DTYPE[self.dtype]
        d.latent_unfused = _lib.LATENT_FORM[self.latent_form]
        d.lista_S = self.S.data_ptr() if self.S is not None else None
        d.lista_loops = int(s.lista_loops)
        d.lista_thresh = float(s.lista_thresh)
        d.kmat = self.kmat.data_ptr()
        d.decoder = self._mlp(self.dec, s.dec_act, False)
        d.mean = mean.data_ptr()
        d.std = std.data_ptr()
        return d

    def _workspace(self, nbytes: int) -> torch.Tensor:
        """Scratch for one call from torch's caching allocator on the current stream (reused in
        stream order once dropped; nothing is held between calls)."""
        return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)

    def _check_obs(self, x: torch.Tensor) -> None:
        if x.dim() != 2 or x.shape[1] != self.obs_size:
            raise ValueError(f"obs must be [B, {self.obs_size}], got {tuple(x.shape)}")

    def _stats(self, mean, std, N):
        m = torch.as_tensor(mean, dtype=torch.float32, device=self.device).reshape(-1)[:N].contiguous()
        s = torch.as_tensor(std, dtype=torch.float32, device=self.device).reshape(-1)[:N].contiguous()
        return m, s

    def rollout(self, obs: torch.Tensor, mean, std, horizon: int, n_assets: int) -> torch.Tensor:
        """yhat [B, H, N] float32 (predicted de-standardized log-returns) for obs [B, obs_size]."""
        _lib.require_gpu(obs)
        x = obs.to(self.device, torch.float32).contiguous()
        self._check_obs(x)
        B = x.shape[0]
        m, s = self._stats(mean, std, n_assets)
        y = torch.empty((B, horizon, n_assets), dtype=torch.float32, device=self.device)
        d = self.rollout_desc(B, horizon, n_assets, m, s)
        L = _lib.load()
        nbytes = L.kmpc_workspace_bytes(ctypes.byref(d), None)
        ws = self._workspace(nbytes)
        with torch.cuda.device(self.device):
            rc = L.kmpc_rollout(ctypes.byref(d), x.data_ptr(), y.data_ptr(), ws.data_ptr(), nbytes,
                                _lib.stream_handle(self.device))
        _lib.check(rc)
        return y

    # -- panel mode: the time-delay embedding read in place from a standardized [T, N] panel --
    def _panel_encoder(self, emb_dim: int, n_assets: int):
        """First encoder layer with its lag blocks reversed (oldest lag first), so that window i
        of the embedded matrix (data_finance.py:262-300: [y_t, y_{t-1}, ..., y_{t-d+1}]) is the
        contiguous panel slice rows i .. i+d-1 (cached per (d, N))."""
        key = (int(emb_dim), int(n_assets))
        if getattr(self, "_panel", None) is None:
            self._panel = {}
        if key not in self._panel:
            W0, b0 = self.enc[0]
            if W0.shape[1] != emb_dim * n_assets:
                raise ValueError(f"encoder input {W0.shape[1]} != emb_dim * n_assets = {emb_dim * n_assets}")
            Wr = W0.reshape(W0.shape[0], emb_dim, n_assets).flip(1).reshape(W0.shape[0], -1).contiguous()
            self._panel[key] = [(Wr, b0)] + list(self.enc[1:])
        return self._panel[key]

    def rollout_panel(self, z: torch.Tensor, emb_dim: int, first: int, n_windows: int, mean, std,
                      horizon: int, n_assets: int) -> torch.Tensor:
        """yhat [n_windows, H, N] for embedded windows first .. first+n_windows-1 of the standardized
        return panel z [T, N] float32 (kmpc_standardize), without materialising the embedding."""
        _lib.require_gpu(z)
        z = z.to(self.device, torch.float32).contiguous()
        T, N = z.shape
        if N != n_assets or first < 0 or first + n_windows + emb_dim - 1 > T:
            raise ValueError("panel window range out of bounds")
        enc = self._panel_encoder(emb_dim, n_assets)
        m, s = self._stats(mean, std, n_assets)
        y = torch.empty((n_windows, horizon, n_assets), dtype=torch.float32, device=self.device)
        d = self.rollout_desc(n_windows, horizon, n_assets, m, s, enc=enc, obs_ld=N)
        L = _lib.load()
        nbytes = L.kmpc_workspace_bytes(ctypes.byref(d), None)
        ws = self._workspace(nbytes)
        with torch.cuda.device(self.device):
            rc = L.kmpc_rollout(ctypes.byref(d), z[first].data_ptr(), y.data_ptr(), ws.data_ptr(), nbytes,
                                _lib.stream_handle(self.device))
        _lib.check(rc)
        return y

    def window(self, obs: torch.Tensor, w_prev: torch.Tensor, mean, std, n_assets: int, mpc_config,
               keep_yhat: bool = False, return_full: bool = False, with_iters: bool = False):
        """Fused window (kmpc_window): obs [B, obs], w_prev [B, N] -> (W0 or W, status, value[, yhat]
        [, iters]) — iters [B] int32 interior-point iterations when with_iters."""
        from .mpc import _solve_desc
        _lib.require_gpu(obs)
        x = obs.to(self.device, torch.float32).contiguous()
        self._check_obs(x)
        B = x.shape[0]
        H = int(mpc_config.horizon)
        wp = w_prev.to(self.device, torch.float64).contiguous()
        if wp.shape != (B, int(n_assets)):
            raise ValueError(f"w_prev must be [{B}, {int(n_assets)}], got {tuple(wp.shape)}")
        if not 0 < int(n_assets) <= self.obs_size:
            raise ValueError(f"n_assets {n_assets} must be in 1..obs_size ({self.obs_size})")
        m, s = self._stats(mean, std, n_assets)
        rd = self.rollout_desc(B, H, n_assets, m, s)
        sd = _solve_desc(B, n_assets, H, mpc_config, return_full)
        L = _lib.load()
        nbytes = L.kmpc_workspace_bytes(ctypes.byref(rd), ctypes.byref(sd))
        ws = self._workspace(nbytes)
        y = torch.empty((B, H, n_assets), dtype=torch.float32, device=self.device) if keep_yhat else None
        W = torch.empty((B, H, n_assets) if return_full else (B, n_assets), dtype=torch.float64, device=self.device)
        status = torch.empty(B, dtype=torch.int32, device=self.device)
        value = torch.empty(B, dtype=torch.float64, device=self.device)
        iters = torch.empty(B, dtype=torch.int32, device=self.device) if with_iters else None
        with torch.cuda.device(self.device):
            rc = L.kmpc_window(ctypes.byref(rd), ctypes.byref(sd), x.data_ptr(), wp.data_ptr(),
                               y.data_ptr() if y is not None else None, W.data_ptr(), status.data_ptr(),
                               value.data_ptr(), iters.data_ptr() if iters is not None else None,
                               ws.data_ptr(), nbytes, _lib.stream_handle(self.device))
        _lib.check(rc)
        out = (W, status, value) + ((y,) if keep_yhat else ()) + ((iters,) if with_iters else ())
        return out


def standardize_panel(log_returns, mean, std, device=None) -> torch.Tensor:
    """z [T, N] float32 = ((y - mean) / std) in float64, cast once — the reference's
    standardize_returns + .astype(np.float32) (data_finance.py:243-260, 331) — on the device."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    y = torch.as_tensor(log_returns, dtype=torch.float64).to(dev).contiguous()
    m = torch.as_tensor(np.asarray(mean, np.float64)).to(dev).contiguous()
    s = torch.as_tensor(np.asarray(std, np.float64)).to(dev).contiguous()
    T, N = y.shape
    z = torch.empty((T, N), dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().kmpc_standardize(T, N, y.data_ptr(), m.data_ptr(), s.data_ptr(), z.data_ptr(),
                                                _lib.stream_handle(dev)))
    return z
