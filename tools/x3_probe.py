"""Dev probe: the fp32 rollout GEMMs on the f32-input MFMA (dtype "fp32") against the three-bf16-plane
form (dtype "fp32", the default; "fp32_f32mfma" the f32-input MFMA): rollout time (HIP events, median of reps) and the error of each against a
float64 restatement of the same model (torch CPU, double), at BASELINE configs[1] (C2) and the C3
rollout shape. Usage: python tools/x3_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec, _lib

if os.environ.get("KMPC_DEV_LIB"):   # a variant library (csrc/Makefile tvar)
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
OBS = int(os.environ.get("OBS", "0"))   # > 0: encoder input width (OBS = 1024: both 1024-wide layers K = 1024)

dev = torch.device("cuda", 0)


def ref64(sd, x, H, N, mean, std):
    """GenericKM (relu encoder, norm id, 1-layer decoder) in float64."""
    h = x.double()
    for i, k in enumerate((0, 2, 4)):
        h = h @ sd[f"encoder.network.{k}.weight"].double().T + sd[f"encoder.network.{k}.bias"].double()
        if i < 2:
            h = torch.relu(h)
    K = sd["kmat"].double()
    D = sd["decoder.network.0.weight"].double()[:N]
    out = []
    for _ in range(H):
        h = h @ K
        out.append((h @ D.T) * std.double() + mean.double())
    return torch.stack(out, 1)


def one(name, B, N, L, H, obs, reps):
    obs = OBS or obs
    sd = bench.make_state_dict(obs, L, 1024, seed=1)
    x, _ = bench.make_inputs(B, N, obs, seed=100, device="cpu")
    mean = torch.full((N,), 5e-4)
    std = torch.full((N,), 0.015)
    nref = min(B, 4096)
    ref = ref64(sd, x[:nref], H, N, mean, std).numpy()
    scale = np.abs(ref - 5e-4).max()
    xd = x.to(dev)
    res = {}
    for dt in ("fp32_f32mfma", "fp32"):
        km = DeviceKoopman(KoopmanModelSpec.from_state_dict(sd, bench.MODEL_CFG), dev, dtype=dt)
        y = km.rollout(xd, mean.to(dev), std.to(dev), H, N)
        torch.cuda.synchronize()
        yh = y[:nref].double().cpu().numpy()
        err = np.abs(yh - ref).max() / scale
        rms = np.sqrt(((yh - ref) ** 2).mean()) / scale
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            km.rollout(xd, mean.to(dev), std.to(dev), H, N)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[dt] = y
        print(f"[{name}] {dt:7s} rollout {np.median(ts):.3f} ms (min {min(ts):.3f})  max rel err vs f64 {err:.3e}"
              f"  rms {rms:.3e}", flush=True)
    d = (res["fp32_f32mfma"] - res["fp32"]).abs().max().item() / scale
    print(f"[{name}] max |f32mfma - x3| / scale {d:.3e}", flush=True)


one("C2 configs[1]", 4096, 30, 128, 5, 600, 50)
one("C3 rollout", 65536, 100, 256, 10, 400, 10)
