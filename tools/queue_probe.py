"""Dev probe: do two torch streams run kernels concurrently? (HIP maps streams onto the process's
GPU_MAX_HW_QUEUES hardware queues; two streams on one queue serialise.) For pairs of streams from
torch's pool, time two single-window C3 solves (one workgroup each, ~0.7 ms) launched on the two
streams: ~1x one solve = concurrent, ~2x = serialised.   python tools/queue_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility_batched

dev = torch.device("cuda", 0)
N, H = 100, 10
rng = np.random.default_rng(0)
wp = torch.tensor(rng.dirichlet(np.ones(N), 1), device=dev)
y = torch.tensor(rng.normal(5e-4, 0.015, (1, H, N)).astype(np.float32), device=dev)
cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, precision="f64")


def run(streams, reps=20):
    for _ in range(2):
        for s in streams:
            with torch.cuda.stream(s):
                solve_mpc_log_utility_batched(wp, y, cfg)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        for s in streams:
            with torch.cuda.stream(s):
                solve_mpc_log_utility_batched(wp, y, cfg)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


pool = [torch.cuda.Stream(dev) for _ in range(int(os.environ.get("NSTREAMS", "12")))]
hi = [torch.cuda.Stream(dev, priority=-1) for _ in range(4)]
main = torch.cuda.current_stream(dev)
one = run([pool[0]])
print(f"one solve {one:.3f} ms", flush=True)
for j in range(1, len(pool)):
    print(f"pool[0] + pool[{j}]: {run([pool[0], pool[j]]) / one:.2f}x", flush=True)
print(f"main + pool[0]: {run([main, pool[0]]) / one:.2f}x", flush=True)
print(f"pool[0..3]: {run(pool[:4]) / one:.2f}x   pool[4..7]: {run(pool[4:8]) / one:.2f}x", flush=True)
print(f"hi[0..3]: {run(hi) / one:.2f}x   pool[0..1]+hi[0..1]: {run(pool[:2] + hi[:2]) / one:.2f}x", flush=True)


def fresh_streams(n):
    """n new HIP streams (hipStreamCreateWithFlags, non-blocking) wrapped as torch ExternalStreams."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = []
    for _ in range(n):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0
        out.append(torch.cuda.ExternalStream(h.value, device=dev))
    return out


fr = fresh_streams(8)
print(f"fresh[0..3]: {run(fr[:4]) / one:.2f}x   fresh[4..7]: {run(fr[4:]) / one:.2f}x   fresh[0..7]: "
      f"{run(fr) / one:.2f}x", flush=True)
for j in range(1, 8):
    print(f"fresh[0] + fresh[{j}]: {run([fr[0], fr[j]]) / one:.2f}x", flush=True)
