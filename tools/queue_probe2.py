"""Dev probe: queue sharing of HIP streams created back to back in a process that never touches
torch's stream pool (the lock-step path groups' situation). Four single-window solves on four
streams: ~1x one solve = four queues, ~2x = two of them share one.   python tools/queue_probe2.py"""
import ctypes
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
hip = ctypes.CDLL("libamdhip64.so")
fr = []
for _ in range(8):
    h = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0
    fr.append(torch.cuda.ExternalStream(h.value, device=dev))


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


one = run([fr[0]])
main = torch.cuda.current_stream(dev)
print(f"one solve {one:.3f} ms", flush=True)
for sel in ([0, 1, 2, 3], [1, 2, 3, 4], [0, 1, 2], [0, 1, 2, 4], [4, 5, 6, 7]):
    print(f"fresh{sel}: {run([fr[i] for i in sel]) / one:.2f}x", flush=True)
for j in range(8):
    print(f"main + fresh[{j}]: {run([main, fr[j]]) / one:.2f}x", flush=True)
