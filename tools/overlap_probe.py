"""Dev probe (GPU): can the next chunk's rollout run under the current chunk's solve? The C3 step
(65,536 windows) as rollout -> solve on one stream, against K chunks with chunk k+1's rollout on a
second stream while chunk k solves (torch streams + events around the C-ABI calls)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec, MPCConfig, solve_mpc_log_utility_batched

dev = torch.device("cuda", 0)
B, N, L, H = 65536, 100, 256, 10
obs = N * 20
model = DeviceKoopman(KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs, L, 1024, seed=0), bench.MODEL_CFG), dev)
x, wp = bench.window_inputs(0, B, N, obs, seed=0, device=dev)
mean = torch.full((N,), 5e-4, device=dev)
std = torch.full((N,), 0.015, device=dev)
cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def fused():
    return model.window(x, wp, mean, std, N, cfg)[0]


def pipelined(K):
    step = B // K
    out = []
    ys = [None] * K
    evs = [torch.cuda.Event() for _ in range(K)]
    with torch.cuda.stream(s2):
        for k in range(K):
            ys[k] = model.rollout(x[k * step:(k + 1) * step], mean, std, H, N)
            evs[k].record(s2)
    with torch.cuda.stream(s1):
        for k in range(K):
            s1.wait_event(evs[k])
            out.append(solve_mpc_log_utility_batched(wp[k * step:(k + 1) * step], ys[k], cfg)[0])
    torch.cuda.current_stream().wait_stream(s1)
    return torch.cat(out)


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, r


t0, W0 = timeit(fused)
print(f"fused: {t0:.2f} ms", flush=True)
for K in (2, 4, 8):
    t, W = timeit(lambda: pipelined(K))
    print(f"pipelined K={K}: {t:.2f} ms ({(t0 - t) / t0 * 100:+.1f}%), equal {torch.equal(W, W0)}", flush=True)
