"""Dev probe: BASELINE configs[1] (C2: 4096 windows, N=30, latent 128, H=5, c=tau=0) step time,
eager launches vs one captured HIP graph replay (torch.cuda.CUDAGraph over the ctypes launches)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec, MPCConfig, solve_mpc_log_utility_batched
from koopman_mpc_portfolio_rebalancing_amd import _lib
if os.environ.get("KMPC_DEV_LIB"):   # a variant library (csrc/Makefile tvar)
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))

dev = torch.device("cuda", 0)
B, N, L, H, hidden = (int(os.environ.get("B", "4096")), int(os.environ.get("N", "30")), int(os.environ.get("LAT", "128")),
                      int(os.environ.get("H", "5")), 1024)
obs = N * 20
model = DeviceKoopman(KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs, L, hidden, seed=1), bench.MODEL_CFG), dev)
mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
x, wp = bench.make_inputs(B, N, obs, seed=100, device=dev)
cfg = MPCConfig(horizon=H, cost_coeff=0.0, max_turnover=0.0, allow_short=False)

def step():
    y = model.rollout(x, mean_d, std_d, H, N)
    return y, solve_mpc_log_utility_batched(wp, y, cfg)

for _ in range(3):
    step()
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
e[0].record(); y = model.rollout(x, mean_d, std_d, H, N); e[1].record(); solve_mpc_log_utility_batched(wp, y, cfg); e[2].record()
torch.cuda.synchronize()
import hashlib
print("yhat sha1", hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
print(f"eager kernels: rollout {e[0].elapsed_time(e[1]):.3f} ms, solve {e[1].elapsed_time(e[2]):.3f} ms", flush=True)
reps = 200
t0 = time.perf_counter()
for _ in range(reps):
    y, (W0, st, val) = step()
torch.cuda.synchronize()
te = (time.perf_counter() - t0) / reps
print(f"eager step {te*1e3:.3f} ms -> {B/te:.0f} windows/s", flush=True)
Wref = W0.clone()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    yg, (Wg, stg, valg) = step()
g.replay(); torch.cuda.synchronize()
print("graph W0 == eager W0:", bool(torch.equal(Wg, Wref)), flush=True)
t0 = time.perf_counter()
for _ in range(reps):
    g.replay()
torch.cuda.synchronize()
tg = (time.perf_counter() - t0) / reps
print(f"graph step {tg*1e3:.3f} ms -> {B/tg:.0f} windows/s", flush=True)
