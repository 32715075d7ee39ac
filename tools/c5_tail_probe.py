"""Dev probe (GPU): the large-window launch's tail at C5 (N = 500, H = 20; BASELINE configs[4]).
The secondary_c5 workload (bench's LISTAKM model, fp32 rollout, 1,024 windows; DT=bf16: the bench's bf16 rollout) solved once with
iteration counts: their distribution, the static slot schedule's makespan (slot s runs windows
s, s + slots, ... in iterations) against the mean, and the launch time at B = 256 / 512 / 768 /
1,024 / 2,048 windows (random yhat for the sizes past the workload's batch)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from koopman_mpc_portfolio_rebalancing_amd import (DeviceKoopman, KoopmanModelSpec, MPCConfig, _lib,
                                                   solve_mpc_log_utility_batched)
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
dev = torch.device("cuda")
N, L, H, B = 500, 512, 20, 1024
obs = N * 20
sd, lc = bench.make_lista_state_dict(obs, L, seed=2)
cfg_m = {"MODEL": {"MODEL_NAME": "LISTAKM", "NORM_FN": "id",
                   "ENCODER": {"LISTA": {"ALPHA": 5e-3, "L": lc, "NUM_LOOPS": 10}}}}
model = DeviceKoopman(KoopmanModelSpec.from_state_dict(sd, cfg_m), dev, dtype=os.environ.get("DT", "fp32"))
mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
x, wp = bench.make_inputs(B, N, obs, seed=200, device=dev)
cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, allow_short=False)
y = model.rollout(x, mean_d, std_d, H, N)
W, st, val, it = solve_mpc_log_utility_batched(wp, y, cfg, with_iters=True)
it = it.cpu().numpy().astype(np.int64)
print("status", np.bincount(st.cpu().numpy(), minlength=5))
print(f"iters mean {it.mean():.2f} min {it.min()} p10 {np.percentile(it, 10):.0f} p50 {np.median(it):.0f} "
      f"p90 {np.percentile(it, 90):.0f} max {it.max()}")
print("hist", dict(zip(*np.unique(it, return_counts=True))))
for slots in (256, 512, 768, 1024):
    per = np.zeros(slots, np.int64)
    for b in range(B):
        per[b % slots] += it[b]
    mk = per.max()
    print(f"static schedule, {slots} slots: makespan {mk} iterations, mean load {it.sum() / slots:.1f} "
          f"-> efficiency {it.sum() / slots / mk:.3f}")
rng = np.random.default_rng(0)


def timed(yb, wpb, reps=3):
    solve_mpc_log_utility_batched(wpb, yb, cfg)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        _, _, _, itb = solve_mpc_log_utility_batched(wpb, yb, cfg, with_iters=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best, itb.float().mean().item()


for b in (256, 512, 768, 1024):
    dt, m = timed(y[:b].contiguous(), wp[:b].contiguous())
    print(f"workload B={b}: {dt * 1e3:.2f} ms, {b / dt:.0f} win/s, mean iters {m:.2f}, "
          f"{dt * 1e3 / (m * b / min(b, 512)):.3f} ms per slot-iteration", flush=True)
y2 = torch.cat([y, y.flip(0)]).contiguous()
wp2 = torch.cat([wp, wp.flip(0)]).contiguous()
dt, m = timed(y2, wp2)
print(f"workload x2 B=2048: {dt * 1e3:.2f} ms, {2048 / dt:.0f} win/s", flush=True)
