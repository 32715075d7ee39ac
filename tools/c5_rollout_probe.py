"""Dev probe: the configs[4] rollout (LISTAKM, 1,024 windows, obs 10,000, latent 512, 10 loops,
H = 20, bf16 MFMA) — event time per call, for rocprofv3 kernel traces (tools/ab_c5r.sh)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec
from koopman_mpc_portfolio_rebalancing_amd import _lib
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
dev = torch.device("cuda", 0)
B, N, L, H = int(os.environ.get("B", "1024")), 500, 512, 20
obs = N * 20
sd, lc = bench.make_lista_state_dict(obs, L, seed=2)
cfg_m = {"MODEL": {"MODEL_NAME": "LISTAKM", "NORM_FN": "id",
                   "ENCODER": {"LISTA": {"ALPHA": 5e-3, "L": lc, "NUM_LOOPS": 10}}}}
model = DeviceKoopman(KoopmanModelSpec.from_state_dict(sd, cfg_m), dev, dtype=os.environ.get("DTYPE", "bf16"))
mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
x, _ = bench.make_inputs(B, N, obs, seed=200, device=dev)
for _ in range(3):
    y = model.rollout(x, mean_d, std_d, H, N)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
e[0].record()
for _ in range(5):
    y = model.rollout(x, mean_d, std_d, H, N)
e[1].record()
torch.cuda.synchronize()
print(f"rollout {e[0].elapsed_time(e[1]) / 5:.3f} ms", flush=True)
