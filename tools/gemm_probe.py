"""Dev probe: the configs[1] rollout (4096 windows, N=30, obs 600, encoder [1024,1024], latent 128,
H=5) run REPS times — a short program for rocprofv3 PMC passes over the encoder GEMMs."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec
from koopman_mpc_portfolio_rebalancing_amd import _lib
if os.environ.get("KMPC_DEV_LIB"):
    _lib._lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["KMPC_DEV_LIB"]))
dev = torch.device("cuda", 0)
B, N, L, H, hidden = int(os.environ.get("B", "4096")), 30, 128, 5, 1024
obs = N * 20
model = DeviceKoopman(KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs, L, hidden, seed=1), bench.MODEL_CFG), dev)
mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
x, _ = bench.make_inputs(B, N, obs, seed=100, device=dev)
for _ in range(int(os.environ.get("REPS", "3"))):
    y = model.rollout(x, mean_d, std_d, H, N)
torch.cuda.synchronize()
print("ok", float(y.abs().sum()))
