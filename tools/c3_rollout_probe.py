"""Dev probe: three C3 rollouts (65,536 windows, obs 2000, enc [1024,1024], latent 256, H = 10) for a kernel trace."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman, KoopmanModelSpec
dev = torch.device("cuda", 0)
N, L, H = 100, 256, 10
obs = N * 20
km = DeviceKoopman(KoopmanModelSpec.from_state_dict(bench.make_state_dict(obs, L, 1024, seed=0), bench.MODEL_CFG), dev)
x, wp = bench.window_inputs(0, 65536, N, obs, seed=0, device=dev)
m = torch.full((N,), 5e-4, device=dev); s = torch.full((N,), 0.015, device=dev)
for _ in range(3):
    y = km.rollout(x, m, s, H, N)
torch.cuda.synchronize()
print("ok")
