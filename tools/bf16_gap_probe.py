"""Dev probe (GPU): bench.secondary_c5 once — BASELINE configs[4] with the bf16 decision gap in the
fp32-yhat program and the fp32 rollout time."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
print(json.dumps(bench.secondary_c5(torch.device("cuda", 0), 2, 1), indent=1), flush=True)
