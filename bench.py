#!/usr/bin/env python3
"""Benchmark: MPC window-solves/sec (BASELINE.json metric) on the C3 workload.

One *window* is one ``KoopmanMPCStrategy.rebalance`` equivalent (reference backtest.py:80-131):
obs_t [obs] and w_prev [N] -> Koopman rollout yhat [H, N] -> log-utility MPC solve -> W[0].
One *step* is one pass of that path over the rank's whole batch of synthetic windows, with all
inputs resident in HBM before the timed region starts:

    W0, status, value = DeviceKoopman.window(obs, w_prev)   (kmpc_window: the fp32 MFMA rollout
                        chain, then the interior-point solve — float32 phase + float64 finish —
                        on one stream; the path KoopmanMPCStrategy.rebalance_batch runs)
    [N > 1] dist.gather(W0 -> rank 0)              (the one RCCL collective)

After the timed region the same step runs once more per timed step as two C-ABI calls
(kmpc_rollout, kmpc_solve) so that HIP events bracket the solve alone (the dominant kernels) for
the roofline figure; the line carries both (timed_path, kernels.two_call_ms_per_step).

Workload. N = 1: BASELINE configs[2], 65536 windows, N = 100 assets, latent
L = 256, H = 10, obs = N * 20 = 2000, the finance_sparse GenericKM layout (encoder
Linear(2000,1024)-ReLU-Linear(1024,1024)-ReLU-Linear(1024,256), norm 'id', linear decoder without
bias), K = random orthogonal x 0.95, MPC cost 1e-3, max_turnover 0.2, no short. N > 1: BASELINE
configs[3] (C4), 2^20 windows of the same model per step, rank r taking the contiguous block
window_range(2^20, N, r) — strong scaling, one RCCL gather of W0 to rank 0. Weights and inputs are
synthetic and seeded; every window's (obs, w_prev) is a function of its index in ONE global stream
(window_inputs), so the N = 1 batch is the first 65536 windows of the C4 stream and a window's
inputs (and result) do not depend on the GPU count.

Usage: python bench.py [--gpus N --steps K --warmup W]; for N > 1 launch under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MPC window-solves/sec (batched backtest) at 1/2/4/8 MI355X vs host-CPU ref"
HBM_PEAK = 8.0e12          # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK = 157.3e12  # FLOP/s, dense fp32 MFMA (v_mfma_f32_32x32x2_f32)
BF16_MFMA_PEAK = 2.5e15    # FLOP/s, dense bf16 MFMA (v_mfma_f32_32x32x16_bf16)
F64_VALU_PEAK = 78.6e12    # FLOP/s, f64 vector (MI355X spec)
# per-window PMC figures of the solve kernel (tools/pmc_json.py over tools/gpu_round.sh's passes)
PMC_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_solve_pmc.json")


def solve_flop_model(N: int, H: int) -> dict:
    """Algorithmic f64 FLOPs of ONE interior-point iteration of the register solve (DESIGN §3.2,
    "FLOP model"), for one window of N assets and H periods: the arithmetic the algorithm needs in
    exact arithmetic, counted once per active (asset, period), a division or reciprocal as 1 flop,
    a multiply-add as 2. Not counted: padding lanes, recomputation, iterative refinement (zero in
    exact arithmetic), reduction trees beyond one add per summand. Per-phase terms:

      residuals      22 / (asset, period): R.w, budget and cap sums, both dual rows, x.l
      factor         26 / (asset, period): slack reciprocals, P, E, the tridiagonal LDL^T of Q,
                     diag(Q^-1), the Schur generators alpha_t, eps_t
      Gram           per asset: the 3H(3H+1)/2 entries of G, 2 flops each (one product of the
                     semiseparable generators + its accumulation), and the Q^-1 columns
                     (H(H+1)/2 products + H(H-1) differences for the v-type generators)
      Schur LDL^T    (3H)^3 / 3 per window
      Newton         2 solves x 48 / (asset, period) (right-hand side 10, s-elimination 7, two
                     tridiagonal solves 10, Z^T x 7, Z q 6, direction + s back-substitution 8),
                     plus 2 x 2 (3H)^2 per window for the triangular solves with L
      step length    2 passes x 45 / (asset, period): dual directions 11, ratio tests 12,
                     complementarity polynomial 21, m.dw 1
      targets        20 / (asset, period): the corrector's x.l + dx.dl - sigma mu
      update         21 / (asset, period): dual directions + five axpys
    """
    K = 3 * H
    ap = N * H
    per_ap = {"residuals": 22, "factor": 26, "newton": 2 * 48, "step_length": 2 * 45, "targets": 20, "update": 21}
    phases = {k: v * ap for k, v in per_ap.items()}
    phases["gram"] = N * (2 * K * (K + 1) // 2 + H * (H + 1) // 2 + H * (H - 1))
    phases["schur_ldlt"] = K ** 3 // 3
    phases["newton"] += 2 * 2 * K * K
    return {"per_iteration": sum(phases.values()), "phases": phases}


LATPOW_MINB = 8192   # KMPC_LATPOW_MINB (kmpc_rollout.hip): the latent-powers GEMM from this many windows


def best_f64_peak():
    """The best f64 FMA rate tools/dev/f64_peak measured on MI355X in any round's profiles/*_f64_peak.txt
    (independent v_fma_f64 chains on every CU; the 78.6 TF spec figure is not reached by it)."""
    import glob
    best, src = 0.0, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_f64_peak.txt"))):
        import re
        for v in re.findall(r"f64 fma: .*?([\d.]+) TFLOP/s", open(f).read()):
            if float(v) * 1e12 > best:
                best, src = float(v) * 1e12, os.path.relpath(f, ROOT)
    return best, (f"measured: tools/dev/f64_peak, the best run in profiles/ ({src})" if src else None)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--windows", type=int, default=65536, help="windows per step at N = 1 (configs[2])")
    p.add_argument("--global-windows", type=int, default=0,
                   help="windows per step over all ranks (default: --windows at N = 1, 2^20 = configs[3] at N > 1)")
    p.add_argument("--assets", type=int, default=100)
    p.add_argument("--latent", type=int, default=256)
    p.add_argument("--horizon", type=int, default=10)
    p.add_argument("--emb", type=int, default=20)
    p.add_argument("--hidden", type=int, default=1024)
    p.add_argument("--cpu-seconds", type=float, default=20.0,
                   help="approximate CPU-baseline budget (0 disables the cpu_baseline leg)")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="process-group backend for N > 1 (nccl = RCCL over xGMI, the default; gloo moves "
                        "the W0 gather and the timing collectives through host copies)")
    p.add_argument("--share-device", action="store_true",
                   help="every rank uses cuda:0 (a readiness check of the sharded path on a one-GPU box, "
                        "with --backend gloo: not a scaling figure)")
    p.add_argument("--headline-only", action="store_true",
                   help="skip the secondary configurations and the CPU baselines")
    p.add_argument("--dump-w0", default="",
                   help="rank 0 saves the (gathered) W0 of the last timed step to this .npy file")
    return p.parse_args()


def make_state_dict(obs: int, L: int, hidden: int, seed: int = 0) -> dict:
    """finance_sparse GenericKM state_dict layout (config.py:438-467, model.py:701-797)."""
    g = torch.Generator().manual_seed(seed)

    def linear(n_out, n_in, bias=True):
        bound = 1.0 / np.sqrt(n_in)      # nn.Linear default init range
        W = (torch.rand(n_out, n_in, generator=g) * 2 - 1) * bound
        b = (torch.rand(n_out, generator=g) * 2 - 1) * bound if bias else None
        return W, b

    sd = {}
    dims = [obs, hidden, hidden, L]
    for k in range(3):
        W, b = linear(dims[k + 1], dims[k])
        sd[f"encoder.network.{2 * k}.weight"], sd[f"encoder.network.{2 * k}.bias"] = W, b
    sd["decoder.network.0.weight"] = linear(obs, L, bias=False)[0]
    q, _ = torch.linalg.qr(torch.randn(L, L, generator=g, dtype=torch.float64))
    sd["kmat"] = (0.95 * q).float()
    return sd


MODEL_CFG = {"MODEL": {"MODEL_NAME": "GenericKM", "NORM_FN": "id",
                       "ENCODER": {"ACTIVATION": "relu", "LAST_RELU": False},
                       "DECODER": {"ACTIVATION": "relu"}}}


def make_inputs(B: int, N: int, obs: int, seed: int, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, obs, generator=g)                                   # standardized embedding
    wp = torch.from_numpy(np.random.default_rng(seed).dirichlet(np.ones(N), B))   # seeded too
    return x.to(device), wp.to(device)


C4_GLOBAL_WINDOWS = 1 << 20   # BASELINE configs[3]
STREAM_CHUNK = 4096


def window_inputs(lo: int, hi: int, N: int, obs: int, seed: int, device):
    """Windows [lo, hi) of one global seeded stream: window i's standardized embedding
    obs_i ~ N(0, 1) and w_prev_i ~ Dirichlet(1_N) (normalised Exp(1) draws) depend only on (seed, i)
    — each 4096-window chunk c of the stream is drawn from its own generator seeded (seed, c) on
    `device` — so rank r of N generating window_range(n, N, r) holds exactly those rows of the
    single-process batch."""
    g = torch.Generator(device=device)
    xs, ws = [], []
    for c in range(lo // STREAM_CHUNK, (hi + STREAM_CHUNK - 1) // STREAM_CHUNK):
        g.manual_seed(seed * 1_000_003 + c)
        x = torch.randn(STREAM_CHUNK, obs, generator=g, device=device)
        e = -torch.log1p(-torch.rand(STREAM_CHUNK, N, generator=g, device=device, dtype=torch.float64))
        w = e / e.sum(1, keepdim=True)
        a, b = max(lo, c * STREAM_CHUNK) - c * STREAM_CHUNK, min(hi, (c + 1) * STREAM_CHUNK) - c * STREAM_CHUNK
        xs.append(x[a:b])
        ws.append(w[a:b])
    if not xs:
        return torch.empty(0, obs, device=device), torch.empty(0, N, dtype=torch.float64, device=device)
    return torch.cat(xs).contiguous(), torch.cat(ws).contiguous()


def timed_loop(step, steps: int, warmup: int, world: int, device, info: dict = None, comm_device=None):
    """The bench contract's timing: `warmup` untimed steps, then exactly `steps` steps bracketed by a
    barrier + device synchronize on both sides; the elapsed time is the MAX over ranks (all_reduce).
    step(k) runs one step (k = None for warmup) and returns its output; returns (elapsed, last).
    The warmup steps include the step's collective, so communicator setup is not timed.
    info (optional) receives this rank's own elapsed time as "local_elapsed_s". comm_device: where
    the timing collective's tensor lives (default `device`; the CPU under gloo)."""
    import torch.distributed as dist
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    out = None
    for _ in range(warmup):
        out = step(None)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        out = step(k)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if info is not None:
        info["local_elapsed_s"] = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm_device or device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def rank_provenance(windows: int, local_elapsed: float, device) -> dict:
    """What the process group itself saw, for the N > 1 line (every rank must call this: it is one
    all_gather): the backend, the group's world size, and each rank's window count and own timed
    seconds — so a SCALE record proves from the line that RCCL ran N ranks over the whole batch."""
    import torch.distributed as dist
    world = dist.get_world_size()
    t = torch.tensor([float(windows), float(local_elapsed)], dtype=torch.float64, device=device)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return {"backend": str(dist.get_backend()), "world_size": world,
            "windows_per_rank": [int(p[0].item()) for p in parts],
            "rank_elapsed_s": [float(p[1].item()) for p in parts]}


def check_world(world: int, gpus: int) -> None:
    """bench.py --gpus N must run as exactly N ranks (torch.distributed.run, one rank per GPU)."""
    if world != gpus:
        sys.exit(f"bench.py --gpus {gpus} but the launch has WORLD_SIZE={world}: run one rank per GPU "
                 f"under torch.distributed.run --nproc-per-node {gpus}")


def torch_cpu_rollout(sd, x, H, N, mean_t, std_t):
    """The reference's rollout ops (backtest.py:99-121 with model.py:756-797) batched over the
    windows in torch on the CPU: encode, then H x (z @ K, full obs-width decode, slice the first N,
    de-standardize)."""
    with torch.no_grad():
        z = x
        for k in range(3):
            z = torch.nn.functional.linear(z, sd[f"encoder.network.{2 * k}.weight"], sd[f"encoder.network.{2 * k}.bias"])
            if k < 2:
                z = torch.relu(z)
        ys = []
        for _ in range(H):
            z = z @ sd["kmat"]
            p_ = torch.nn.functional.linear(z, sd["decoder.network.0.weight"])
            ys.append(p_[:, :N] * std_t + mean_t)
        return torch.stack(ys, 1)


def cpu_baseline(sd, mean, std, x_gpu, wp_gpu, W0_gpu, val_gpu, y_gpu, H, N, cfg, budget_s):
    """SURVEY §8(d) item 2, "all-cores batched": the reference's rollout ops batched in torch on the
    CPU (torch_cpu_rollout, all host threads) + the OpenMP float64 C restatement of the solve
    (oracle/kmpc_oracle.c), timed on a bounded sample of the same windows on this host's cores.
    The numpy restatement of the rollout (oracle/rollout.py) is kept as a cross-check only.
    Returns (cpu_baseline dict, parity dict)."""
    from oracle import rollout as orollout, solver as osolver
    spec = {"kind": "generic",
            "enc_w": [sd[f"encoder.network.{2 * k}.weight"].numpy() for k in range(3)],
            "enc_b": [sd[f"encoder.network.{2 * k}.bias"].numpy() for k in range(3)],
            "enc_act": "relu", "kmat": sd["kmat"].numpy(), "norm_fn": "id",
            "dec_w": [sd["decoder.network.0.weight"].numpy()], "dec_b": [None]}
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = torch.get_num_threads()
    torch.set_num_threads(cores)
    mean_t, std_t = torch.tensor(mean), torch.tensor(std)

    def run(lo, hi):
        x = x_gpu[lo:hi].cpu()
        wp = wp_gpu[lo:hi].cpu().numpy()
        t0 = time.perf_counter()
        y = torch_cpu_rollout(sd, x, H, N, mean_t, std_t).numpy()
        W, st, obj, it = osolver.solve_batch(wp, y, cfg.cost_coeff, cfg.max_turnover, cfg.allow_short,
                                             max_iter=cfg.max_iter, tol=cfg.tol, precision="d")
        return time.perf_counter() - t0, y, W, st

    try:
        run(0, 2 * cores)                                  # warms BLAS / OpenMP
        dt, _, _, _ = run(0, 8 * cores)                    # calibration
        per = dt / (8 * cores)
        n = int(min(max(budget_s / max(per, 1e-6), 2 * cores), x_gpu.shape[0]))
        dt, y, W, st = run(0, n)
    finally:
        torch.set_num_threads(threads)
    base = {"value": n / dt, "unit": "windows/s", "cores": cores, "kind": "port",
            "sample": f"first {n} windows of rank 0's C3 batch: batched torch-CPU rollout in the reference's "
                      f"ops (full obs-width decode, {cores} threads) + OpenMP float64 IPM "
                      f"(oracle/kmpc_oracle.c, {cores} threads), {dt:.1f} s"}
    y_np = orollout.rollout(spec, x_gpu[:256].cpu().numpy(), H, N, mean, std)   # cross-check only
    # parity on the same inputs: the float64 oracle solve of the device's own yhat (256 windows),
    # and the rollout (numpy fp32 vs MFMA fp32) relative error over the timed sample
    k = min(256, n)
    yg = y_gpu[:k].cpu().numpy()
    Wo, sto, vo, _ = osolver.solve_batch(wp_gpu[:k].cpu().numpy(), yg, cfg.cost_coeff, cfg.max_turnover,
                                         cfg.allow_short, precision="ld")
    W0 = W0_gpu[:k].cpu().numpy()
    vg = val_gpu[:k].cpu().numpy()
    ynp = y_gpu[:n].cpu().numpy()
    parity = {"windows": k, "oracle_optimal": int((sto <= 1).sum()),
              "max_abs_dW0": float(np.abs(W0 - Wo[:, 0]).max()),
              "max_abs_dobj": float(np.abs(vg - vo).max()), "max_abs_obj": float(np.abs(vo).max()),
              "rollout_max_rel_err": float(np.abs(ynp - y).max() / np.abs(y).max()),
              "torch_cpu_vs_numpy_rollout_max_rel_err": float(np.abs(y[:256] - y_np).max() / np.abs(y_np).max())}
    return base, parity


def cpu_baseline_serial(sd, mean, std, x_gpu, wp_gpu, H, N, cfg, budget_s):
    """BASELINE.md §3 item 1, "reference-semantics serial": one window at a time on one core, as
    the reference's run_backtest drives KoopmanMPCStrategy.rebalance — a torch-CPU batch-1 rollout
    in the op order of backtest.py:99-121 (full obs-width decode, slice, de-standardize per step)
    and the float64 C restatement of the solve (oracle/kmpc_oracle.c, single window, no OpenMP)."""
    from oracle import solver as osolver
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        enc = [(sd[f"encoder.network.{2 * k}.weight"], sd[f"encoder.network.{2 * k}.bias"]) for k in range(3)]
        K = sd["kmat"]
        D = sd["decoder.network.0.weight"]
        mean_t, std_t = torch.tensor(mean), torch.tensor(std)
        xs = x_gpu[:2048].cpu()
        wps = wp_gpu[:2048].cpu().numpy()

        def window(i):
            with torch.no_grad():
                z = xs[i:i + 1]
                for k, (W, b) in enumerate(enc):              # GenericKM.encode (model.py:756-766)
                    z = torch.nn.functional.linear(z, W, b)
                    if k < 2:
                        z = torch.relu(z)
                ys = []
                for _ in range(H):                             # backtest.py:107-119
                    z = z @ K                                  # step_latent (model.py:787-797), norm 'id'
                    p_ = torch.nn.functional.linear(z, D)      # decode: full obs width (model.py:768-777)
                    ys.append((p_[..., :N] * std_t + mean_t).numpy().flatten())
            y = np.array(ys)                                   # backtest.py:121
            osolver.solve(wps[i], y, cfg.cost_coeff, cfg.max_turnover, cfg.allow_short, max_iter=cfg.max_iter,
                          tol=cfg.tol, precision="d")

        window(0)
        t0 = time.perf_counter()
        n = 0
        while n < xs.shape[0] and (n < 1024 or time.perf_counter() - t0 < budget_s):
            window(n)
            n += 1
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(threads)
    return {"value": n / dt, "unit": "windows/s", "cores": 1, "kind": "port",
            "sample": f"first {n} windows of rank 0's C3 batch, one at a time: torch-CPU batch-1 rollout "
                      f"(backtest.py:99-121 op order, full decode) + float64 C solve (oracle/kmpc_oracle.c), "
                      f"1 thread, {dt:.1f} s"}


def cpu_baseline_c1(n_test: int = 1000) -> dict:
    """BASELINE configs[0]: the reference plumbing on one CPU thread — run_backtest
    (backtest.py:133-219, restated in oracle/backtest_ref.py) over a synthetic 1000-row test set,
    10 assets, finance_sparse GenericKM (obs 200, encoder [1024, 1024], latent 128, linear decoder),
    MPCConfig(horizon=5) / BacktestConfig(horizon=5). Each of the 995 steps runs
    KoopmanMPCStrategy.rebalance as the reference does: a torch-CPU batch-1 rollout in the op order
    of backtest.py:99-121 (full obs-width decode, slice, de-standardize per step) and the float64 C
    solve (oracle/kmpc_oracle.c), then the numpy bookkeeping (cost, realized return, drift)."""
    from oracle import backtest_ref, solver as osolver
    N, L, H, emb, hidden = 10, 128, 5, 20, 1024
    obs = N * emb
    sd = make_state_dict(obs, L, hidden, seed=10)
    g = torch.Generator().manual_seed(10)
    data = torch.randn(n_test, obs, generator=g)                    # standardized embedded test rows
    mean_t = torch.full((N,), 5e-4)
    std_t = torch.full((N,), 0.015)
    all_returns = (data[:, :N] * std_t + mean_t).numpy()            # backtest.py:169-171
    cfg_m = {"horizon": H, "cost_coeff": 1e-3, "max_turnover": 0.2}
    enc = [(sd[f"encoder.network.{2 * k}.weight"], sd[f"encoder.network.{2 * k}.bias"]) for k in range(3)]
    K, D = sd["kmat"], sd["decoder.network.0.weight"]
    threads = torch.get_num_threads()
    torch.set_num_threads(1)

    def rebalance(t, w):
        with torch.no_grad():
            z = data[t].unsqueeze(0)                                  # backtest.py:85
            for k, (W, b) in enumerate(enc):
                z = torch.nn.functional.linear(z, W, b)
                if k < 2:
                    z = torch.relu(z)
            ys = []
            for _ in range(H):
                z = z @ K
                p_ = torch.nn.functional.linear(z, D)
                ys.append((p_[..., :N] * std_t + mean_t).numpy().flatten())
        Wm, st, _, _ = osolver.solve(w, np.array(ys), cfg_m["cost_coeff"], cfg_m["max_turnover"], False,
                                     precision="d")
        return Wm[0] if st <= 1 else w.copy()

    try:
        rebalance(0, np.ones(N) / N)
        t0 = time.perf_counter()
        hist = backtest_ref.run_backtest(rebalance, all_returns, n_test, H, N, 10000.0, 1, 1e-3)
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(threads)
    return {"value": len(hist) / dt, "unit": "windows/s", "cores": 1, "kind": "port", "steps": len(hist),
            "seconds": dt, "final_value": hist[-1]["portfolio_value"],
            "sample": f"BASELINE configs[0] (C1): full run_backtest, {n_test} synthetic test rows -> {len(hist)} "
                      f"sequential rebalance steps, 10 assets, latent 128, H=5, obs 200, enc [1024,1024]; torch-CPU "
                      f"batch-1 rollout + float64 C solve + numpy bookkeeping, 1 thread, {dt:.1f} s"}


def secondary_c2(dev, steps: int, warmup: int) -> dict:
    """BASELINE configs[1] beside the headline (same step, same timing rule, rank 0 only): 4,096
    windows, 30 assets, latent 128, H = 5, c = tau = 0 no-short (the simplex program)."""
    from koopman_mpc_portfolio_rebalancing_amd import (DeviceKoopman, KoopmanModelSpec, MPCConfig,
                                                       solve_mpc_log_utility_batched)
    B, N, L, H, hidden = 4096, 30, 128, 5, 1024
    obs = N * 20
    model = DeviceKoopman(KoopmanModelSpec.from_state_dict(make_state_dict(obs, L, hidden, seed=1), MODEL_CFG), dev)
    mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
    std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
    x, wp = make_inputs(B, N, obs, seed=100, device=dev)
    cfg = MPCConfig(horizon=H, cost_coeff=0.0, max_turnover=0.0, allow_short=False)
    reps = 20 * max(steps, 1)

    def step():   # the fused window (kmpc_window), as the headline
        return model.window(x, wp, mean_d, std_d, N, cfg)
    for _ in range(max(warmup, 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        W0, st, val = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"workload": f"C2 (BASELINE configs[1]): {B} windows, {N} assets, latent {L}, H={H}, obs {obs}, "
                        f"enc [{hidden},{hidden}], c=0 tau=0 no-short", "windows_per_s": B * reps / el,
            "ms_per_step": el / reps * 1e3, "steps": reps,
            "optimal_or_inaccurate": int((st.cpu().numpy() <= 1).sum()), "windows": B}


def secondary_c1(dev, steps: int, warmup: int, B: int = 65536) -> dict:
    """The BASELINE configs[0] model (10 assets, latent 128, H = 5, obs 200, encoder [1024, 1024],
    MPCConfig(horizon=5, cost 1e-3, turnover cap 0.2) — the model and MPC of cpu_baseline_c1) with
    its windows batched on the GPU: the small-window solve packs four windows per wave (16-lane
    groups, kmpc_solve_kernel.h)."""
    from koopman_mpc_portfolio_rebalancing_amd import (DeviceKoopman, KoopmanModelSpec, MPCConfig,
                                                       solve_mpc_log_utility_batched)
    N, L, H, hidden = 10, 128, 5, 1024
    obs = N * 20
    model = DeviceKoopman(KoopmanModelSpec.from_state_dict(make_state_dict(obs, L, hidden, seed=10), MODEL_CFG), dev)
    mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
    std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
    x, wp = window_inputs(0, B, N, obs, seed=10, device=dev)
    cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, allow_short=False)
    reps = max(steps, 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step():   # the fused window (kmpc_window), as the headline
        return model.window(x, wp, mean_d, std_d, N, cfg, with_iters=True)
    for _ in range(max(warmup, 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        W0, st, val, its = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    y = model.rollout(x, mean_d, std_d, H, N)
    ev[0].record()
    solve_mpc_log_utility_batched(wp, y, cfg)
    ev[1].record()
    torch.cuda.synchronize()
    return {"workload": f"configs[0] model batched on the GPU: {B} windows, {N} assets, latent {L}, H={H}, obs {obs}, "
                        f"enc [{hidden},{hidden}], c=1e-3 tau=0.2 no-short (packed solve: 4 windows per wave)",
            "windows_per_s": B * reps / el, "ms_per_step": el / reps * 1e3, "steps": reps,
            "solve_ms": ev[0].elapsed_time(ev[1]), "mean_ipm_iterations": float(its.float().mean().item()),
            "optimal_or_inaccurate": int((st.cpu().numpy() <= 1).sum()), "windows": B}


def secondary_lockstep(dev, P: int = 64, T: int = 130, N: int = 100, L: int = 256, H: int = 10,
                       seed: int = 0) -> dict:
    """SURVEY §8(f) row 1 at a small path count: P backtest paths of the
    headline model (100 assets, latent 256, H = 10, c = 1e-3, tau = 0.2; or, with N = 10, L = 128,
    H = 5, seed 10, the configs[0] model — VERDICT r05 item 7) over T test rows,
    run_backtest_lockstep with its defaults (forecasts rolled out up front, then every step of every
    path in one path-persistent launch, kmpc_backtest_run; bit-identical to the lock-step loop);
    path-steps/s = P x steps / wall time of the second of two identical runs. Beside it the
    lock-step loop (three path groups on streams) for comparison."""
    from koopman_mpc_portfolio_rebalancing_amd import BacktestConfig, KoopmanModelSpec, KoopmanMPCStrategy, MPCConfig
    from koopman_mpc_portfolio_rebalancing_amd.backtest import run_backtest_lockstep
    obs = N * 20
    spec = KoopmanModelSpec.from_state_dict(make_state_dict(obs, L, 1024, seed=seed), MODEL_CFG)
    strat = KoopmanMPCStrategy(spec, MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2), device=str(dev))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(P, T, obs, generator=g).to(dev)
    r = (torch.randn(P, T, N, generator=g) * 0.015 + 5e-4).to(dev)
    mean, std = np.full(N, 5e-4, np.float32), np.full(N, 0.015, np.float32)
    cfg = BacktestConfig(horizon=H)
    run_backtest_lockstep(strat, x, r, cfg, mean, std)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = run_backtest_lockstep(strat, x, r, cfg, mean, std)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    S = int(out["return"].shape[1])
    run_backtest_lockstep(strat, x, r, cfg, mean, std, persistent=False)   # (warm-up: its streams, first calls)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop = run_backtest_lockstep(strat, x, r, cfg, mean, std, persistent=False)
    torch.cuda.synchronize()
    el_loop = time.perf_counter() - t0
    res = {"workload": f"{P} backtest paths x {S} steps, {'C3' if N == 100 else 'configs[0]'} model ({N} assets, "
                       f"latent {L}, H={H}), run_backtest_lockstep defaults (path-persistent kernel)",
           "path_steps_per_s": P * S / el, "ms_per_step": el / S * 1e3,
           "lockstep_loop_path_steps_per_s": P * S / el_loop, "speedup_vs_loop": el_loop / el,
           "bit_identical_to_loop": bool(torch.equal(out["portfolio_value"], loop["portfolio_value"]))}
    if N == 100:
        res["r04_path_steps_per_s"] = 30.5e3
    return res


def make_lista_state_dict(obs: int, L: int, seed: int = 0) -> dict:
    """LISTAKM layout (model.py:190-209, 804-850) with LINEAR_ENCODER: the classic LISTA start
    We = D / Lc, S = I - D D^T / Lc for a random unit-row dictionary D [L, obs], Lc = 1.1 ||D||_2^2
    (BASELINE configs[4])."""
    g = torch.Generator().manual_seed(seed)
    D = torch.randn(L, obs, generator=g)
    D = D / D.norm(dim=1, keepdim=True)
    v = torch.randn(obs, generator=g)
    for _ in range(30):                       # power iteration for ||D||_2
        v = D.t() @ (D @ v)
        v = v / v.norm()
    lc = 1.1 * float((D @ v).norm() ** 2)
    q, _ = torch.linalg.qr(torch.randn(L, L, generator=g, dtype=torch.float64))
    sd = {"dict": D, "kmat": (0.95 * q).float(), "dict_init": D.t().contiguous(),
          "lista.S": torch.eye(L) - (D @ D.t()) / lc, "lista.We.weight": D / lc}
    return sd, lc


def secondary_c5(dev, steps: int, warmup: int, B: int = 1024) -> dict:
    """BASELINE configs[4] beside the headline: LISTAKM encoder, 500 assets, latent 512, H = 20,
    bf16 MFMA rollout, the large-window f64 solve (c = 1e-3, tau = 0.2, no short).

    The reference rolls out in fp32 (model.py:828-850), so the bf16 forecast is not the program the
    reference would solve. bf16_decision_gap prices that: the bf16 path's decision W^bf16 evaluated
    in the fp32-yhat program, f*(fp32) - f(W^bf16; fp32 yhat) per window (problem.value units,
    mpc.py:103; the fp32 solve's own W is the optimum at the solver's bar 1e-6 + 1e-5 |f*|), next to
    the fp32 rollout's time. The fp32 rollout is the default of DeviceKoopman / the strategy path;
    bf16 is the opt-in configuration BASELINE names."""
    from koopman_mpc_portfolio_rebalancing_amd import (DeviceKoopman, KoopmanModelSpec, MPCConfig,
                                                       log_utility_value_batched, solve_mpc_log_utility_batched)
    N, L, H = 500, 512, 20
    obs = N * 20
    sd, lc = make_lista_state_dict(obs, L, seed=2)
    cfg_m = {"MODEL": {"MODEL_NAME": "LISTAKM", "NORM_FN": "id",
                       "ENCODER": {"LISTA": {"ALPHA": 5e-3, "L": lc, "NUM_LOOPS": 10}}}}
    spec = KoopmanModelSpec.from_state_dict(sd, cfg_m)
    model = DeviceKoopman(spec, dev, dtype="bf16")
    model32 = DeviceKoopman(spec, dev, dtype="fp32")
    mean_d = torch.full((N,), 5e-4, dtype=torch.float32, device=dev)
    std_d = torch.full((N,), 0.015, dtype=torch.float32, device=dev)
    x, wp = make_inputs(B, N, obs, seed=200, device=dev)
    cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, allow_short=False)
    for _ in range(max(warmup, 1)):
        solve_mpc_log_utility_batched(wp, model.rollout(x, mean_d, std_d, H, N), cfg)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t0 = time.perf_counter()
    roll, solv = 0.0, 0.0
    for _ in range(max(steps, 1)):
        e[0].record()
        y = model.rollout(x, mean_d, std_d, H, N)
        e[1].record()
        W0, st, val = solve_mpc_log_utility_batched(wp, y, cfg)
        e[2].record()
        torch.cuda.synchronize()
        roll += e[0].elapsed_time(e[1])
        solv += e[1].elapsed_time(e[2])
    el = time.perf_counter() - t0
    k = max(steps, 1)
    # the fp32 rollout (the reference's arithmetic): its time, and the bf16 decision priced in it
    model32.rollout(x, mean_d, std_d, H, N)
    torch.cuda.synchronize()
    r32 = 0.0
    for _ in range(k):
        e[0].record()
        y32 = model32.rollout(x, mean_d, std_d, H, N)
        e[1].record()
        torch.cuda.synchronize()
        r32 += e[0].elapsed_time(e[1])
    W16, st16, _ = solve_mpc_log_utility_batched(wp, y, cfg, return_full=True)
    W32, st32, v32 = solve_mpc_log_utility_batched(wp, y32, cfg, return_full=True)
    ok = (st16 <= 1) & (st32 <= 1)
    f32 = log_utility_value_batched(W32, wp, y32, cfg.cost_coeff)
    f16 = log_utility_value_batched(W16, wp, y32, cfg.cost_coeff)
    gap = (f32 - f16)[ok].cpu().numpy()
    bar = (1e-6 + 1e-5 * f32.abs())[ok].cpu().numpy()
    rel_y = float(((y - y32).abs().amax((1, 2)) / y32.abs().amax((1, 2))).max().item())
    return {"workload": f"C5 (BASELINE configs[4]): {B} windows, {N} assets, LISTAKM latent {L} (10 loops, linear "
                        f"encoder), H={H}, obs {obs}, bf16 MFMA rollout, f64 large-window solve c=1e-3 tau=0.2",
            "windows_per_s": B * k / el, "ms_per_step": el / k * 1e3, "steps": k,
            "rollout_ms": roll / k, "solve_ms": solv / k,
            "optimal_or_inaccurate": int((st.cpu().numpy() <= 1).sum()), "windows": B,
            "fp32_rollout_ms": r32 / k,
            # the default (fp32) rollout's configs[4] rate from the same kernel timings
            "windows_per_s_fp32_rollout_kernels": B / ((r32 + solv) / k * 1e-3),
            "bf16_decision_gap": {"max": float(gap.max()), "p99": float(np.percentile(gap, 99)),
                                  "median": float(np.median(gap)), "windows": int(gap.size),
                                  "windows_over_objective_bar": int((gap > bar).sum()),
                                  "objective_bar": "1e-6 + 1e-5 |f*|", "max_rel_yhat_err": rel_y,
                                  "meaning": "f*(fp32 yhat) - f(W_bf16; fp32 yhat), problem.value units"}}


def rollout_f64(sd: dict, x: torch.Tensor, H: int, N: int, mean, std) -> np.ndarray:
    """The bench model (GenericKM, relu encoder, identity norm, one-layer decoder) in float64 on the
    CPU: the yardstick of the rollout's fp32 arithmetic (rollout_parity)."""
    h = x.double().cpu()
    for i, k in enumerate((0, 2, 4)):
        h = h @ sd[f"encoder.network.{k}.weight"].double().T + sd[f"encoder.network.{k}.bias"].double()
        if i < 2:
            h = torch.relu(h)
    K = sd["kmat"].double()
    D = sd["decoder.network.0.weight"].double()[:N]
    out = []
    for _ in range(H):
        h = h @ K
        out.append((h @ D.T) * torch.as_tensor(std).double() + torch.as_tensor(mean).double())
    return torch.stack(out, 1).numpy()


def rollout_parity(model, sd, x, mean_d, std_d, H, N, n=512) -> dict:
    """Max error of the timed rollout (fp32 GEMMs as three bf16 planes; at the timed batch size the
    latent loop runs as one GEMM against the latent powers, kmpc_rollout.hip) and of the f32-input
    MFMA form, against float64, relative to max|yhat - mean|, on the first n windows of a rollout of
    the whole batch (the timed kernels), after the timed region."""
    from koopman_mpc_portfolio_rebalancing_amd import DeviceKoopman
    ref = rollout_f64(sd, x[:n], H, N, mean_d.cpu().numpy(), std_d.cpu().numpy())
    scale = float(np.abs(ref - mean_d.cpu().numpy()).max())
    y3 = model.rollout(x, mean_d, std_d, H, N)[:n].double().cpu().numpy()
    native = DeviceKoopman(model.spec, model.device, dtype="fp32_f32mfma")
    y1 = native.rollout(x, mean_d, std_d, H, N)[:n].double().cpu().numpy()
    return {"windows": n, "of_batch": int(x.shape[0]), "vs": "float64 restatement (torch CPU, double)",
            "three_plane_max_rel_err": float(np.abs(y3 - ref).max() / scale),
            "f32_input_mfma_max_rel_err": float(np.abs(y1 - ref).max() / scale)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(world, args.gpus)
    import torch.distributed as dist
    gpu = 0 if args.share_device else local
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
        check_world(dist.get_world_size(), args.gpus)
    dev = torch.device("cuda", gpu if world > 1 else 0)
    torch.cuda.set_device(dev)
    # collectives: on the device under RCCL, through host copies under gloo
    comm = dev if args.backend == "nccl" else torch.device("cpu")

    from koopman_mpc_portfolio_rebalancing_amd import (DeviceKoopman, KoopmanModelSpec, MPCConfig,
                                                       solve_mpc_log_utility_batched)
    from koopman_mpc_portfolio_rebalancing_amd.shard import gather_rows, window_range
    N, L, H = args.assets, args.latent, args.horizon
    # N = 1: configs[2] (65536 windows); N > 1: configs[3], 2^20 global windows sharded
    G = args.global_windows or (args.windows if world == 1 else C4_GLOBAL_WINDOWS)
    lo, hi = window_range(G, world, rank)
    B = hi - lo
    obs = N * args.emb
    sd = make_state_dict(obs, L, args.hidden, seed=0)
    model = DeviceKoopman(KoopmanModelSpec.from_state_dict(sd, MODEL_CFG), dev)
    mean = np.full(N, 5e-4, np.float32)
    std = np.full(N, 0.015, np.float32)
    mean_d = torch.tensor(mean, device=dev)
    std_d = torch.tensor(std, device=dev)
    x, wp = window_inputs(lo, hi, N, obs, seed=0, device=dev)
    cfg = MPCConfig(horizon=H, cost_coeff=1e-3, max_turnover=0.2, allow_short=False)

    # the timed step is the product path: DeviceKoopman.window -> kmpc_window (rollout -> solve on
    # one stream, one workspace), what KoopmanMPCStrategy.rebalance_batch runs
    def step(k):
        W0, st, val, its = model.window(x, wp, mean_d, std_d, N, cfg, with_iters=True)
        Wg = W0
        if world > 1:   # the one RCCL collective
            Wg = gather_rows(W0 if comm.type == "cuda" else W0.cpu(), G, world, rank, dst=0)
        return W0, st, val, its, Wg

    tinfo = {}
    elapsed, (W0, st, val, its, Wg) = timed_loop(step, args.steps, args.warmup, world, dev, tinfo, comm)
    prov = rank_provenance(B, tinfo["local_elapsed_s"], comm) if world > 1 else None
    if prov is not None:
        prov["share_device"] = bool(args.share_device)
    if args.dump_w0 and rank == 0:
        np.save(args.dump_w0, Wg.cpu().numpy())

    # kernel split, after the timed region: the same step as two C-ABI calls (kmpc_rollout, then
    # kmpc_solve), each bracketed by HIP events on the launch stream — the solve's launch time is
    # the roofline's; their sum is checked against the fused step's time (two_call_ms_per_step)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for e in ev:
        e[0].record()
        y = model.rollout(x, mean_d, std_d, H, N)
        e[1].record()
        W0s, _, _ = solve_mpc_log_utility_batched(wp, y, cfg)
        e[2].record()
    torch.cuda.synchronize()
    if not torch.equal(W0s, W0):
        sys.exit("bench: the fused window and rollout-then-solve disagree")
    roll_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    solve_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    st_np = st.cpu().numpy()
    n_opt = int((st_np <= 1).sum())

    if rank == 0:
        value = G * args.steps / elapsed
        # roofline of the dominant kernel (the solve), SURVEY §8(d): ALGORITHMIC HBM bytes of one
        # launch — read yhat f32 [B,H,N] + w_prev f64 [B,N]; write W0 f64 [B,N] + status i32 +
        # value f64 + iters i32 per window — over its HIP-event launch time, against 8 TB/s.
        # traffic: PMC HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, profiles/, scaled to B).
        solve_bytes = B * (4 * H * N + 8 * N + 8 * N + 4 + 8 + 4)
        achieved = solve_bytes / (solve_ms * 1e-3)
        pmc = json.load(open(PMC_JSON)) if os.path.exists(PMC_JSON) and (N, H) == (100, 10) else None
        traffic = (pmc["fetch_bytes_per_window"] + pmc["write_bytes_per_window"]) * B if pmc else None
        roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel": "kmpc_solve (ipm_mixed_kernel: float32 phase + float64 finish, then the retry ipm_kernel; register IPM)",
                "launch_ms": solve_ms, "algorithmic_bytes_per_window": solve_bytes // B,
                "windows_per_launch": B}
        # what actually bounds the solve: f64 issue / latency. Executed f64 FLOPs per window from the
        # PMC passes (64 lanes x (ADD + MUL + TRANS + 2 FMA) per wave-instruction), scaled by the
        # active-lane fraction N / blockDim (an upper bound on useful work: wave 0's serial Schur
        # phases idle more lanes), against the f64 FMA peak measured on this part (profiles/).
        # algorithmic f64 FLOPs (solve_flop_model x this run's mean iteration count) against the
        # same measured peak: the fraction of the f64 ceiling the ALGORITHM achieves; the executed
        # (PMC) figure beside it counts padding lanes, recomputation and refinement as work
        iters_mean = float(its.float().mean().item())
        fm = solve_flop_model(N, H)
        alg = fm["per_iteration"] * iters_mean
        peak = F64_VALU_PEAK
        # mixed precision: about half of the iterations run in float32 (float32 phase),
        # the rest in float64; the algorithmic FLOPs are counted once per iteration either way and set
        # against the float64 VALU peak, the lower of the two pipes' peaks
        util = {"pipe": "f64 VALU (float32 phase + float64 finish; f32 work counted against the f64 peak)",
                "algorithmic_f64_flops_per_window": alg,
                "algorithmic_f64_flops_per_iteration": fm["per_iteration"],
                "algorithmic_phases_per_iteration": fm["phases"], "mean_ipm_iterations": iters_mean,
                "unit": "TFLOP/s"}
        if pmc and "f64_flops_per_window" in pmc:
            lanes = pmc.get("active_lane_fraction", N / (64 * -(-N // 64)))
            useful = pmc["f64_flops_per_window"] * lanes * B / (solve_ms * 1e-3)
            peak = best_f64_peak()[0] or pmc.get("f64_peak_flops", F64_VALU_PEAK)
            if "f32_flops_per_window" in pmc:
                util["executed_f32_flops_per_window"] = pmc["f32_flops_per_window"]
            util.update({"executed_f64_flops_per_window": pmc["f64_flops_per_window"],
                         "executed_over_algorithmic": pmc["f64_flops_per_window"] / alg,
                         "active_lane_fraction": lanes, "achieved": useful / 1e12,
                         "frac": useful / peak, "counts_from": os.path.relpath(PMC_JSON, ROOT)})
        util.update({"algorithmic_achieved": alg * B / (solve_ms * 1e-3) / 1e12, "peak": peak / 1e12,
                     "algorithmic_frac": alg * B / (solve_ms * 1e-3) / peak,
                     "peak_source": best_f64_peak()[1] if best_f64_peak()[0] else "spec"})
        # rollout FLOPs the timed path EXECUTES: the encoder, then the latent loop as the library
        # runs it at this batch size — from 8,192 windows (KMPC_LATPOW_MINB, identity norm) one GEMM
        # of z_0 against the latent powers [H N, L] (L H N multiply-adds per window) plus the
        # per-call powers chain (H N L^2, latent_powers_kernel); below it H (L^2 + L N) per window
        latpow = B >= LATPOW_MINB
        lat_flops = 2.0 * B * H * N * L + 2.0 * H * N * L * L if latpow else 2.0 * B * H * (L * L + L * N)
        roll_flops = 2.0 * B * (obs * args.hidden + args.hidden * args.hidden + args.hidden * L) + lat_flops
        c4 = world > 1
        line = {
            "metric": METRIC, "value": value, "unit": "windows/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if c4 else "weak", "vs_baseline": None,
            "dtype": "f32 rollout (fp32 GEMMs as three exact bf16 planes); mixed f32->f64 IPM solve "
                     "(float32 phase to mu 3e-5, float64 finish: stopping rule, status and W in float64)",
            "data": "synthetic (seeded N(0,1) standardized embeddings, Dirichlet w_prev, random-init finance_sparse weights)",
            "config": {"workload": (f"C4 (BASELINE configs[3]): {G} windows/step over {world} GPUs" if c4 else
                                    f"C3 (BASELINE configs[2]): {G} windows/GPU") +
                                   f", {N} assets, latent {L}, H={H}, obs {obs}, GenericKM enc "
                                   f"[{args.hidden},{args.hidden}], L1-turnover MPC c=1e-3 tau=0.2 no-short",
                       "windows_per_gpu": B, "global_windows_per_step": G,
                       "parallelism": ((f"windows sharded over {world} ranks sharing cuda:0 (readiness check, not "
                                        f"a scaling figure), {args.backend} gather of W0 to rank 0")
                                       if args.share_device and c4 else
                                       f"windows sharded over {world} GPUs (contiguous blocks of one global "
                                       f"stream), {'RCCL' if args.backend == 'nccl' else 'gloo'} gather of W0 to rank 0"
                                       if c4 else "1 GPU, no collective")}
                      | ({"dist": prov} if prov else {}),
            "roofline": roof,
            "compute_utilization": util,
            # SURVEY.md §8(d)'s whole-path bound: compulsory bytes per window = obs (f32 N d) +
            # w_prev + w0 (f32 as there), weights amortized: windows/s x bytes / 8 TB/s
            "path_hbm_roofline": {"bound": "hbm", "bytes_per_window": 4 * obs + 8 * N,
                                  "achieved": value / world * (4 * obs + 8 * N) / 1e9, "peak": HBM_PEAK / 1e9,
                                  "unit": "GB/s", "frac": value / world * (4 * obs + 8 * N) / HBM_PEAK,
                                  "ceiling_windows_per_s_per_gpu": HBM_PEAK / (4 * obs + 8 * N)},
            "timed_path": "kmpc_window via DeviceKoopman.window (the KoopmanMPCStrategy.rebalance_batch path); "
                          "kernels: the same step as kmpc_rollout + kmpc_solve, HIP events, after the timed region",
            # rollout: algorithmic fp32 FLOPs / time, against the f32-input MFMA peak; the GEMMs and the
            # L = 256 latent loop run as three bf16 planes (six bf16 products per fp32 product), so
            # the bf16 MFMA pipe executes 6x those FLOPs (rollout_bf16_mfma_executed_frac)
            "kernels": {"rollout_ms": roll_ms, "solve_ms": solve_ms, "two_call_ms_per_step": roll_ms + solve_ms,
                        "rollout_tflops": roll_flops / (roll_ms * 1e-3) / 1e12,
                        "rollout_frac_of_f32_mfma_peak": roll_flops / (roll_ms * 1e-3) / FP32_MFMA_PEAK,
                        "rollout_bf16_mfma_executed_frac": 6 * roll_flops / (roll_ms * 1e-3) / BF16_MFMA_PEAK,
                        "rollout_gemm_form": "fp32 as three exact bf16 planes on v_mfma_f32_32x32x16_bf16",
                        "rollout_flops_counted": "executed: encoder + " + (
                            "latent powers GEMM (2 L H N per window) + the per-call powers chain (2 H N L^2)"
                            if latpow else "sequential latent loop (2 H (L^2 + L N) per window)")},
            "solver": {"optimal_or_inaccurate": n_opt, "windows": B,
                       "mean_ipm_iterations": float(its.float().mean().item())},
        }
        line["rollout_parity"] = rollout_parity(model, sd, x, mean_d, std_d, H, N)
        if world == 1 and not args.headline_only:
            line["secondary"] = secondary_c2(dev, args.steps, args.warmup)
            line["secondary_c1"] = secondary_c1(dev, args.steps, args.warmup)
            line["secondary_c5"] = secondary_c5(dev, min(args.steps, 3), min(args.warmup, 1))
            line["secondary_lockstep"] = secondary_lockstep(dev)
            line["secondary_lockstep_c1"] = secondary_lockstep(dev, N=10, L=128, H=5, seed=10)
        if world == 1 and args.cpu_seconds > 0 and not args.headline_only:
            base, parity = cpu_baseline(sd, mean, std, x, wp, W0, val, y, H, N, cfg, args.cpu_seconds)
            line["cpu_baseline"] = base
            line["cpu_baseline_serial"] = cpu_baseline_serial(sd, mean, std, x, wp, H, N, cfg,
                                                              min(8.0, args.cpu_seconds / 2))
            line["cpu_baseline_c1"] = cpu_baseline_c1()
            line["cpu_parity"] = parity
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
