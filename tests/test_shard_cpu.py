"""Multi-rank window sharding on CPU: world_size 2 over gloo, ragged blocks,
one gather to rank 0; the gathered result must equal the single-process result bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from koopman_mpc_portfolio_rebalancing_amd.shard import gather_rows, run_sharded, window_range


def test_window_range_partitions():
    for n in (0, 1, 7, 64, 65537):
        for world in (1, 2, 3, 8):
            blocks = [window_range(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
            sizes = [hi - lo for lo, hi in blocks]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        window_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _solve_block(wp, y):
    from oracle import solver
    W, st, obj, _ = solver.solve_batch(wp.numpy(), y.numpy(), 1e-3, 0.3, precision="d")
    return torch.from_numpy(W[:, 0].copy())


def _worker(rank, world, port, out_path, wp, y):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = run_sharded(_solve_block, wp.shape[0], wp, y, world=world, rank=rank)
        if rank == 0:
            np.save(out_path, res.numpy())
        else:
            assert res is None
        # a second collective on the same group: ragged integer rows
        lo, hi = window_range(5, world, rank)
        g = gather_rows(torch.arange(lo, hi, dtype=torch.int64)[:, None].repeat(1, 3), 5, world, rank)
        if rank == 0:
            assert torch.equal(g, torch.arange(5)[:, None].repeat(1, 3))
    finally:
        dist.destroy_process_group()


def test_sharded_solve_equals_single_process(tmp_path):
    rng = np.random.default_rng(5)
    B, N, H = 7, 6, 3
    wp = torch.from_numpy(rng.dirichlet(np.ones(N), B))
    y = torch.from_numpy(rng.normal(5e-4, 0.02, (B, H, N)).astype(np.float32))
    out = str(tmp_path / "w0.npy")
    mp.spawn(_worker, args=(2, _free_port(), out, wp, y), nprocs=2, join=True)
    ref = _solve_block(wp, y).numpy()
    assert np.array_equal(np.load(out), ref)
