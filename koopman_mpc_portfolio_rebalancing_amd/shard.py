"""Window sharding across ranks: one process per GPU, contiguous window ranges per
rank, no inter-GPU traffic during compute, one gather of the per-window weights to rank 0.

Rolling-backtest windows are independent given (obs_t, w_prev) — forecasts never depend on
weights — so a batch of windows partitions with no data-path collective. The same helpers run
under the "nccl" (RCCL over xGMI) backend on GPUs and under "gloo" on CPU (tests).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


def window_range(n_windows: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) block of rank `rank`; sizes differ by at most one window."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n_windows, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_rows(t: torch.Tensor, n_windows: int, world: int, rank: int, dst: int = 0) -> Optional[torch.Tensor]:
    """Gather each rank's row block of a [rows, ...] tensor to `dst` (one collective).

    Blocks may be ragged (window_range); they are padded to the largest block for the collective and
    trimmed on `dst`. Returns the [n_windows, ...] concatenation on `dst`, None elsewhere.
    """
    if world == 1:
        return t
    sizes = [window_range(n_windows, world, r) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    mine = t
    if t.shape[0] < cap:
        mine = torch.cat([t, t.new_zeros((cap - t.shape[0],) + tuple(t.shape[1:]))])
    bufs: Optional[List[torch.Tensor]] = None
    if rank == dst:
        bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.gather(mine.contiguous(), bufs, dst=dst)
    if rank != dst:
        return None
    return torch.cat([b[: hi - lo] for b, (lo, hi) in zip(bufs, sizes)])


def run_sharded(fn: Callable[..., torch.Tensor], n_windows: int, *per_window: torch.Tensor,
                world: int = 1, rank: int = 0, dst: int = 0) -> Optional[torch.Tensor]:
    """Apply fn to this rank's block of every per-window input; gather the results to `dst`."""
    lo, hi = window_range(n_windows, world, rank)
    out = fn(*[x[lo:hi] for x in per_window])
    return gather_rows(out, n_windows, world, rank, dst)
