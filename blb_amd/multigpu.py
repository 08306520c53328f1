"""Multi-GPU stripe sharding.

Stripes are independent units: N GPUs split a batch contiguously and never exchange data
(no RCCL collective on the data path).  One process per GPU (torchrun); torch.distributed is
used only to line the ranks up (barrier) and to take the max-over-ranks wall time.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Rank:
    rank: int
    world: int
    local: int


def env_rank() -> Rank:
    return Rank(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                int(os.environ.get("LOCAL_RANK", "0")))


def stripe_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous share [start, start+count) of `total` stripes for `rank`: the first
    total % world ranks take one extra stripe.  Shares are disjoint and cover the batch."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _coll_device(device):
    """Where the scalar all-reduce runs: the rank's GPU under RCCL, the CPU under gloo."""
    import torch.distributed as dist
    return "cpu" if dist.get_backend() == "gloo" else device


def max_over_ranks(value: float, device=None) -> float:
    """All-reduce MAX of a per-rank wall time (identity when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    """All-reduce SUM of a per-rank count (units processed), identity when single-rank."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def aggregate_gibps(bytes_per_rank: float, seconds_per_rank: float, device=None) -> float:
    """Whole-job throughput: data bytes of ALL ranks / max-over-ranks time, in GiB/s."""
    total = sum_over_ranks(bytes_per_rank, device)
    t = max_over_ranks(seconds_per_rank, device)
    return total / float(1 << 30) / t
