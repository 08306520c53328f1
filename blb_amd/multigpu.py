"""Multi-GPU stripe sharding.

Stripes are independent units: N GPUs split a batch contiguously and never exchange data
(no RCCL collective on the data path).  One process per GPU (torchrun); torch.distributed is
used only to line the ranks up (barrier) and to take the max-over-ranks wall time.
"""
from __future__ import annotations

import os
import platform
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


# ---- NUMA placement of a rank (one process per GPU on a 2-socket, 8-GPU host) ----

_SYS_SET_MEMPOLICY = 238   # x86_64
_MPOL_PREFERRED = 1


def parse_cpulist(text: str) -> set:
    """ "0-3,8,10-11" -> {0, 1, 2, 3, 8, 10, 11} (sysfs cpulist format)."""
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            lo, hi = part.split("-")
            cpus.update(range(int(lo), int(hi) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def bind_to_node(node: int, sysfs: str = "/sys/devices/system/node") -> dict:
    """Bind this process's CPUs to `node`'s (intersected with the affinity it already has, so a
    job's cgroup share is respected) and make `node` the preferred node for its future page
    allocations (set_mempolicy MPOL_PREFERRED: pinned host stripes land next to the GPU and fall
    back to other nodes only when it is full).  Call before any pin_memory.  Returns what was
    done; nothing is changed when the node is unknown or the intersection is empty."""
    import ctypes
    out = {"node": node, "cpus_bound": 0, "mempolicy": None, "bound": False}
    if node is None or node < 0:
        out["reason"] = "GPU NUMA node unknown"
        return out
    try:
        cpus = parse_cpulist(open(os.path.join(sysfs, f"node{node}", "cpulist")).read())
    except OSError as e:
        out["reason"] = f"no cpulist: {e}"
        return out
    mine = os.sched_getaffinity(0)
    both = cpus & mine
    if both:
        # sched_setaffinity(0) binds only the calling thread: bind every thread the process
        # already has (the HIP runtime's among them), and the caller's future threads inherit it.
        for tid in _threads():
            try:
                os.sched_setaffinity(tid, both)
            except OSError:
                pass  # the thread ended meanwhile
        out["cpus_bound"] = len(both)
    else:
        out["reason"] = "node's CPUs outside this job's affinity"
    mask = ctypes.c_ulong(1 << node) if node < 64 else None
    if platform.machine() != "x86_64":
        mask = None  # the syscall number is x86_64's (238 is migrate_pages on aarch64)
        out["mempolicy"] = f"skipped on {platform.machine()}"
    if mask is not None:
        libc = ctypes.CDLL(None, use_errno=True)
        rc = libc.syscall(_SYS_SET_MEMPOLICY, _MPOL_PREFERRED, ctypes.byref(mask), ctypes.c_ulong(64))
        out["mempolicy"] = "preferred" if rc == 0 else f"failed errno {ctypes.get_errno()}"
    out["bound"] = bool(both) and out["mempolicy"] == "preferred"
    return out


def _threads() -> list:
    """Thread ids of this process (/proc/self/task), the calling thread when unreadable."""
    try:
        return [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        return [0]
