"""Host <-> device copies that never hand pageable memory to HIP.

HIP copies a pageable source or destination larger than 1 MiB by locking the caller's pages in
place for the DMA (hsa_amd_memory_lock_to_pool over the page-rounded range; AMD_LOG_LEVEL=4
logs "Locking to pool ... memFlags = 0x8h" then "HSA Copy Using Pinned resource",
profiles/r06/fault/).  Every GPU memory fault of round 5 whose log survives was raised in
such a copy made by test code (torch's .cuda() / .cpu() of a 1.4 MB heap array,
tests/test_rtc.py), and the library itself never takes that path: its host calls stage pageable shards by CPU copies into pinned,
device-mapped buffers (blbrs.hip host_run).  These helpers give the Python side the same rule:
numpy data goes through a pinned torch tensor (hipHostMalloc memory, which HIP copies with no
lock), in both directions.  tests/test_no_inplace_pin.py checks the rule from HIP's own log.
"""
from __future__ import annotations

import numpy as np


def to_device(a, device="cuda"):
    """numpy array (any layout) -> a new device tensor, through pinned host memory."""
    import torch
    src = torch.from_numpy(np.ascontiguousarray(a))
    staged = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
    staged.copy_(src)                         # CPU copy into the pinned block
    return staged.to(device)                  # blocking DMA from pinned memory


def to_numpy(t) -> np.ndarray:
    """device (or CPU) tensor -> numpy array, through pinned host memory.  The result is a
    plain (pageable) array, the same kind of memory .cpu().numpy() returns, so a caller that
    hands it to the library still exercises the library's pageable-shard path."""
    import torch
    if not t.is_cuda:
        return t.numpy()
    out = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    out.copy_(t)                              # blocking DMA into pinned memory
    return out.numpy().copy()


def from_numpy_pinned(a):
    """numpy array -> a pinned CPU tensor (a source for device tensor .copy_())."""
    import torch
    src = torch.from_numpy(np.ascontiguousarray(a))
    staged = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
    staged.copy_(src)
    return staged
