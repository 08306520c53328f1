"""CRC-32C (Castagnoli) of shard blocks on the GPU.

blb checksums every shard written on the RS path: ChecksumFile stores 64 KiB blocks of
65532 data bytes plus a CRC-32C each (pkg/disk/checksum_block.go:18-34,70-80), and the bulk
RPC codec appends a CRC-32C of the whole bulk buffer (pkg/rpc/bulk_codec.go:6-14,47).
Results equal Go's crc32.Checksum(block, crc32.MakeTable(crc32.Castagnoli)).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .hostcopy import to_numpy
from .reedsolomon import ErrInvalidArgument, _check, _is_torch, _torch_stream

CHECKSUM_BLOCK_DATA = 64 * 1024 - 4  # pkg/disk/checksum_block.go:21-29 blockDataLength


def Checksum(data, block: int = 0):
    """CRC-32C of each `block`-byte block of `data` (block 0 = the whole buffer).
    numpy uint8 (host) -> numpy uint32 array; torch.uint8 CUDA tensor -> torch.int32 CUDA
    tensor holding the CRC bits (async on the current stream)."""
    lib = _lib.load()
    if _is_torch(data):
        import torch
        if data.dim() != 1 or data.dtype != torch.uint8 or not data.is_cuda:
            raise ErrInvalidArgument("expected a 1-D torch.uint8 CUDA tensor")
        return ChecksumBatch(data.view(1, -1), block).view(-1)
    a = np.ascontiguousarray(data, dtype=np.uint8)
    n = a.size
    if n == 0:
        return np.zeros(0, np.uint32)
    blk = block or n
    out = np.zeros((n + blk - 1) // blk, np.uint32)
    _check(lib.blbrs_crc32c(a.ctypes.data, n, blk, out.ctypes.data))
    return out


def ChecksumBatch(buffers, block: int = 0, phase: int = 0, seeds=None):
    """[B, len] torch.uint8 CUDA tensor (rows may be strided) -> [B, nblocks] torch.int32
    CRC bits, computed on the device on the current stream.

    phase / seeds (blbrs_crc32c_dev_at): each row is a window of a file whose byte 0 sits
    `phase` bytes into a `block`-byte block; nblocks = ceil((phase + len) / block) and entry
    0 continues seeds[b] (crc32.Update, pkg/disk/checksum_block.go:80).  seeds: [B] int32
    CUDA tensor of CRC bits or None."""
    import torch
    if not (_is_torch(buffers) and buffers.is_cuda and buffers.dtype == torch.uint8 and buffers.dim() == 2):
        raise ErrInvalidArgument("expected a [B, len] torch.uint8 CUDA tensor")
    B, n = buffers.shape
    if n > 1 and buffers.stride(1) != 1:
        raise ErrInvalidArgument("row bytes must be contiguous")
    if not block:
        phase = 0
    blk = block or max(n, 1)
    nb = (n + phase + blk - 1) // blk
    out = torch.empty((B, nb), dtype=torch.int32, device=buffers.device)
    sp = _seeds_ptr(seeds, B, buffers.device)
    if B and n:
        _check(_lib.load().blbrs_crc32c_dev_at(buffers.data_ptr(), buffers.stride(0), B, n, blk, phase, sp,
                                               out.data_ptr(), _torch_stream(buffers)))
    return out


def _seeds_ptr(seeds, count: int, device):
    import torch
    if seeds is None:
        return None
    if not (_is_torch(seeds) and seeds.is_cuda and seeds.dtype == torch.int32 and seeds.is_contiguous()
            and seeds.numel() == count and seeds.device == device):
        raise ErrInvalidArgument(f"seeds must be a contiguous int32 CUDA tensor of {count} entries")
    return seeds.data_ptr()


def as_uint32(t) -> np.ndarray:
    """CRC bits from a torch.int32 tensor as numpy uint32 (copied out through pinned memory,
    hostcopy.py)."""
    return to_numpy(t).view(np.uint32)
