"""PackTracts on the GPU: the step before RS encode that lays out the
data pieces the encoder reads.

* `pack_tracts(tracts, target)` is the curator's first-fit-decreasing bin packing
  (internal/curator/pack_tracts.go:124-169): tracts sorted by length (largest first),
  each padded to a multiple of padToLength = 64 KiB - 4 (the ChecksumFile block data
  size, :27), placed in the first chunk with room under `target`; chunks sorted by
  length, and only those with at most acceptSlop = 10 % empty space (:23) are kept.
* `PackPieces(dst, piece_len, extents)` is the byte work of Store.PackTracts
  (internal/tractserver/store.go:922-994) on the device, for many pieces at once:
  each tract lands at its offset, every other byte is zero (holes and the tail pad,
  store.go:974-980).  It runs in `blbrs_pack_dev`; there is no CPU fallback.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _lib
from .blbcore import TractID
from .reedsolomon import ErrInvalidArgument, _check, _is_torch, _torch_stream

PAD_TO_LENGTH = 64 * 1024 - 4   # internal/curator/pack_tracts.go:27 padToLength
ACCEPT_SLOP = 0.10              # internal/curator/pack_tracts.go:23 acceptSlop

EXTENT_DTYPE = np.dtype([("src", np.uint64), ("offset", np.uint64), ("length", np.uint64),
                         ("piece", np.uint64)])  # blbrs_pack_extent


@dataclass
class PackTractSpec:
    """internal/core/tractserver_messages.go:117-123."""
    id: TractID
    from_: list = field(default_factory=list)   # []TSAddr
    version: int = 0
    offset: int = -1
    length: int = -1


@dataclass
class PackedChunk:
    """internal/curator/pack_tracts.go:378-381."""
    tracts: list
    length: int


def padded_length(n: int) -> int:
    return (n + PAD_TO_LENGTH - 1) // PAD_TO_LENGTH * PAD_TO_LENGTH


def pack_tracts(tracts: Sequence[PackTractSpec], target: int) -> list[PackedChunk]:
    """tractPacker.packTracts (pack_tracts.go:124-169).  Sets each placed tract's .offset;
    returns the accepted chunks, fullest first.  Sorting is stable (Go's sort.Sort is not;
    ties between equal lengths may be ordered differently there, which changes which
    equal-length tract lands where but not any chunk's length)."""
    chunks: list[PackedChunk] = []
    for t in sorted(tracts, key=lambda t: -t.length):
        if t.length < 0:
            break  # could not stat it: skip it and the rest (sorted) -- :137-139
        pl = padded_length(t.length)
        for c in chunks:
            if c.length + pl <= target:
                t.offset = c.length
                c.length += pl
                c.tracts.append(t)
                break
        else:
            t.offset = 0
            chunks.append(PackedChunk([t], pl))
    chunks.sort(key=lambda c: -c.length)
    slop = int(np.float32(target) * np.float32(ACCEPT_SLOP))  # int(float32(target) * acceptSlop)
    idx = next((i for i, c in enumerate(chunks) if target - c.length > slop), len(chunks))
    return chunks[:idx]


def check_tract_spec(srcs: Sequence[PackTractSpec], length: int) -> bool:
    """checkTractSpec (store.go:996-1009): in order, non-overlapping, inside length."""
    end = 0
    for s in srcs:
        if not s.id.is_valid() or len(s.from_) < 1 or s.offset < end:
            return False
        end = s.offset + s.length
    return length >= end


def _addr(x) -> int:
    if _is_torch(x):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    return int(x)


def PackPieces(dst, piece_len: int, extents: Sequence[tuple], stream=None) -> None:
    """Assemble pieces on the device.  dst: [npieces, >= piece_len] torch.uint8 tensor
    (CUDA or pinned host; rows contiguous, any row stride).  extents: (src, offset, length,
    piece) tuples sorted by (piece, offset), src a CUDA or pinned torch.uint8 tensor (or
    an address) holding at least `length` bytes.  Asynchronous on `stream` (default: the
    current stream)."""
    import torch
    if not (_is_torch(dst) and dst.dtype == torch.uint8 and dst.dim() == 2):
        raise ErrInvalidArgument("dst must be a [npieces, len] torch.uint8 tensor")
    npieces, width = dst.shape
    if width < piece_len or (width > 1 and dst.stride(1) != 1):
        raise ErrInvalidArgument("dst rows must be contiguous and hold piece_len bytes")
    ex = np.zeros(len(extents), EXTENT_DTYPE)
    for i, (src, off, ln, piece) in enumerate(extents):
        if off < 0 or ln < 0 or piece < 0:
            raise ErrInvalidArgument(f"extent {i}: negative field")
        if _is_torch(src) and src.numel() < ln:
            raise ErrInvalidArgument(f"extent {i}: source shorter than its length")
        ex[i] = (_addr(src) if ln else 0, off, ln, piece)
    if stream is not None:
        s = stream
    else:
        s = _torch_stream(dst) if dst.is_cuda else torch.cuda.current_stream().cuda_stream
    _check(_lib.load().blbrs_pack_dev(dst.data_ptr(), dst.stride(0), npieces, piece_len,
                                     ex.ctypes.data if len(ex) else None, len(ex), s))


def PackEncode(enc, stripes, extents: Sequence[tuple], stream=None) -> None:
    """PackTracts fused with Encode (blbrs_pack_encode_dev): for each stripe b of a
    [B, k+m, S] CUDA tensor, data shard j is assembled from the extents of piece b*k + j
    (same (src, offset, length, piece) tuples as PackPieces, piece_len = S) and the m parity
    shards are encoded from it -- one pass over HBM.  Asynchronous on `stream`."""
    B, S, ss, bs = enc._stripes(stripes)
    ex = np.zeros(len(extents), EXTENT_DTYPE)
    for i, (src, off, ln, piece) in enumerate(extents):
        if off < 0 or ln < 0 or piece < 0:
            raise ErrInvalidArgument(f"extent {i}: negative field")
        if _is_torch(src) and src.numel() < ln:
            raise ErrInvalidArgument(f"extent {i}: source shorter than its length")
        ex[i] = (_addr(src) if ln else 0, off, ln, piece)
    s = stream if stream is not None else _torch_stream(stripes)
    _check(_lib.load().blbrs_pack_encode_dev(enc._h, stripes.data_ptr(), ss, bs, B, S,
                                            ex.ctypes.data if len(ex) else None, len(ex), s))
