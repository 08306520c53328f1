"""Synthetic PackTracts extent sets for the benches (bench.py, tools/pmc_prod.py).

A curator pack request lays tracts of any length at padToLength-aligned offsets into the data
pieces (internal/curator/pack_tracts.go:124-169); the tractserver reads each tract into its own
RPC buffer and copies it in (internal/tractserver/store.go:922-994).  So on the device every tract
is its own source bytes.  Two source sets are built here over the same layout:

  shared    every tract is a window of one 4 GiB pool at a random offset (round 2-4's bench):
            windows overlap, so part of the reads can be served by L2 / MALL instead of HBM;
  distinct  every tract has its own bytes, each at the start of its own page-aligned buffer (the
            RPC buffer CtlRead returns, store.go:956-959), in a shuffled order, so every byte
            read is a distinct HBM byte -- the traffic the algorithmic count assumes.  Within a
            piece, tract j lands at a multiple of padToLength = 64 KiB - 4, so its source is
            (-offset) mod 16 in {0, 4, 8, 12} bytes off the piece's 16-byte grid, as in blb.
            jitter=True adds 0-15 more bytes (rounds 4-5 PMC runs: a harsher, non-blb layout).
"""
from __future__ import annotations

import numpy as np

PAD_TO_LENGTH = 64 * 1024 - 4  # internal/curator/pack_tracts.go:27


def padded_length(n: int) -> int:
    return (n + PAD_TO_LENGTH - 1) // PAD_TO_LENGTH * PAD_TO_LENGTH


def layout(npieces: int, S: int, prng, lo: int = 64 << 10, hi: int = 8 << 20) -> list:
    """(piece, offset, length) for tracts of lo..hi bytes laid end to end (padded) into each of
    `npieces` pieces of S bytes, sorted by (piece, offset)."""
    out = []
    for p in range(npieces):
        off = 0
        while True:
            ln = int(prng.integers(lo, hi + 1))
            if off + ln > S:
                break
            out.append((p, off, ln))
            off += padded_length(ln)
    return out


def distinct_sources(lay: list, dev, gen, prng, jitter: bool = False):
    """One device pool holding every tract's own bytes; returns (pool, [start of tract i])."""
    import torch
    align = 256 if jitter else 4096
    slots = [(ln + 16 + align - 1) // align * align for _, _, ln in lay]
    pool = torch.empty(sum(slots) + 4096, dtype=torch.uint8, device=dev)
    pool.random_(0, 256, generator=gen)
    starts, pos = [0] * len(lay), 0
    for i in prng.permutation(len(lay)):
        starts[i] = pos + (int(prng.integers(0, 16)) if jitter else 0)
        pos += slots[i]
    return pool, starts


def shared_sources(lay: list, pool_bytes: int, dev, prng):
    """A `pool_bytes` device pool and a random window start for every tract."""
    import torch
    pool = torch.randint(0, 256, (pool_bytes,), dtype=torch.uint8, device=dev)
    starts = [int(prng.integers(0, pool_bytes - ln)) for _, _, ln in lay]
    return pool, starts


def extents(lay: list, pool, starts: list, piece_of=lambda p: p) -> list:
    """(src, offset, length, piece) tuples for PackPieces / PackEncode."""
    return [(pool[starts[i]:], off, ln, piece_of(p)) for i, (p, off, ln) in enumerate(lay)]
