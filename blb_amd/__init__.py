"""blb_amd -- MI355X-native Reed-Solomon engine for blb's 8 MiB-tract durability layer.

The hot path is GF(2^8) RS encode / reconstruct / verify (klauspost/reedsolomon semantics,
as blb pins it at /root/reference/go.mod:20), done by hand-written gfx950 HIP kernels in
libblbrs.so behind the C ABI in include/blb_rs.h.  `reedsolomon` mirrors the Go Encoder
interface over that ABI; `tractserver` mirrors blb's callers of it.
"""
from . import reedsolomon  # noqa: F401
from .reedsolomon import New  # noqa: F401

__all__ = ["reedsolomon", "New"]
