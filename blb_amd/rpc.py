"""rpc.GetBuffer / rpc.PutBuffer (pkg/rpc/pool.go:16-62) as the Go shim builds them
(go/rsgpu/rsgpu.go), so the Python callers and tests follow blb's buffer lifetime rule.

blb's pool is three sync.Pools of Go-heap buffers (8, 4 and 1 MiB + disk.ExtraRoom).  A buffer
that is never PutBuffer'd is garbage-collected, and blb relies on that: reconstruct.go:126-152
puts back only the first n good replies (errored and straggling ones are dropped), and
bulk_codec.go:212-221 returns on a read error with the buffer it took.  So the pinned drop-in
cannot hand out library-owned pinned memory (nothing would ever free a dropped buffer).  It
keeps blb's pool as it is and pins the buffers the pool creates instead:

  * GetBuffer(n): n <= 128 KiB + ExtraRoom or above the 8 MiB class -> a plain buffer, as in
    pool.go (never pinned); otherwise a buffer of the class from its pool.  A new buffer is
    page-aligned host memory the caller's runtime owns, registered with blbrs_buffer_register
    (pinned, mapped for every GPU: shards on it are coded in place, zero-copy).  Its owner
    carries a finalizer that unregisters it, so a dropped buffer is unpinned when it is
    collected (Go: runtime.SetFinalizer on the backing array; here weakref.finalize on the
    owning numpy array, which CPython runs when the last view is dropped).
  * Registration counts against the library's live limit (blbrs_pool_set_live_limit).  Past
    it the registration is refused (ErrLimit) and the buffer stays pageable -- correct, only
    staged; a pooled buffer that is still pageable is registered again when it is reused.
  * PutBuffer(b, exclusive): as pool.go -- only exclusive buffers of a class capacity (a slice
    that starts at the buffer's base) go back to their pool.  It is fine to call on any
    buffer.
  * gc(): what a Go GC cycle does to a sync.Pool -- the idle buffers are dropped (and so
    unregistered once nothing else holds them).
  * set_pool_small(True) (off by default, as in pool.go): requests of up to 128 KiB + ExtraRoom
    also come from a pool of registered buffers of that size, so small replies are coded in
    place instead of staged by CPU copies (a 64 KiB degraded read 31 -> 25 us, 128 KiB
    53 -> 41 us cold).  The Go shim's rsgpu.SetPoolSmall is the same.
"""
from __future__ import annotations

import threading
import time
import weakref

import numpy as np

from . import _lib

EXTRA_ROOM = 64 << 10                    # disk.ExtraRoom (pkg/disk/checksum_file.go:27)
SMALL_MAX = (128 << 10) + EXTRA_ROOM     # pool.go:31: "Don't bother with pools for small buffers."
CLASSES = ((1 << 20) + EXTRA_ROOM, (4 << 20) + EXTRA_ROOM, (8 << 20) + EXTRA_ROOM)
_PAGE = 4096

# Reentrant: a finalizer (_unregister) runs whenever the last view of a buffer is dropped,
# which can happen while this thread holds the lock.
_mu = threading.RLock()
_free: dict[int, list] = {c: [] for c in CLASSES + (SMALL_MAX,)}   # sync.Pool contents per class
_pool_small = False                                 # set_pool_small
_pinned: set[int] = set()                           # base addresses currently registered
stats = {"registered": 0, "refused": 0, "unregistered": 0, "reregistered": 0,
         "register_s": 0.0, "unregister_s": 0.0}   # wall time inside blbrs_buffer_(un)register


def _unregister(addr: int) -> None:
    with _mu:
        if addr not in _pinned:
            return
        _pinned.discard(addr)
        stats["unregistered"] += 1
    t0 = time.perf_counter()
    _lib.load().blbrs_buffer_unregister(addr)
    with _mu:
        stats["unregister_s"] += time.perf_counter() - t0


def _register(base: np.ndarray) -> bool:
    addr = base.ctypes.data
    t0 = time.perf_counter()
    rc = _lib.load().blbrs_buffer_register(addr, base.size)
    dt = time.perf_counter() - t0
    if rc != 0:
        with _mu:
            stats["refused"] += 1
        return False
    with _mu:
        _pinned.add(addr)
        stats["registered"] += 1
        stats["register_s"] += dt
    return True


def _new_buffer(size: int) -> np.ndarray:
    """A page-aligned class buffer, registered when the live limit allows."""
    raw = np.empty(size + _PAGE, np.uint8)
    off = (-raw.ctypes.data) % _PAGE
    base = raw[off:off + size]
    if _register(base):
        # Unregister before the memory is freed: runs when `raw` (the owner every view keeps
        # alive) is collected, before numpy releases its data.
        weakref.finalize(raw, _unregister, base.ctypes.data)
    return base


def _class_base(b: np.ndarray):
    """The class buffer `b` starts at (Go: cap(b) == a class size), else None."""
    owner = b.base if isinstance(b.base, np.ndarray) else b
    size = owner.size - _PAGE
    if owner.ndim != 1 or size not in _free:
        return None
    off = (-owner.ctypes.data) % _PAGE
    if b.ctypes.data != owner.ctypes.data + off:
        return None
    return owner[off:off + size]


def set_pool_small(on: bool) -> None:
    """Pool (and pin) requests of up to 128 KiB + ExtraRoom too; off restores pool.go's plain
    buffers for them (buffers already handed out keep their class)."""
    global _pool_small
    _pool_small = bool(on)


def GetBuffer(n: int) -> np.ndarray:
    """A []byte with length n; NOT zeroed (pool.go:28-43)."""
    if n <= 0 or (n <= SMALL_MAX and not _pool_small) or n > CLASSES[-1]:
        return np.empty(max(n, 0), np.uint8)
    size = SMALL_MAX if n <= SMALL_MAX else next(c for c in CLASSES if n <= c)
    with _mu:
        base = _free[size].pop() if _free[size] else None
        again = base is not None and base.ctypes.data not in _pinned
    if base is None:
        base = _new_buffer(size)
    elif again and _register(base):
        with _mu:
            stats["reregistered"] += 1
        weakref.finalize(base.base, _unregister, base.ctypes.data)
    return base[:n]


def PutBuffer(b: np.ndarray, exclusive: bool = True) -> None:
    """pool.go:45-62: exclusive class buffers go back to their pool; anything else is left
    to the collector."""
    if not exclusive or b is None:
        return
    base = _class_base(b)
    if base is None:
        return
    with _mu:
        _free[base.size].append(base)


def is_pinned(b: np.ndarray) -> bool:
    """True when b lies in a buffer registered by this pool (coded zero-copy)."""
    base = _class_base(b)
    return base is not None and base.ctypes.data in _pinned


def gc() -> None:
    """A GC cycle's effect on the pools: idle buffers are dropped."""
    with _mu:
        dropped = [_free[c][:] for c in _free]
        for c in _free:
            _free[c].clear()
    del dropped  # collected (and unregistered) outside the lock
