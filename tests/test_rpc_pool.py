"""Buffer lifetime and host-path shapes at the drop-in boundary:

  * rpc.GetBuffer / PutBuffer (pkg/rpc/pool.go:16-62) as the Go shim builds them
    (blb_amd/rpc.py = go/rsgpu/rsgpu.go): Go-heap-style buffers pinned by registration and
    unpinned when collected, so blb's drop-without-PutBuffer pattern (client/blb/
    reconstruct.go:126-152 stragglers, bulk_codec.go:212-221 read errors) cannot strand
    pinned memory, and a live limit bounds what is pinned at once;
  * per-slot zero copy: pinned, pageable and device shards mixed in one host call;
  * the host CRC call's staging stays within the worker bound for any length;
  * device-list lanes balanced by bytes in flight.

Every coding result is compared with the oracle restatement (oracle/)."""
import ctypes
import gc
import threading
import time

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401
from blb_amd import _lib, rpc
from blb_amd import reedsolomon as rs
from blb_amd.blbcore import Error
from blb_amd.hostcopy import to_numpy, from_numpy_pinned

MIB = 1 << 20


# ---------------------------------------------------------------- CPU: pool logic

def test_rpc_pool_classes_like_pool_go():
    """pool.go's size rules: small and large requests are plain buffers; class buffers come
    back from the pool after an exclusive Put; non-exclusive and mid-buffer Puts are ignored."""
    small = rpc.GetBuffer(rpc.SMALL_MAX)
    assert small.size == rpc.SMALL_MAX and rpc._class_base(small) is None
    big = rpc.GetBuffer(rpc.CLASSES[-1] + 1)
    assert big.size == rpc.CLASSES[-1] + 1 and rpc._class_base(big) is None
    a = rpc.GetBuffer(rpc.SMALL_MAX + 1)                 # -> the 1 MiB class
    base = rpc._class_base(a)
    assert base is not None and base.size == rpc.CLASSES[0] and base.ctypes.data % 4096 == 0
    rpc.PutBuffer(a[1:], True)                          # not at the base: cap != class
    rpc.PutBuffer(a, False)                             # not exclusive
    b = rpc.GetBuffer(4096 + rpc.SMALL_MAX)
    assert b.ctypes.data != a.ctypes.data
    rpc.PutBuffer(a, True)
    c = rpc.GetBuffer(rpc.CLASSES[0])
    assert c.ctypes.data == a.ctypes.data               # reused
    d = rpc.GetBuffer(4 * MIB)
    assert rpc._class_base(d).size == rpc.CLASSES[1]
    rpc.gc()


def test_rpc_pool_small_class_opt_in():
    """set_pool_small(True): requests of up to 128 KiB + ExtraRoom come from a pool of their own
    class (reused after an exclusive Put); with it off (pool.go's rule, the default) they are
    plain buffers again."""
    try:
        rpc.set_pool_small(True)
        a = rpc.GetBuffer(4096)
        base = rpc._class_base(a)
        assert base is not None and base.size == rpc.SMALL_MAX and a.size == 4096
        rpc.PutBuffer(a, True)
        b = rpc.GetBuffer(rpc.SMALL_MAX)
        assert b.ctypes.data == a.ctypes.data and b.size == rpc.SMALL_MAX   # reused
        assert rpc.GetBuffer(0).size == 0
    finally:
        rpc.set_pool_small(False)
        rpc.gc()
    assert rpc._class_base(rpc.GetBuffer(4096)) is None


def test_pool_live_limit_refuses_before_pinning():
    """blbrs_buffer_get past the live limit is ErrLimit (checked before any allocation, so this
    runs without a GPU); registration with no device releases its reservation."""
    lib = _lib.load()
    try:
        rs.set_live_limit(2 * MIB)
        before = rs.pool_stats()
        p, cap = ctypes.c_void_p(), ctypes.c_size_t()
        assert lib.blbrs_buffer_get(4 * MIB, ctypes.byref(p), ctypes.byref(cap)) == rs.ErrLimit.code
        assert p.value is None
        st = rs.pool_stats()
        assert st["limit_rejects"] == before["limit_rejects"] + 1 and st["live_limit"] == 2 * MIB
        buf = np.empty(3 * MIB, np.uint8)
        assert lib.blbrs_buffer_register(buf.ctypes.data, buf.size) == rs.ErrLimit.code
        assert lib.blbrs_buffer_unregister(buf.ctypes.data) == rs.ErrInvalidArgument.code
        assert lib.blbrs_buffer_register(None, 10) == rs.ErrInvalidArgument.code
        assert rs.pool_stats()["registered_bytes"] == before["registered_bytes"]
    finally:
        rs.set_live_limit(16 << 30)
    assert rs.ErrLimit.code == -10 and lib.blbrs_strerror(-10) == b"pinned-memory live limit reached"


def test_rpc_pool_without_gpu_stays_pageable():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    before = dict(rpc.stats)
    a = rpc.GetBuffer(2 * MIB)
    assert not rpc.is_pinned(a) and rpc.stats["refused"] == before["refused"] + 1
    a[:] = 7   # a working buffer all the same
    rpc.PutBuffer(a, True)
    rpc.gc()


# ---------------------------------------------------------------- GPU helpers

def _oracle_stripe(O, k, m, S, rng):
    sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
    O.encode(k, m, sh)
    return sh


class _Slots:
    """Buffers of one kind per slot: 'page' (numpy), 'pin' (blbrs_buffer_get), 'reg'
    (rpc.GetBuffer, registered) or 'dev' (torch CUDA)."""

    def __init__(self, kinds, S):
        import torch
        self.kinds, self.S, self.bufs, self.ptrs = kinds, S, [], []
        for kd in kinds:
            if kd == "page":
                b = np.empty(S, np.uint8)
                p = b.ctypes.data
            elif kd == "pin":
                b = rs.GetBuffer(S)
                p = b.ctypes.data
            elif kd == "reg":
                b = rpc.GetBuffer(max(S, rpc.SMALL_MAX + 1))[:S]
                p = b.ctypes.data
            else:
                b = torch.empty(S, dtype=torch.uint8, device="cuda:0")
                p = b.data_ptr()
            self.bufs.append(b)
            self.ptrs.append(p)

    def put(self, i, host):
        import torch
        b = self.bufs[i]
        if self.kinds[i] == "dev":
            b.copy_(from_numpy_pinned(host))
        else:
            b[:] = host

    def get(self, i):
        b = self.bufs[i]
        return to_numpy(b) if self.kinds[i] == "dev" else b.copy()

    def poison(self, i):
        import torch
        if self.kinds[i] == "dev":
            self.bufs[i].fill_(0xA5)
        else:
            self.bufs[i][:] = 0xA5

    def close(self):
        import torch
        torch.cuda.synchronize()
        for kd, b in zip(self.kinds, self.bufs):
            if kd == "pin":
                rs.PutBuffer(b)
            elif kd == "reg":
                rpc.PutBuffer(b, True)
        self.bufs = []


# ---------------------------------------------------------------- GPU: mixed slots

@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True])
def test_mixed_slot_kinds_vs_oracle(oracle_lib, batched):
    """Encode / Reconstruct / ReconstructData / reconstructAndVerify with every shard slot drawn
    from pinned, registered, pageable and device memory in one call (the client's degraded read
    is k pool buffers + the user's pageable thisB, reconstruct.go:172-173).  Pinned and device
    slots are coded in place, pageable ones staged; bytes are the oracle's."""
    import torch
    lib = _lib.load()
    k, m = 6, 3
    n = k + m
    enc = rs.New(k, m, devices=[0])
    b = rs.Batcher(max_batch=16, window_us=0, devices=[0]) if batched else None
    if b is not None:
        enc.SetBatcher(b)
    rng = np.random.default_rng(31 + batched)
    kinds_all = ["page", "pin", "reg", "dev"]
    sizes = [4096 + 16, 1 * MIB, 3 * MIB + 48, 8 * MIB] if not batched else [4096 + 16, 1 * MIB, 3 * MIB + 48]
    patterns = [["pin"] * k + ["page"], None, ["page"] * n, ["dev"] + ["pin"] * (n - 2) + ["page"]]
    try:
        for S in sizes:
            for pi, pat in enumerate(patterns):
                kinds = list(pat) if pat else [kinds_all[x] for x in rng.integers(0, 4, n)]
                kinds = (kinds * n)[:n]
                ref = _oracle_stripe(oracle_lib, k, m, S, rng)
                sl = _Slots(kinds, S)
                try:
                    ptrs = (ctypes.c_void_p * n)(*sl.ptrs)
                    # Encode
                    for i in range(k):
                        sl.put(i, ref[i])
                    for i in range(k, n):
                        sl.poison(i)
                    torch.cuda.synchronize()
                    lens = (ctypes.c_size_t * n)(*([S] * n))
                    assert lib.blbrs_encode(enc._h, ptrs, lens) == 0, lib.blbrs_last_error()
                    for i in range(k, n):
                        assert np.array_equal(sl.get(i), ref[i]), (S, kinds, "encode", i)
                    # Reconstruct (data 1 + parity 7) and ReconstructData (data 2 + 4)
                    for lost, fn in (((1, 7), lib.blbrs_reconstruct), ((2, 4), lib.blbrs_reconstruct_data)):
                        for i in lost:
                            sl.poison(i)
                        torch.cuda.synchronize()
                        lens = (ctypes.c_size_t * n)(*[0 if i in lost else S for i in range(n)])
                        assert fn(enc._h, ptrs, lens) == 0, lib.blbrs_last_error()
                        for i in lost:
                            assert np.array_equal(sl.get(i), ref[i]), (S, kinds, lost, i)
                            assert lens[i] == S
                    # reconstructAndVerify: consistent, then with a corrupted survivor
                    for corrupt in (False, True):
                        sl.poison(0)
                        if corrupt:
                            bad = ref[8].copy()
                            bad[S // 2] ^= 1
                            sl.put(8, bad)
                        torch.cuda.synchronize()
                        lens = (ctypes.c_size_t * n)(*[0 if i == 0 else S for i in range(n)])
                        ok = ctypes.c_int(-1)
                        assert lib.blbrs_reconstruct_verify(enc._h, ptrs, lens, ctypes.byref(ok)) == 0
                        assert np.array_equal(sl.get(0), ref[0])
                        assert ok.value == (0 if corrupt else 1), (S, kinds, corrupt)
                        sl.put(8, ref[8])
                finally:
                    sl.close()
        if b is not None:
            r, launches = b.stats()
            assert r > 0 and launches > 0
    finally:
        if b is not None:
            enc.SetBatcher(None)
            b.close()
        rpc.gc()
        gc.collect()


# ---------------------------------------------------------------- GPU: pool lifetime

class _PoolReader:
    """A tractserver talker whose Read replies come from rpc.GetBuffer, as gob/bulk_codec
    decodes them (bulk_codec.go:210-213).  Hosts in `failing` take a buffer and then fail
    (bulk_codec.go:212-221 returns with it); hosts in `slow` answer late (stragglers after
    reconstruct.go:154's cancel).  `held` keeps every handed-out buffer reachable until
    collect() -- a GC that has not run yet."""

    def __init__(self, pieces, failing=(), slow=(), hold=False):
        self.pieces, self.failing, self.slow, self.hold = pieces, set(failing), set(slow), hold
        self.held, self.lock = [], threading.Lock()

    def read(self, addr, tid, version, length, off):
        b = rpc.GetBuffer(length)
        if self.hold:
            with self.lock:
                self.held.append(b)
        if addr in self.failing:
            return None, Error.ErrRPC       # the buffer is dropped
        if addr in self.slow:
            time.sleep(0.002)
        b[:] = self.pieces[addr][off:off + length]
        return b, Error.NoError

    def read_into(self, addr, tid, version, b, off):
        return 0, Error.ErrRPC               # the direct read fails: reconstruct

    def collect(self):
        with self.lock:
            self.held.clear()


@pytest.mark.gpu
def test_pool_small_replies_coded_in_place():
    """With small replies pooled (rpc.set_pool_small), a 64 KiB degraded read's replies are
    registered buffers -- coded in place, not staged -- and the rebuilt piece is bit-exact
    against the restatement."""
    from oracle import rs_numpy as N
    k, m, S = 6, 3, 64 << 10
    rng = np.random.default_rng(64)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    full = data + list(N.encode(k, m, data))
    try:
        rpc.set_pool_small(True)
        sh = []
        for i in range(k + m):
            b = rpc.GetBuffer(S)
            b[:] = full[i]
            sh.append(b)
        assert all(rpc.is_pinned(b) for b in sh)
        enc = rs.New(k, m)
        for lost in (1, 4):
            work = list(sh)
            work[lost] = None
            enc.ReconstructData(work)
            assert np.array_equal(work[lost], full[lost]), lost
        for b in sh:
            rpc.PutBuffer(b, True)
    finally:
        rpc.set_pool_small(False)
        rpc.gc()


@pytest.mark.gpu
@pytest.mark.parametrize("delayed_gc", [False, True])
def test_degraded_reads_drop_buffers_pinned_bounded(oracle_lib, delayed_gc):
    """reconstruct.go:126-152's pattern, thousands of times: every degraded read takes n+m-1
    pool buffers, PutBuffers only the first n good replies and drops the failed and straggling
    ones.  Pinned live bytes never exceed the limit, every dropped buffer is unpinned once
    collected (nothing stays registered after the pools are drained), and every read is
    bit-exact against the oracle's bytes.  delayed_gc: dropped buffers stay reachable for 100
    reads (a GC that runs late), so the limit is hit and the overflow is coded from pageable
    buffers -- still exact."""
    from blb_amd.client import Client, ReconstructBehavior
    from test_callers import rs_tract
    n, m, target = 6, 3, 2
    S, length = 4 * MIB, 300 << 10                      # replies land in the 1 MiB class
    limit = (24 if delayed_gc else 64) * MIB
    rng = np.random.default_rng(4711 + delayed_gc)
    shards = _oracle_stripe(oracle_lib, n, m, S, rng)
    pieces = {f"ts{i}": shards[i] for i in range(n + m)}
    reader = _PoolReader(pieces, failing={"ts5"}, slow={"ts0"}, hold=delayed_gc)
    cli = Client(reader, ReconstructBehavior(enabled=True, max_in_flight=8))
    tr = rs_tract(n, m, target)
    reads = 2000
    rs.set_live_limit(limit)
    rpc.gc()
    gc.collect()
    st0 = rs.pool_stats()
    r0 = dict(rpc.stats)
    peak = [0]
    errors = []

    def worker(t):
        try:
            g = np.random.default_rng(t)
            for it in range(reads // 8):
                off = int(g.integers(0, S - length)) & ~3
                buf = np.full(length, 0xEE, np.uint8)     # the user's pageable Blob.ReadAt buffer
                res = cli.read_one_tract_rs(tr, buf, off)
                if res.err != Error.NoError or res.read != length:
                    errors.append((t, it, res))
                    return
                if not np.array_equal(buf, shards[target][off:off + length]):
                    errors.append((t, it, "bytes differ"))
                    return
                live = rs.pool_stats()["registered_bytes"]
                peak[0] = max(peak[0], live)
                if delayed_gc and it % 100 == 99 and t == 0:
                    reader.collect()
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:3]
        assert cli.reconstructs == reads
        assert peak[0] <= limit, (peak[0], limit)
        st = rs.pool_stats()
        assert st["registered_bytes"] <= limit
        assert rpc.stats["registered"] - r0["registered"] > 0            # pool buffers were pinned
        if delayed_gc:
            assert st["limit_rejects"] > st0["limit_rejects"]            # the limit was reached
            assert rpc.stats["refused"] > r0["refused"]
        reader.collect()
    finally:
        rs.set_live_limit(16 << 30)
    # Drain the pools (a GC cycle) and collect: every registration is undone.
    cli._pool.shutdown(wait=True)
    del cli
    rpc.gc()
    gc.collect()
    assert rs.pool_stats()["registered_bytes"] == st0["registered_bytes"] == 0, rs.pool_stats()
    # every registration (first ones and re-registrations of reused pageable buffers) undone
    assert rpc.stats["unregistered"] - r0["unregistered"] == rpc.stats["registered"] - r0["registered"]


# ---------------------------------------------------------------- GPU: host CRC staging

@pytest.mark.gpu
@pytest.mark.parametrize("length,block", [(64 * MIB, 65532), (64 * MIB + 13, 0), (40 * MIB + 8, 24 * MIB)])
def test_host_crc_pageable_staging_bounded(oracle_lib, length, block):
    """blbrs_crc32c on a pageable buffer larger than a ring slot: chunks of <= 16 MiB keep the
    worker's staging within blb_rs.h's bound, and every block CRC equals the oracle's
    crc32.Checksum (whole-buffer frame, 65532-byte ChecksumFile blocks, a block longer than a
    chunk)."""
    from blb_amd import checksum
    rs.trim()
    rng = np.random.default_rng(length)
    buf = rng.integers(0, 256, length, dtype=np.uint8)
    got = np.asarray(checksum.Checksum(buf, block), dtype=np.uint32)
    want = np.asarray(oracle_lib.crc32c_blocks(buf, block or length), dtype=np.uint32)
    assert np.array_equal(got, want)
    st = rs.device_stats(0)
    assert st["staging_bytes"] <= max(1, st["workers"]) * 2 * (16 * MIB), st
    assert st["staging_bytes"] <= 16 * MIB, st        # one call, one worker, one slot


# ---------------------------------------------------------------- GPU: lanes by bytes

@pytest.mark.gpu
def test_lanes_balance_bytes_in_flight(oracle_lib):
    """[0, 0] (two lanes on GPU 0): concurrent 4 KiB and 8 MiB host calls are routed by shard
    bytes in flight, so both lanes carry a similar byte load (within 2x), and every result is
    the oracle's.  (One GPU here: the routing is measured, the 8-GPU spread is not.)"""
    k, m = 6, 3
    enc = rs.New(k, m, devices=[0, 0])
    before = [enc.LaneStats(i) for i in range(2)]
    big = [rs.GetBuffer(8 * MIB) for _ in range(4 * (k + m))]
    errors = []

    def worker(t):
        try:
            g = np.random.default_rng(t)
            for it in range(12):
                if t < 4:
                    sh = big[t * (k + m):(t + 1) * (k + m)]
                    if it == 0:
                        for i in range(k):
                            sh[i][:] = g.integers(0, 256, 8 * MIB, dtype=np.uint8)
                else:
                    sh = [g.integers(0, 256, 4096, dtype=np.uint8) for _ in range(k)] + \
                         [np.empty(4096, np.uint8) for _ in range(m)]
                for i in range(k, k + m):
                    sh[i][:] = 0xA5
                enc.Encode(sh)
                if it == 0 or (t >= 4 and it % 4 == 0):
                    ref = [s.copy() for s in sh[:k]] + [np.zeros(sh[0].size, np.uint8) for _ in range(m)]
                    oracle_lib.encode(k, m, ref)
                    for i in range(k, k + m):
                        if not np.array_equal(sh[i], ref[i]):
                            errors.append((t, it, i))
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        for b in big:
            rs.PutBuffer(b)
    assert not errors, errors[:3]
    after = [enc.LaneStats(i) for i in range(2)]
    got = [after[i]["bytes"] - before[i]["bytes"] for i in range(2)]
    calls = [after[i]["calls"] - before[i]["calls"] for i in range(2)]
    assert sum(calls) == 12 * 12
    assert min(got) > 0 and max(got) <= 2 * min(got), (got, calls)
    assert all(after[i]["inflight_calls"] == 0 and after[i]["inflight_bytes"] == 0 for i in range(2))
