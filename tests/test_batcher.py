"""Batched client reconstructs.  client/blb/reconstruct.go:65-195 runs
one `reedsolomon.New(n, m)` + `ReconstructData` per degraded read, up to MaxInFlight at
once; with a Batcher attached, concurrent calls share kernel launches.  Results must be
byte-identical to the unbatched path / the oracle, and errors unchanged."""
import threading

import numpy as np
import pytest

from blb_amd import reedsolomon
from oracle import rs_numpy as N

pytestmark = pytest.mark.gpu


def _torch():
    return pytest.importorskip("torch")


def _stripe(rng, k, m, size):
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    return data + N.encode(k, m, data)


def test_batched_concurrent_reconstructs_match_oracle():
    torch = _torch()
    k, m = 6, 3
    rng = np.random.default_rng(42)
    sizes = [4096, 65536, 100_001]
    patterns = [(1,), (0, 7), (2, 4, 5), (8,)]
    stripes = {s: _stripe(rng, k, m, s) for s in sizes}
    pinned = {s: [torch.from_numpy(x).pin_memory().numpy() for x in stripes[s]] for s in sizes}
    b = reedsolomon.Batcher(max_batch=32, window_us=2000)
    errors, calls = [], [0]
    lock = threading.Lock()

    def client(tid):
        r = np.random.default_rng(tid)
        for it in range(8):
            size = sizes[(tid + it) % len(sizes)]
            erased = patterns[(tid * 3 + it) % len(patterns)]
            src = pinned[size] if (tid + it) % 2 else stripes[size]
            data_only = bool(r.integers(0, 2))
            enc = reedsolomon.New(k, m)   # a fresh encoder per read, as reconstruct.go:172 does
            enc.SetBatcher(b)
            shards = [None if i in erased else src[i] for i in range(k + m)]
            try:
                (enc.ReconstructData if data_only else enc.Reconstruct)(shards)
                for i in range(k + m):
                    if i in erased and (i < k or not data_only):
                        assert np.array_equal(shards[i], stripes[size][i]), (tid, it, i)
                    elif i in erased:
                        assert shards[i] is None
            except Exception as e:  # noqa: BLE001 -- collected and re-raised on the main thread
                errors.append(e)
            finally:
                enc.SetBatcher(None)
            with lock:
                calls[0] += 1

    ths = [threading.Thread(target=client, args=(t,)) for t in range(24)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:3]
    reqs, launches = b.stats()
    b.close()
    # data_only calls with only parity erased ((8,)) return before reaching the batcher
    assert 0 < reqs <= calls[0] == 24 * 8
    assert launches < reqs, (reqs, launches)   # concurrent calls really shared launches


def test_batched_errors_unchanged():
    k, m = 4, 2
    b = reedsolomon.Batcher(max_batch=8, window_us=100)
    enc = reedsolomon.New(k, m)
    enc.SetBatcher(b)
    rng = np.random.default_rng(1)
    st = _stripe(rng, k, m, 1000)
    with pytest.raises(reedsolomon.ErrTooFewShards):
        enc.ReconstructData([st[0], None, None, None, st[4], None])
    with pytest.raises(reedsolomon.ErrShardSize):
        enc.ReconstructData([st[0][:999], None, st[2], st[3], st[4], st[5]])
    full = list(st)
    enc.ReconstructData(full)  # nothing missing: no-op
    shards = [None, st[1], st[2], st[3], None, st[5]]
    enc.Reconstruct(shards)
    assert np.array_equal(shards[0], st[0]) and np.array_equal(shards[4], st[4])
    assert b.stats()[0] == 1
    enc.SetBatcher(None)
    b.close()


def test_batched_large_and_reconstruct_verify():
    """A 1 MiB + 13 stripe with four erasures, then reconstructAndVerify
    (internal/tractserver/store.go:1132-1142) through the batcher: decode and verify run as
    one group (one sync), a good stripe verifies, a corrupted survivor does not."""
    k, m = 10, 4
    rng = np.random.default_rng(3)
    st = _stripe(rng, k, m, (1 << 20) + 13)
    b = reedsolomon.Batcher(max_batch=4, window_us=0)
    enc = reedsolomon.New(k, m)
    enc.SetBatcher(b)
    shards = [None if i in (0, 3, 11, 13) else st[i] for i in range(k + m)]
    enc.Reconstruct(shards)
    for i in (0, 3, 11, 13):
        assert np.array_equal(shards[i], st[i]), i
    shards = [None if i in (5,) else st[i] for i in range(k + m)]
    assert enc.ReconstructAndVerify(shards)
    assert np.array_equal(shards[5], st[5])
    bad = [None if i in (5,) else st[i].copy() for i in range(k + m)]
    bad[12][777] ^= 0x40   # a surviving parity shard is wrong: the re-encode disagrees
    assert not enc.ReconstructAndVerify(bad)
    assert enc.Verify(list(st)) and not enc.Verify(bad[:5] + [st[5]] + bad[6:])
    assert b.stats() == (5, 5)
    enc.SetBatcher(None)
    b.close()


def test_batched_concurrent_reconstruct_verify():
    """The curator-driven recovery path under load: concurrent reconstructAndVerify calls
    (RSEncode RPCs with an indexMap, store.go:1102) from 16 threads share launches; every
    rebuilt shard equals the original and exactly the corrupted stripes fail to verify."""
    torch = _torch()
    k, m, S, T, R = 6, 3, 300_001, 16, 4
    rng = np.random.default_rng(11)
    stripes = [_stripe(rng, k, m, S) for _ in range(4)]
    b = reedsolomon.Batcher(max_batch=32, window_us=2000)
    enc = reedsolomon.New(k, m)
    enc.SetBatcher(b)
    # Every call's shards are built up front (pinning is slow), then the threads start together.
    work = {}
    for tid in range(T):
        for it in range(R):
            full = stripes[(tid + it) % len(stripes)]
            lost = [1 + it % 2, k + 1]   # a failed tractserver: the same slots for many chunks
            corrupt = (tid + it) % 3 == 0
            pinned = (tid + it) % 2 == 0
            mk = (lambda a: torch.from_numpy(a.copy()).pin_memory().numpy()) if pinned else (lambda a: a.copy())
            sh = [None if i in lost else mk(full[i]) for i in range(k + m)]
            if corrupt:
                victim = next(i for i in range(k + m) if i not in lost)
                sh[victim][S // 2] ^= 0x01
            work[tid, it] = (full, lost, corrupt, sh)
    errors = []
    start = threading.Barrier(T)

    def server(tid):
        start.wait()
        for it in range(R):
            full, lost, corrupt, sh = work[tid, it]
            try:
                ok = enc.ReconstructAndVerify(sh)
                assert ok == (not corrupt), (tid, it, ok)
                if not corrupt:
                    for i in lost:
                        assert np.array_equal(sh[i], full[i]), (tid, it, i)
            except Exception as e:  # noqa: BLE001 -- collected and re-raised on the main thread
                errors.append(e)

    ths = [threading.Thread(target=server, args=(t,)) for t in range(T)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:3]
    reqs, launches = b.stats()
    assert reqs == T * R and launches < reqs, (reqs, launches)
    enc.SetBatcher(None)
    b.close()


def test_batched_concurrent_encodes_match_oracle():
    """The tractserver side: concurrent RSEncode RPCs each Encode one increment per call
    (internal/tractserver/store.go:1099).  With a Batcher attached, Encode calls from many
    threads share launches; parity (written over stale pool bytes) equals the oracle's."""
    torch = _torch()
    k, m = 6, 3
    rng = np.random.default_rng(7)
    sizes = [4096, 65536, (1 << 20) + 13]
    data = {s: [rng.integers(0, 256, s, dtype=np.uint8) for _ in range(k)] for s in sizes}
    want = {s: N.encode(k, m, data[s]) for s in sizes}
    b = reedsolomon.Batcher(max_batch=32, window_us=2000)
    enc = reedsolomon.New(k, m)
    enc.SetBatcher(b)
    errors = []

    def server(tid):
        for it in range(6):
            size = sizes[(tid + it) % len(sizes)]
            pinned = (tid + it) % 2 == 0
            mk = (lambda a: torch.from_numpy(a).pin_memory().numpy()) if pinned else (lambda a: a.copy())
            shards = [mk(x) for x in data[size]] + [mk(np.full(size, 0xEE, np.uint8)) for _ in range(m)]
            try:
                enc.Encode(shards)
                for j in range(m):
                    assert np.array_equal(shards[k + j], want[size][j]), (tid, it, j)
                for i in range(k):
                    assert np.array_equal(shards[i], data[size][i]), (tid, it, i)
            except Exception as e:  # noqa: BLE001 -- collected and re-raised on the main thread
                errors.append(e)

    ths = [threading.Thread(target=server, args=(t,)) for t in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:3]
    reqs, launches = b.stats()
    assert reqs == 16 * 6
    assert launches < reqs, (reqs, launches)
    # Errors keep their types on the batched path; Verify goes through the batcher too.
    with pytest.raises(reedsolomon.ErrShardSize):
        enc.Encode([data[4096][0][:4095]] + [x.copy() for x in data[4096][1:]] + [np.zeros(4096, np.uint8)] * m)
    ok_shards = [x.copy() for x in data[4096]] + [x.copy() for x in want[4096]]
    assert enc.Verify(ok_shards)
    ok_shards[k][0] ^= 1
    assert not enc.Verify(ok_shards)
    assert b.stats()[0] == reqs + 2
    enc.SetBatcher(None)
    b.close()
