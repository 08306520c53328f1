"""GPU parity tests: the HIP engine (through the C ABI) vs the CPU oracle and the committed
golden vectors.  Bar: bit-exact (integer GF(2^8) byte work).

Mirrors the reference's RS tests (internal/tractserver/store_test.go:749-879 TestRSEncode /
TestRSReconstruct: RS(3,2), lengths 12000/20000, erasures {1,3}; test_rs_recovery.go
offsets 4000/123000 and TractLength-56789/98765) plus blb's classes and BASELINE sizes.
"""
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from blb_amd import reedsolomon as rs  # noqa: E402
from blb_amd.hostcopy import to_device, to_numpy

TRACT = 8 * 1024 * 1024  # core.TractLength (internal/core/constants.go:15)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def rand_shards(rng, n, S):
    return [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(n)]


def oracle_encode(O, k, m, data):
    S = data[0].size
    sh = [d.copy() for d in data] + [np.zeros(S, np.uint8) for _ in range(m)]
    O.encode(k, m, sh, use_avx2=True, threads=8)
    return sh[k:]


# ---------------------------------------------------------------- golden vectors

def golden_cases(golden):
    for (k, m), g in sorted(golden.items()):
        i = 0
        while f"S{i}" in g:
            yield k, m, g, i
            i += 1


def test_golden_encode_host(golden):
    for k, m, g, i in golden_cases(golden):
        data, parity = g[f"data{i}"], g[f"parity{i}"]
        enc = rs.New(k, m)
        sh = [data[j].copy() for j in range(k)] + [np.full(data.shape[1], 0xEE, np.uint8) for _ in range(m)]
        enc.Encode(sh)  # outputs are overwritten, not accumulated into
        for j in range(m):
            assert np.array_equal(sh[k + j], parity[j]), (k, m, i, j)
        assert enc.Verify(sh)


def test_golden_encode_device_batch(golden, dev):
    for k, m, g, i in golden_cases(golden):
        data, parity = g[f"data{i}"], g[f"parity{i}"]
        S = data.shape[1]
        B = 3
        host = np.empty((B, k + m, S), np.uint8)
        host[:, :k] = data
        host[:, k:] = 0x5A
        st = to_device(host, dev)
        enc = rs.New(k, m)
        enc.EncodeBatch(st)
        got = to_numpy(st)
        for b in range(B):
            assert np.array_equal(got[b, k:], parity), (k, m, i, b)
        assert bool(enc.VerifyBatch(st).all())


def test_golden_reconstruct_host_and_device(golden, dev):
    for (k, m), g in sorted(golden.items()):
        enc = rs.New(k, m)
        full = [g["data0"][j] for j in range(k)] + [g["parity0"][j] for j in range(m)]
        S = full[0].size
        p = 0
        while f"pattern{p}" in g:
            pat = [int(x) for x in g[f"pattern{p}"]]
            for data_only in (False, True):
                sh = [None if i in pat else full[i].copy() for i in range(k + m)]
                (enc.ReconstructData if data_only else enc.Reconstruct)(sh)
                for i in range(k + m):
                    if i < k or not data_only:
                        assert np.array_equal(sh[i], full[i]), (k, m, pat, i, data_only)
                    else:
                        assert (sh[i] is None) == (i in pat)
                # batched device path, erased shards poisoned first
                B = 2
                st = to_device(np.stack([np.stack(full)] * B), dev)
                want = st.clone()
                for i in pat:
                    st[:, i] = 0xC3
                present = [i not in pat for i in range(k + m)]
                enc.ReconstructBatch(st, present, data_only=data_only)
                for i in range(k + m):
                    if i in pat and data_only and i >= k:
                        assert bool((st[:, i] == 0xC3).all())
                    else:
                        assert torch.equal(st[:, i], want[:, i]), (k, m, pat, i, data_only)
            p += 1
        assert S > 0


# ---------------------------------------------------------------- reference test shapes

def test_store_test_rsencode_increments(oracle_lib):
    """TestRSEncode: RS(3,2), B=12000 coded in EncodeIncrementSize=5000 windows
    (store_test.go:749-815); parity of the windows concatenated must verify."""
    k, m, B, inc = 3, 2, 12000, 5000
    rng = np.random.default_rng(97531)
    data = rand_shards(rng, k, B)
    enc = rs.New(k, m)
    parity = [np.empty(0, np.uint8) for _ in range(m)]
    for off in range(0, B, inc):
        ln = min(inc, B - off)
        sh = [d[off:off + ln].copy() for d in data] + [np.empty(ln, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        parity = [np.concatenate([parity[j], sh[k + j]]) for j in range(m)]
    assert enc.Verify(data + parity)
    want = oracle_encode(oracle_lib, k, m, data)
    assert all(np.array_equal(a, b) for a, b in zip(parity, want))


def test_store_test_rsreconstruct():
    """TestRSReconstruct: RS(3,2), B=20000, missing {1 (data), 3 (parity)},
    Reconstruct then Verify (store_test.go:817-879, reconstructAndVerify store.go:1132)."""
    k, m, B = 3, 2, 20000
    rng = np.random.default_rng(97532)
    enc = rs.New(k, m)
    sh = rand_shards(rng, k, B) + [np.empty(B, np.uint8) for _ in range(m)]
    enc.Encode(sh)
    full = [s.copy() for s in sh]
    sh[1] = None
    sh[3] = None
    enc.Reconstruct(sh)
    assert enc.Verify(sh)
    assert all(np.array_equal(a, b) for a, b in zip(sh, full))


@pytest.mark.parametrize("off,length", [(4000, 123000), (TRACT - 56789, 98765)])
def test_client_reconstruct_data_into_caller_buffer(off, length):
    """client/blb/reconstruct.go:166-184 with test_rs_recovery.go's read windows: the
    reconstructed piece must land in the caller's buffer (thisB[0:0:length])."""
    k, m = 6, 3
    rng = np.random.default_rng(off)
    enc = rs.New(k, m)
    sh = rand_shards(rng, k, length) + [np.empty(length, np.uint8) for _ in range(m)]
    enc.Encode(sh)
    truth = sh[2].copy()
    thisB = np.full(length + 17, 0x77, np.uint8)  # caller buffer larger than the piece
    sh[2] = None
    sh[7] = None
    enc.ReconstructData(sh, outs={2: thisB})
    assert np.shares_memory(sh[2], thisB) and sh[2].ctypes.data == thisB.ctypes.data
    assert np.array_equal(thisB[:length], truth)
    assert np.all(thisB[length:] == 0x77)  # bytes past the piece untouched
    assert sh[7] is None  # ReconstructData leaves parity missing


# ---------------------------------------------------------------- random shapes vs oracle

SHAPES = [(1, 1), (2, 1), (3, 2), (4, 2), (5, 3), (6, 3), (7, 2), (8, 3), (10, 3), (10, 4),
          (12, 5), (13, 4), (17, 3), (20, 9), (24, 12), (32, 8), (50, 20)]


@pytest.mark.parametrize("k,m", SHAPES)
def test_random_encode_vs_oracle(oracle_lib, k, m, dev):
    rng = np.random.default_rng(k * 131 + m)
    for S in (1, 3, 16, 255, 8191, 8192, 8193, 70001):
        data = rand_shards(rng, k, S)
        want = oracle_encode(oracle_lib, k, m, data)
        enc = rs.New(k, m)
        sh = [d.copy() for d in data] + [np.full(S, 0x11, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        for j in range(m):
            assert np.array_equal(sh[k + j], want[j]), (k, m, S, j)
        # device shards (pointer-table path), one of them deliberately misaligned
        base = to_device(np.stack(data + [np.zeros(S, np.uint8)] * m), dev)
        odd = torch.empty(S + 1, dtype=torch.uint8, device=dev)[1:]
        odd.copy_(base[0])
        dsh = [odd] + [base[i] for i in range(1, k + m)]
        enc.Encode(dsh)
        got = to_numpy(base[k:])
        for j in range(m):
            assert np.array_equal(got[j], want[j]), (k, m, S, j, "dev")


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4), (12, 5), (17, 3), (20, 9), (24, 12)])
def test_random_erasures_vs_oracle(oracle_lib, k, m):
    rng = np.random.default_rng(k * 7 + m)
    enc = rs.New(k, m)
    for trial in range(12):
        S = int(rng.integers(1, 40000))
        sh = rand_shards(rng, k, S) + [np.empty(S, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        full = [s.copy() for s in sh]
        ne = int(rng.integers(1, m + 1))
        pat = sorted(rng.choice(k + m, ne, replace=False).tolist())
        data_only = bool(trial & 1)
        cur = [None if i in pat else full[i].copy() for i in range(k + m)]
        (enc.ReconstructData if data_only else enc.Reconstruct)(cur)
        ref = oracle_lib.reconstruct(k, m, [None if i in pat else full[i] for i in range(k + m)], data_only)
        for i in range(k + m):
            if ref[i] is None:
                assert cur[i] is None
            else:
                assert np.array_equal(cur[i], ref[i]) and np.array_equal(cur[i], full[i]), (k, m, pat, i)


def test_too_many_erasures_and_all_present():
    enc = rs.New(6, 3)
    S = 1000
    rng = np.random.default_rng(9)
    sh = rand_shards(rng, 6, S) + [np.empty(S, np.uint8) for _ in range(3)]
    enc.Encode(sh)
    with pytest.raises(rs.ErrTooFewShards):
        enc.Reconstruct([None, None, None, None] + sh[4:])
    before = [s.copy() for s in sh]
    enc.Reconstruct(sh)  # all present: no work
    assert all(np.array_equal(a, b) for a, b in zip(sh, before))


@pytest.mark.parametrize("k,m", [(6, 3), (10, 4), (12, 5)])  # (10,4), (12,5): verify at U = 1
def test_verify_detects_corruption(dev, k, m):
    S, B = 65536 + 7, 5
    enc = rs.New(k, m)
    st = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device=dev)
    enc.EncodeBatch(st)
    assert bool(enc.VerifyBatch(st).all())
    st[2, k + 1, S - 1] ^= 1   # last byte (tail path) of a parity shard
    st[4, 0, 12345] ^= 0x80    # a data byte
    ok = to_numpy(enc.VerifyBatch(st)).tolist()
    assert ok == [True, True, False, True, False]
    host = [to_numpy(st[2, i]) for i in range(k + m)]
    assert not enc.Verify(host)
    host0 = [to_numpy(st[0, i]) for i in range(k + m)]
    assert enc.Verify(host0)
    assert not enc.Verify([st[2, i] for i in range(k + m)])  # device shards


def test_strided_batch_layouts(oracle_lib, dev):
    """Shards of a stripe need not be adjacent: a [B, S, k+m]-ordered buffer viewed as
    [B, k+m, S] is rejected (bytes not contiguous); padded strides work."""
    k, m, S, B = 6, 3, 5000, 4
    enc = rs.New(k, m)
    big = torch.randint(0, 256, (B, k + m, S + 48), dtype=torch.uint8, device=dev)
    view = big[:, :, 16:16 + S]
    enc.EncodeBatch(view)
    h = to_numpy(view)
    for b in range(B):
        want = oracle_encode(oracle_lib, k, m, [h[b, i].copy() for i in range(k)])
        for j in range(m):
            assert np.array_equal(h[b, k + j], want[j])
    with pytest.raises(rs.ErrInvalidArgument):
        enc.EncodeBatch(torch.zeros(B, S, k + m, dtype=torch.uint8, device=dev).transpose(1, 2))


def test_concurrent_host_calls(oracle_lib):
    """Many threads through the C ABI at once (cgo calls from goroutines)."""
    k, m = 6, 3
    enc = rs.New(k, m)
    errors = []

    def worker(seed):
        try:
            rng = np.random.default_rng(seed)
            for _ in range(4):
                S = int(rng.integers(1000, 300000))
                data = rand_shards(rng, k, S)
                sh = data + [np.empty(S, np.uint8) for _ in range(m)]
                enc.Encode(sh)
                want = oracle_encode(oracle_lib, k, m, data)
                assert all(np.array_equal(sh[k + j], want[j]) for j in range(m))
                sh[0] = None
                enc.ReconstructData(sh)
                assert np.array_equal(sh[0], data[0])
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(s,)) for s in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("nstreams,S", [(0, 1 << 20), (1, 1 << 20), (3, 1 << 20), (3, (1 << 20) + 13), (8, 4096)])
def test_streaming_host_batch(oracle_lib, nstreams, S):
    """Pinned stripes: in place over PCIe (nstreams = 0) or through the copy engines on a device
    ring (nstreams >= 1, BASELINE config 5's hipMemcpyAsync form); parity is the oracle's, shard
    lengths off the ring's 256-byte pitch included."""
    k, m, B = 6, 3, 7
    enc = rs.New(k, m)
    pinned = torch.empty((B, k + m, S), dtype=torch.uint8).pin_memory()
    host = pinned.numpy()
    rng = np.random.default_rng(3 + nstreams)
    host[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:] = 0xA5
    enc.EncodeHostBatch([[host[b, i] for i in range(k + m)] for b in range(B)], nstreams=nstreams)
    for b in range(B):
        want = oracle_encode(oracle_lib, k, m, [host[b, i].copy() for i in range(k)])
        for j in range(m):
            assert np.array_equal(host[b, k + j], want[j]), (b, j)


def test_large_shard_host_path_chunks(oracle_lib):
    """Host path pipelines 1 MiB column chunks over two streams; a full 8 MiB tract with an
    odd tail must still be bit-exact."""
    k, m = 10, 4
    S = TRACT + 123
    rng = np.random.default_rng(11)
    data = rand_shards(rng, k, S)
    enc = rs.New(k, m)
    sh = data + [np.empty(S, np.uint8) for _ in range(m)]
    enc.Encode(sh)
    want = oracle_encode(oracle_lib, k, m, data)
    for j in range(m):
        assert np.array_equal(sh[k + j], want[j])
    full = [s.copy() for s in sh]
    sh[1] = None
    sh[7] = None
    enc.Reconstruct(sh)
    assert all(np.array_equal(a, b) for a, b in zip(sh, full))


# ---------------------------------------------------------------- BASELINE sizes

def _sample_check(O, enc, st, k, m, stripes):
    """Oracle check of whole 8 MiB stripes sampled from a device batch."""
    for b in stripes:
        h = to_numpy(st[b])
        want = oracle_encode(O, k, m, [h[i].copy() for i in range(k)])
        for j in range(m):
            assert np.array_equal(h[k + j], want[j]), (b, j)


def test_baseline_rs63_b1024_roundtrip(oracle_lib, dev):
    """BASELINE configs 2+3 at full size: RS(6,3), B=1024 stripes of 8 MiB tracts.
    Encode, oracle-check sampled stripes, Verify all, erase data shard 1 everywhere,
    ReconstructData, compare with the saved shard (size-independent round trip)."""
    k, m, B, S = 6, 3, 1024, TRACT
    enc = rs.New(k, m)
    st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(97531)
    st[:, :k].random_(0, 256, generator=g)
    enc.EncodeBatch(st)
    _sample_check(oracle_lib, enc, st, k, m, [0, 511, 1023])
    assert bool(enc.VerifyBatch(st).all())
    saved = st[:, 1].clone()
    st[:, 1].zero_()
    enc.ReconstructBatch(st, [i != 1 for i in range(k + m)], data_only=True)
    assert torch.equal(st[:, 1], saved)
    del st, saved
    torch.cuda.empty_cache()


def test_baseline_rs104_b512_two_erasures(oracle_lib, dev):
    """BASELINE config 4, one GPU's share: RS(10,4), 512 stripes (4096 / 8 GPUs), encode +
    2-erasure reconstruct ({data 1, data 7} and mixed {data 2, parity 11})."""
    k, m, B, S = 10, 4, 512, TRACT
    enc = rs.New(k, m)
    st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    st[:, :k].random_(0, 256)
    enc.EncodeBatch(st)
    _sample_check(oracle_lib, enc, st, k, m, [0, 257, 511])
    for pat in ([1, 7], [2, 11]):
        saved = st[:, pat].clone()
        st[:, pat] = 0
        enc.ReconstructBatch(st, [i not in pat for i in range(k + m)], data_only=False)
        assert torch.equal(st[:, pat], saved), pat
    assert bool(enc.VerifyBatch(st).all())
    del st
    torch.cuda.empty_cache()


def test_cold_class_rs83_b512_full_size(oracle_lib, dev):
    """blb's COLD transition class RS(8,3) (targetClass, internal/curator/
    storage_class_loop.go:41-44) at the bench's size: 512 stripes of 8 MiB.  Encode
    (oracle-checked stripes), Verify, 1- and 2-erasure rebuilds (data and mixed), and the
    fused encode + ChecksumFile CRCs of rsEncodeOne's parity window at file offset 4 MiB
    (phase 256, seeded), checked against the oracle's crc32.Update per file-aligned block."""
    k, m, B, S = 8, 3, 512, TRACT
    enc = rs.New(k, m)
    st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(8303)
    st[:, :k].random_(0, 256, generator=g)
    enc.EncodeBatch(st)
    _sample_check(oracle_lib, enc, st, k, m, [0, 255, 511])
    assert bool(enc.VerifyBatch(st).all())
    for pat, data_only in (([1], True), ([1, 5], False), ([3, 9], False)):
        saved = st[:, pat].clone()
        st[:, pat] = 0xA5
        enc.ReconstructBatch(st, [i not in pat for i in range(k + m)], data_only=data_only)
        assert torch.equal(st[:, pat], saved), pat
    seeds = torch.randint(-2**31, 2**31 - 1, (m, B), dtype=torch.int32, device=dev)
    st[:, k:] = 0x5A
    crc = enc.EncodeBatchCRC(st, 65532, phase=256, seeds=seeds)
    assert bool(enc.VerifyBatch(st).all())
    crc = to_numpy(crc).view(np.uint32)
    sd = to_numpy(seeds).view(np.uint32)
    first = 65532 - 256
    for b in (0, 511):
        par = to_numpy(st[b, k:])
        for j in range(m):
            want0 = oracle_lib.crc32c(par[j][:first], int(sd[j, b]))
            rest = np.asarray(oracle_lib.crc32c_blocks(par[j][first:], 65532), dtype=np.uint32)
            assert crc[j, b, 0] == want0, (b, j)
            assert np.array_equal(crc[j, b, 1:], rest), (b, j)
    del st, seeds
    torch.cuda.empty_cache()


def _pinned(a):
    return torch.from_numpy(a).pin_memory().numpy()


def test_zero_copy_pinned_host_calls(oracle_lib):
    """Pinned host shards take the zero-copy path (the kernel reads/writes host memory in
    place over PCIe); results must match the staged (pageable) path and the oracle."""
    for k, m, S in [(6, 3, 1 << 20), (10, 4, 12345), (3, 2, 1)]:
        rng = np.random.default_rng(S)
        data = rand_shards(rng, k, S)
        want = oracle_encode(oracle_lib, k, m, data)
        enc = rs.New(k, m)
        sh = [_pinned(d.copy()) for d in data] + [_pinned(np.full(S, 0x3C, np.uint8)) for _ in range(m)]
        enc.Encode(sh)
        for j in range(m):
            assert np.array_equal(sh[k + j], want[j]), (k, m, S, j)
        assert enc.Verify(sh)
        sh[k][S // 2] ^= 0x40
        assert not enc.Verify(sh)
        sh[k][S // 2] ^= 0x40
        full = [s.copy() for s in sh]
        lost = [0, k] if m > 1 else [0]
        cur = [None if i in lost else sh[i] for i in range(k + m)]
        out0 = _pinned(np.zeros(S + 64, np.uint8))
        enc.Reconstruct(cur, outs={0: out0})   # pinned output buffer -> zero-copy
        for i in range(k + m):
            assert np.array_equal(cur[i], full[i]), (k, m, S, i)
        assert cur[0].ctypes.data == out0.ctypes.data


def test_streaming_host_batch_pageable_fallback(oracle_lib):
    """Pageable stripes are never handed to HIP's copy engines: with nstreams >= 1 the batch
    still takes the CPU-staged path (pinned, device-mapped chunks), bit-exact."""
    k, m, S, B = 6, 3, 300001, 5
    enc = rs.New(k, m)
    rng = np.random.default_rng(4)
    stripes = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
               for _ in range(B)]
    enc.EncodeHostBatch(stripes, nstreams=2)
    for st in stripes:
        want = oracle_encode(oracle_lib, k, m, st[:k])
        for j in range(m):
            assert np.array_equal(st[k + j], want[j])


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (8, 3), (10, 4), (12, 5), (5, 9)])
def test_reconstruct_and_verify_one_pass_vs_oracle(oracle_lib, dev, k, m):
    """reconstructAndVerify in one pass (missing shards written, the present shards the decode
    does not read compared): the rebuilt bytes and the verdict equal the oracle's Reconstruct
    then Verify for every erasure count, with a corrupted shard inside the decode's inputs
    (the oracle's Verify then fails unless no shard is left over), a corrupted leftover
    shard, and none; host path and device batch.  (5, 9): 14 rows, two kernel passes."""
    n = k + m
    rng = np.random.default_rng(k * 100 + m)
    S = 70001
    enc = rs.New(k, m)
    full = rand_shards(rng, k, S) + [np.empty(S, np.uint8) for _ in range(m)]
    oracle_lib.encode(k, m, full)
    cases = 0
    for e in range(1, m + 1):
        lost = sorted(rng.choice(n, e, replace=False).tolist())
        present = [i not in lost for i in range(n)]
        inputs = [i for i in range(n) if present[i]][:k]
        leftovers = [i for i in range(n) if present[i] and i not in inputs]
        for corrupt in (None, inputs[-1], leftovers[0] if leftovers else None):
            base = [x.copy() for x in full]
            if corrupt is not None:
                base[corrupt][S // 3] ^= 0x21
            want = oracle_lib.reconstruct(k, m, [None if i in lost else base[i].copy() for i in range(n)], False)
            want_ok = oracle_lib.verify(k, m, want)
            cur = [None if i in lost else base[i].copy() for i in range(n)]
            ok = enc.ReconstructAndVerify(cur)
            assert ok == want_ok, (k, m, lost, corrupt)
            for i in lost:
                assert np.array_equal(cur[i], want[i]), (k, m, lost, corrupt, i)
            st = to_device((np.stack(base + base)).reshape(2, n, S), dev)
            for i in lost:
                st[:, i] = 0xA5
            oks = to_numpy(enc.ReconstructAndVerifyBatch(st, present))
            assert list(oks) == [want_ok, want_ok], (k, m, lost, corrupt)
            got = to_numpy(st)
            for i in lost:
                assert np.array_equal(got[0, i], want[i]) and np.array_equal(got[1, i], want[i])
            cases += 1
    assert cases >= 2 * m


def test_reconstruct_and_verify_fused(oracle_lib):
    """reconstructAndVerify (store.go:1132-1142) in one round trip: true for a consistent
    stripe (incl. when nothing is missing), false when a surviving shard disagrees."""
    for k, m, S in [(3, 2, 20000), (6, 3, (1 << 20) + 5), (10, 4, 4096)]:
        rng = np.random.default_rng(S)
        enc = rs.New(k, m)
        full = rand_shards(rng, k, S) + [np.empty(S, np.uint8) for _ in range(m)]
        enc.Encode(full)
        cur = [None if i in (1, k) else full[i].copy() for i in range(k + m)]
        assert enc.ReconstructAndVerify(cur)
        assert all(np.array_equal(a, b) for a, b in zip(cur, full))
        assert enc.ReconstructAndVerify([s.copy() for s in full])
        bad = [None if i == 1 else full[i].copy() for i in range(k + m)]
        bad[k + m - 1][S // 2] ^= 0x5A   # an extra present parity that disagrees
        assert not enc.ReconstructAndVerify(bad)
        pinned = [None if i == 0 else torch.from_numpy(full[i].copy()).pin_memory().numpy() for i in range(k + m)]
        assert enc.ReconstructAndVerify(pinned)   # zero-copy variant
        assert np.array_equal(pinned[0], full[0])


# ---------------------------------------------------------------- SURVEY §8(d) edge fixtures

@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4), (12, 5)])
@pytest.mark.parametrize("fill", [0x00, 0xFF])
def test_constant_data_edge_fixtures(oracle_lib, dev, k, m, fill):
    """All-0x00 / all-0xFF data at the §8(d) edge lengths: host Encode and device EncodeBatch
    equal the oracle (all-zero data -> all-zero parity; all-0xFF -> one constant per row),
    and a 2-erasure Reconstruct restores the data."""
    enc = rs.New(k, m)
    for S in (1, 15, 12000, 20000, 98765, 123000):
        data = [np.full(S, fill, np.uint8) for _ in range(k)]
        want = oracle_encode(oracle_lib, k, m, data)
        if fill == 0:
            assert all(not w.any() for w in want)
        else:
            assert all(np.all(w == w[0]) for w in want)
        sh = [d.copy() for d in data] + [np.full(S, 0x5A, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        for j in range(m):
            assert np.array_equal(sh[k + j], want[j]), (k, m, fill, S, j)
        st = to_device(np.stack(data + [np.full(S, 0xA5, np.uint8)] * m)[None], dev)
        enc.EncodeBatch(st)
        got = to_numpy(st[0, k:])
        for j in range(m):
            assert np.array_equal(got[j], want[j]), (k, m, fill, S, j, "dev")
        cur = [None if i in (0, k - 1) else sh[i].copy() for i in range(k + m)]
        enc.Reconstruct(cur)
        assert all(np.array_equal(cur[i], sh[i]) for i in range(k + m)), (k, m, fill, S)



@pytest.mark.parametrize("k,m", [(250, 6), (200, 56), (1, 255), (128, 128)])
def test_maximum_shard_counts_vs_oracle(oracle_lib, dev, k, m):
    """k + m = 256 (klauspost's limit, ErrMaxShardNum above it): encode of host shards and of a
    device batch against the oracle, then Reconstruct / ReconstructData with all m slots lost
    (m above the kernel's 8 rows per pass: the plan splits the rows into passes)."""
    rng = np.random.default_rng(k * 3 + m)
    enc = rs.New(k, m)
    for S in (1, 4099):
        data = rand_shards(rng, k, S)
        want = oracle_encode(oracle_lib, k, m, data)
        sh = [d.copy() for d in data] + [np.full(S, 0x11, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        assert all(np.array_equal(sh[k + j], want[j]) for j in range(m)), (k, m, S)
        st = to_device(np.stack(data + want)[None], dev)
        st[:, k:].fill_(0x5A)
        enc.EncodeBatch(st)
        assert np.array_equal(to_numpy(st[0]), np.stack(data + want)), (k, m, S, "batch")
        full = data + want
        lost = sorted(rng.choice(k + m, m, replace=False).tolist())
        for data_only in (False, True):
            cur = [None if i in lost else full[i].copy() for i in range(k + m)]
            (enc.ReconstructData if data_only else enc.Reconstruct)(cur)
            ref = oracle_lib.reconstruct(k, m, [None if i in lost else full[i] for i in range(k + m)], data_only)
            for i in range(k + m):
                if ref[i] is None:
                    assert cur[i] is None, (k, m, i)
                else:
                    assert np.array_equal(cur[i], ref[i]) and np.array_equal(cur[i], full[i]), (k, m, lost, i)


@pytest.mark.parametrize("k,m,S,kind", [
    (6, 3, 4096, "page"),              # one unit through the pinned bounce, inline table
    (6, 3, 3 * 1024 * 1024 + 48, "page"),  # 4 units per stripe through the two pinned slots
    (30, 5, 100_000, "page"),          # n = 35 > kInlinePtrs: the table rides in the slot
    (30, 5, 100_000, "pin"),           # zero copy with n > kInlinePtrs: the worker's device table
])
def test_host_staging_paths_verify_and_reconstruct(oracle_lib, k, m, S, kind):
    """Every host staging path since round 5 (pageable memory never reaches HIP's copy engines,
    DESIGN §4h): Encode, Verify and ReconstructAndVerify through the pinned bounce, the chunked
    two-slot pinning and zero copy, with tables inline, in the slot and on the device.  A parity
    byte corrupted in the LAST chunk must turn Verify / ReconstructAndVerify false; the rebuilt
    shards are the oracle's."""
    rng = np.random.default_rng(S + k)
    data = rand_shards(rng, k, S)
    want = oracle_encode(oracle_lib, k, m, data)
    enc = rs.New(k, m)

    def buf(src):
        if kind == "pin":
            b = rs.GetBuffer(S)[:S]
            b[:] = src
            return b
        return src.copy()

    held = []
    sh = [buf(d) for d in data] + [buf(np.full(S, 0x77, np.uint8)) for _ in range(m)]
    held += sh
    enc.Encode(sh)
    assert all(np.array_equal(sh[k + j], want[j]) for j in range(m)), "encode"
    assert enc.Verify(sh)
    sh[k + m - 1][S - 3] ^= 0x40                     # inside the last chunk
    assert not enc.Verify(sh)
    sh[k + m - 1][S - 3] ^= 0x40
    lost = [1, k + 1]
    cur = [None if i in lost else sh[i] for i in range(k + m)]
    assert enc.ReconstructAndVerify(cur) is True
    for i in lost:
        assert np.array_equal(cur[i], (data + want)[i]), ("rebuilt", i)
    cur = [None if i in lost else sh[i].copy() for i in range(k + m)]
    cur[k + m - 1][S - 1] ^= 0x01                    # a present parity piece the decode does not read
    assert enc.ReconstructAndVerify(cur) is False
    if kind == "pin":
        for b in held:
            rs.PutBuffer(b)
