"""The host runtime under the C ABI (blb_amd/csrc/runtime.hip):

  * device lists: encoders bound to a device list spread host calls over it and split host
    batches across it; device-resident calls run on the stripes' device -- on the 1-GPU box
    the list [0, 0] exercises the split (two lanes on GPU 0);
  * the bounded stream-worker pool: 4x more concurrent callers than workers, bit-exact
    against the oracle, device memory bounded (hipMemGetInfo before / after);
  * the pinned buffer pool (rpc.GetBuffer / PutBuffer, pkg/rpc/pool.go:16-62): capacity
    classes, reuse, zero-copy coding on pool buffers.

Every coding result is checked against the oracle restatement (oracle/)."""
import ctypes
import threading

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401
from blb_amd import _lib
from blb_amd import reedsolomon as rs
from blb_amd.hostcopy import to_numpy
from oracle import rs_numpy as N

MIB = 1 << 20
EXTRA = 64 << 10  # disk.ExtraRoom (pkg/disk/checksum_file.go:27)


# ---------------------------------------------------------------- CPU: argument checks

def test_new_on_argument_checks():
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.blbrs_new_on(6, 3, None, 0, ctypes.byref(h)) == rs.ErrInvalidArgument.code
    neg = (ctypes.c_int * 2)(0, -1)
    assert lib.blbrs_new_on(6, 3, neg, 2, ctypes.byref(h)) == rs.ErrInvalidArgument.code
    ok = (ctypes.c_int * 2)(0, 0)
    assert lib.blbrs_new_on(0, 3, ok, 2, ctypes.byref(h)) == rs.ErrInvShardNum.code
    assert lib.blbrs_new_on(6, 3, ok, 2, ctypes.byref(h)) == 0  # ids are checked lazily
    lib.blbrs_free(h)
    assert lib.blbrs_set_worker_limit(0) == rs.ErrInvalidArgument.code
    assert lib.blbrs_set_default_devices(None, -1) == rs.ErrInvalidArgument.code
    assert lib.blbrs_buffer_put(ctypes.c_void_p(0x1000)) == rs.ErrInvalidArgument.code
    assert lib.blbrs_buffer_get(1, None, None) == rs.ErrInvalidArgument.code


def test_host_batch_rejects_negative_nstreams():
    """blbrs_encode_host_batch: nstreams < 0 is INVALID_ARG, checked before anything else."""
    enc = rs.New(6, 3)
    with pytest.raises(rs.ErrInvalidArgument):
        enc.EncodeHostBatch([[np.zeros(64, np.uint8) for _ in range(9)]], nstreams=-1)


def test_device_calls_fail_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    enc = rs.New(6, 3, devices=[0])
    with pytest.raises((rs.ErrNoDevice, rs.ErrHIP, rs.ErrInvalidArgument)):
        enc.Devices()
    with pytest.raises((rs.ErrNoDevice, rs.ErrHIP)):
        rs.GetBuffer(4096)


# ---------------------------------------------------------------- GPU

def _oracle_parity(O, k, m, data):
    sh = [d.copy() for d in data] + [np.zeros(data[0].size, np.uint8) for _ in range(m)]
    O.encode(k, m, sh)
    return sh[k:]


@pytest.mark.gpu
def test_device_list_lanes_concurrent_host_calls(oracle_lib):
    """[0, 0]: two lanes on GPU 0.  Concurrent Encode / ReconstructData / Verify calls from
    8 threads spread over the list; every result bit-exact against the oracle."""
    k, m = 6, 3
    enc = rs.New(k, m, devices=[0, 0])
    assert enc.Devices() == [0, 0]
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(97531 * (t + 1))
            for it in range(6):
                S = [4096, 65536, 123000, 1 << 20, 98765, 4 * MIB][(t + it) % 6]
                data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
                sh = data + [np.full(S, 0xEE, np.uint8) for _ in range(m)]
                enc.Encode(sh)
                ref = _oracle_parity(oracle_lib, k, m, data)
                for j in range(m):
                    assert np.array_equal(sh[k + j], ref[j]), f"thread {t} parity {j}"
                assert enc.Verify(sh)
                lost = (t + it) % k
                orig = sh[lost].copy()
                sh[lost] = None
                enc.ReconstructData(sh)
                assert np.array_equal(sh[lost], orig)
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]
    st = rs.device_stats(0)
    assert st["calls"] >= 8 * 6 * 3
    assert st["inflight"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("pinned,nstreams", [(False, 0), (True, 0), (True, 3), (False, 3)])
def test_device_list_host_batch_split(oracle_lib, pinned, nstreams):
    """EncodeHostBatch splits its stripes contiguously over [0, 0] (two host threads, two
    workers); pageable stripes go through the staging ring, pinned ones zero-copy -- or, with
    nstreams >= 1, through the copy engines, both parts' rings on the one device at once."""
    import torch
    k, m, B, S = 10, 4, 7, 3 * MIB + 4100
    enc = rs.New(k, m, devices=[0, 0])
    rng = np.random.default_rng(11)
    if pinned:
        host = torch.empty((B, k + m, S), dtype=torch.uint8).pin_memory().numpy()
    else:
        host = np.empty((B, k + m, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:] = 0xC3
    stripes = [[host[b, i] for i in range(k + m)] for b in range(B)]
    enc.EncodeHostBatch(stripes, nstreams=nstreams)
    for b in range(B):
        ref = _oracle_parity(oracle_lib, k, m, [host[b, i] for i in range(k)])
        for j in range(m):
            assert np.array_equal(host[b, k + j], ref[j]), f"stripe {b} parity {j}"


@pytest.mark.gpu
def test_device_parts_split_batch(oracle_lib):
    """EncodeParts / ReconstructParts / VerifyParts over two shares of one batch on GPU 0
    (the multi-device form: one part per device)."""
    import torch
    k, m, B, S = 6, 3, 10, 70001
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    st[:, :k].random_(0, 256, generator=g)
    st[:, k:].fill_(0x5A)
    parts = [st[:4], st[4:]]
    enc = rs.New(k, m)
    enc.EncodeParts(parts)
    torch.cuda.synchronize()
    host = to_numpy(st)
    for b in range(B):
        ref = _oracle_parity(oracle_lib, k, m, [host[b, i] for i in range(k)])
        for j in range(m):
            assert np.array_equal(host[b, k + j], ref[j])
    oks = enc.VerifyParts(parts)
    assert all(bool(o.all()) for o in oks)
    lost = st.clone()
    lost[:, 2].fill_(0)
    lost[:, 7].fill_(0)
    present = [i not in (2, 7) for i in range(k + m)]
    enc.ReconstructParts([lost[:4], lost[4:]], present)
    torch.cuda.synchronize()
    assert torch.equal(lost, st)


@pytest.mark.gpu
def test_bounded_workers_4x_threads(oracle_lib):
    """32 threads against a limit of 8 workers: callers wait for a worker instead of
    creating more; results bit-exact; device memory growth bounded by the limit."""
    import torch
    k, m, S = 6, 3, 4 * MIB  # EncodeIncrementSize (internal/tractserver/config.go:117)
    limit, nthreads = 8, 32
    rs.trim()
    rs.set_worker_limit(limit)
    try:
        enc = rs.New(k, m, devices=[0])
        enc.Encode([np.ones(S, np.uint8)] * k + [np.empty(S, np.uint8) for _ in range(m)])  # plans uploaded
        torch.cuda.synchronize()
        free0, _ = torch.cuda.mem_get_info(0)
        errors = []
        barrier = threading.Barrier(nthreads)

        def worker(t):
            try:
                rng = np.random.default_rng(1000 + t)
                data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
                ref = _oracle_parity(oracle_lib, k, m, data)
                barrier.wait()
                for _ in range(3):
                    sh = data + [np.full(S, 0xA5, np.uint8) for _ in range(m)]  # pageable: staged
                    enc.Encode(sh)
                    for j in range(m):
                        assert np.array_equal(sh[k + j], ref[j]), f"thread {t} parity {j}"
            except Exception as e:
                errors.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[0]
        st = rs.device_stats(0)
        assert st["workers"] <= limit
        assert st["waits"] > 0
        free1, _ = torch.cuda.mem_get_info(0)
        # per worker: 2 ring slots of (k+m) x 1 MiB staging + streams, flag, table
        bound = limit * (2 * (k + m) * MIB + 4 * MIB) + 64 * MIB
        assert free0 - free1 <= bound, (free0 - free1, bound)
        assert st["staging_bytes"] <= limit * 2 * (k + m) * MIB
    finally:
        rs.set_worker_limit(8)
        rs.trim()
    assert rs.device_stats(0)["workers"] == 0


@pytest.mark.gpu
def test_pinned_pool_classes_and_reuse():
    """blbrs_buffer_get keeps blb's capacity classes (1/4/8 MiB + ExtraRoom, plus a small
    class), hands back the same buffers after PutBuffer, and frees odd sizes on put."""
    lib = _lib.load()

    def get(n):
        p = ctypes.c_void_p()
        cap = ctypes.c_size_t()
        assert lib.blbrs_buffer_get(n, ctypes.byref(p), ctypes.byref(cap)) == 0
        return p.value, cap.value

    cases = [(100, (128 << 10) + EXTRA), ((128 << 10) + EXTRA, (128 << 10) + EXTRA),
             ((128 << 10) + EXTRA + 1, MIB + EXTRA), (MIB + EXTRA, MIB + EXTRA),
             (4 * MIB, 4 * MIB + EXTRA), (4 * MIB + EXTRA + 1, 8 * MIB + EXTRA),
             (8 * MIB + EXTRA, 8 * MIB + EXTRA), (9 * MIB, 9 * MIB)]
    for n, want in cases:
        p, cap = get(n)
        assert cap == want, (n, cap, want)
        assert lib.blbrs_buffer_put(ctypes.c_void_p(p)) == 0
    s0 = rs.pool_stats()
    p1, _ = get(4 * MIB)
    lib.blbrs_buffer_put(ctypes.c_void_p(p1))
    p2, _ = get(4 * MIB)
    assert p2 == p1  # reused, no new pinned allocation
    lib.blbrs_buffer_put(ctypes.c_void_p(p2))
    s1 = rs.pool_stats()
    assert s1["allocs"] == s0["allocs"]
    assert s1["live_bytes"] == 0
    assert lib.blbrs_buffer_put(ctypes.c_void_p(p2)) == rs.ErrInvalidArgument.code  # double put


@pytest.mark.gpu
def test_pool_buffers_code_zero_copy(oracle_lib):
    """rsEncodeOne with every shard from the pool (CtlRead replies and the parity buffers of
    store.go:1096-1098): Encode, ReconstructAndVerify and ReconstructData bit-exact; the
    calls take the zero-copy path (no staging allocated)."""
    k, m, S = 6, 3, 4 * MIB
    rs.trim()
    enc = rs.New(k, m, devices=[0])
    rng = np.random.default_rng(3)
    sh = [rs.GetBuffer(S) for _ in range(k + m)]
    try:
        for i in range(k):
            sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        for j in range(m):
            sh[k + j][:] = 0xEE  # pooled buffers are not zeroed
        enc.Encode(sh)
        ref = _oracle_parity(oracle_lib, k, m, [sh[i] for i in range(k)])
        for j in range(m):
            assert np.array_equal(sh[k + j], ref[j])
        assert rs.device_stats(0)["staging_bytes"] == 0
        saved = sh[1].copy()
        work = list(sh)
        work[1] = None
        assert enc.ReconstructAndVerify(work, outs={1: sh[1]})
        assert np.array_equal(sh[1], saved)
    finally:
        for b in sh:
            rs.PutBuffer(b)


@pytest.mark.gpu
def test_batcher_on_device_list():
    """A batcher created on an explicit device list serves a host Encode and a host
    ReconstructData call, one launch each (its lanes live on the listed device)."""
    import torch
    k, m, S = 4, 2, 4096
    b = rs.Batcher(max_batch=8, window_us=100, devices=[0])
    try:
        enc = rs.New(k, m, devices=[0])
        enc.SetBatcher(b)
        rng = np.random.default_rng(9)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        sh = data + [np.zeros(S, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        ref = sh[0].copy()
        sh[0] = None
        enc.ReconstructData(sh)
        assert np.array_equal(sh[0], ref)
        r, launches = b.stats()
        assert r == 2 and launches == 2
        enc.SetBatcher(None)
    finally:
        b.close()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_per_read_new_builds_each_plan_once():
    """blb's client makes reedsolomon.New per degraded read and drops it (client/blb/
    reconstruct.go:166-173).  Cores live for the process: 50 reads of one erasure pattern through
    fresh encoders invert and upload its plan once (before round 5 the core died with its last
    handle, and every read rebuilt and re-uploaded -- hipMalloc + hipMemcpy + hipFree per call)."""
    import gc
    k, m, S = 6, 3, 4096
    rng = np.random.default_rng(66)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    full = data + list(N.encode(k, m, data))
    gc.collect()
    before = None
    for i in range(50):
        enc = rs.New(k, m)
        sh = [full[j].copy() if j not in (2,) else None for j in range(k)] + [full[j].copy() for j in range(k, k + m)]
        sh[k + 1] = None   # a parity reply missing too: present = data but 2, parities 6 and 8
        enc.ReconstructData(sh)
        assert np.array_equal(sh[2], full[2])
        del enc
        gc.collect()
        if i == 0:
            before = rs.plan_stats()
    assert rs.plan_stats() == before, (before, rs.plan_stats())


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(6, 3), (10, 3), (12, 5)])
def test_gpu_small_calls_end_on_completion_word(knob, k, m):
    """Small single-launch host calls (pieces of at most 64 KiB) with no verify flag run on the
    small-call kernels and end on their completion word (rs_small.hpp, runtime.hpp
    kDoneMaxPiece / kDoneMaxBytes): Encode, ReconstructData and
    Reconstruct of pageable (staged) and pool (in place) shards, whole 4 KiB chunks and ragged
    ends, are bit-exact against the restatement; each call counts one done wait and none falls
    back to the stream wait.  Verify, and BLBRS_DONE_WORD = 0, wait for the stream and count
    nothing.  One-stripe calls take rs_small1_kernel (entries resolved by the host), a host batch
    of three stripes the multi-stripe rs_small_kernel, whose RS(10,3) / RS(12,5) load 16 inputs
    as one group."""
    knob("BLBRS_DONE_WORD", 1)
    rng = np.random.default_rng(k * 100 + m)
    before = rs.device_stats(0)
    calls = 0
    for S in (4096, 12000, 40000, 65536):
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        full = data + list(N.encode(k, m, data))
        for pooled in (False, True):
            bufs = []

            def shard(src):
                if not pooled:
                    return src.copy()
                b = rs.GetBuffer(S)
                b[:] = src
                bufs.append(b)
                return b
            try:
                enc = rs.New(k, m)
                sh = [shard(full[j]) for j in range(k)] + [shard(np.full(S, 0xEE, np.uint8)) for _ in range(m)]
                enc.Encode(sh)
                for j in range(k, k + m):
                    assert np.array_equal(sh[j], full[j]), (S, pooled, "encode", j)
                sh = [shard(full[j]) for j in range(k + m)]
                sh[1] = None
                sh[k + m - 1] = None
                enc.ReconstructData(sh)
                assert np.array_equal(sh[1], full[1]), (S, pooled, "reconstruct data")
                sh = [shard(full[j]) for j in range(k + m)]
                sh[0] = None
                sh[k] = None
                enc.Reconstruct(sh)
                assert np.array_equal(sh[0], full[0]) and np.array_equal(sh[k], full[k]), (S, pooled, "reconstruct")
                calls += 3
            finally:
                for b in bufs:
                    rs.PutBuffer(b)
    # Several stripes in one small call (a host batch that fits the worker's bounce buffer,
    # runtime.hpp kBounceMaxBytes): the multi-stripe form of the kernel, whole chunk and ragged.
    for S in (4096, 4000):
        host = np.zeros((3, k + m, S), np.uint8)
        host[:, :k] = rng.integers(0, 256, (3, k, S), dtype=np.uint8)
        host[:, k:] = 0xEE
        rs.New(k, m).EncodeHostBatch([[host[b, i] for i in range(k + m)] for b in range(3)])
        for b in range(3):
            ref = N.encode(k, m, [host[b, i] for i in range(k)])
            for j in range(m):
                assert np.array_equal(host[b, k + j], ref[j]), (S, "host batch", b, j)
        calls += 1
    mid = rs.device_stats(0)
    assert mid["done_fallbacks"] == before["done_fallbacks"]
    assert mid["done_waits"] - before["done_waits"] == calls, (before, mid, calls)
    enc = rs.New(k, m)
    # Pieces above 64 KiB (runtime.hpp kDoneMaxPiece) keep rs_code_kernel and the stream wait.
    S = 98765
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    full = data + list(N.encode(k, m, data))
    sh = [f.copy() for f in full]
    sh[0] = None
    enc.ReconstructData(sh)
    assert np.array_equal(sh[0], full[0])
    S = 4096
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    full = data + list(N.encode(k, m, data))
    assert enc.Verify([f.copy() for f in full])
    knob("BLBRS_DONE_WORD", 0)
    sh = [f.copy() for f in full]
    sh[2] = None
    enc.ReconstructData(sh)
    assert np.array_equal(sh[2], full[2])
    after = rs.device_stats(0)
    assert after["done_waits"] == mid["done_waits"] and after["done_fallbacks"] == mid["done_fallbacks"]
