"""blb's two callers of the RS path, restated over the GPU engine (blb_amd/tractserver.py,
client.py, curator.py) and driven the way blb's own unit tests drive the Go code.

CPU tests cover the control logic that never reaches the GPU; `gpu` tests are the parity
tests of the full caller paths (TestRSEncode / TestRSReconstruct of
internal/tractserver/store_test.go:749-879 and test_rs_recovery.go's degraded reads).
"""
import numpy as np
import pytest

from blb_amd.blbcore import (RS_CHUNK_VERSION, RS_PIECE_LENGTH, TRACT_LENGTH, Error, RSChunkID,
                             StorageClass, TSAddr, rs_params)
from blb_amd import curator
from blb_amd.client import Client, ReconstructBehavior, TractPointer
from blb_amd.tractserver import MemTractserverTalker, Store

CID = RSChunkID(0x80000005, 5000)  # store_test.go:757


def addrs(n):
    return [TSAddr(i, f"addr{i}") for i in range(n)]


# ------------------------------------------------------------------ CPU: control logic

def test_core_types():
    assert CID.is_valid()
    assert not RSChunkID(0x00000005, 5000).is_valid()   # regular partition
    assert not RSChunkID(0x80000005, 0).is_valid()
    assert not RSChunkID(0x80000005, 1 << 48).is_valid()
    t = RSChunkID(0x80000005, 0x123456789).to_tract_id()
    assert t.blob == (0x80000005 << 32) | 0x12345 and t.index == 0x6789
    assert [rs_params(c) for c in StorageClass if c] == [(6, 3), (8, 3), (10, 3), (12, 5)]
    assert RS_PIECE_LENGTH == 67043264


def test_store_rsencode_argument_errors():
    s = Store(MemTractserverTalker(), encode_increment_size=5000)
    a = addrs(5)
    assert s.rs_encode(RSChunkID(5, 5000), 12000, a[:3], a[3:], None) == Error.ErrInvalidArgument
    assert s.rs_encode(RSChunkID(0x80000005, (1 << 48) - 2), 12000, a[:3], a[3:], None) == \
        Error.ErrInvalidArgument   # baseid.Add(N+M-1) overflows the 48-bit key
    assert s.rs_encode(CID, 12000, [], a[3:], None) == Error.ErrInvalidArgument  # New(0, 2)
    assert s.rs_encode(CID, 12000, a[:3], a[3:], [0, 1, 2]) == Error.ErrInvalidArgument  # bad indexMap


def test_store_read_failures_before_coding():
    """Short reads -> ErrVersionMismatch; RPC failure -> that error; no coding happens."""
    t = MemTractserverTalker()
    s = Store(t, encode_increment_size=5000)
    a = addrs(5)
    t.add_ctl_read_reply("addr0", np.zeros(5000, np.uint8), Error.ErrEOF)
    t.add_ctl_read_reply("addr1", np.zeros(4999, np.uint8), Error.ErrEOF)
    t.add_ctl_read_reply("addr2", np.zeros(5000, np.uint8), Error.NoError)
    assert s.rs_encode(CID, 5000, a[:3], a[3:], None) == Error.ErrVersionMismatch
    t2 = MemTractserverTalker()   # no scripted replies: ErrRPC
    assert Store(t2, 5000).rs_encode(CID, 5000, a[:3], a[3:], None) == Error.ErrRPC
    assert t2.ctl_read_calls["addr0"][0][1] == RS_CHUNK_VERSION


def test_curator_reconstruct_request_indexmap():
    """reconstruct.go:15-104 -- the SURVEY.md §3B example: RS(5,3), pieces 1 and 5 bad ->
    indexMap [0,2,3,4,6,1,5,-1]."""
    hosts = [TSAddr(10 + i, f"ts{i}") for i in range(8)]
    req, err = curator.reconstruct_request(CID, 5, hosts, [11, 15],
                                           lambda c: [TSAddr(100 + j, f"new{j}") for j in range(c)])
    assert err == Error.NoError
    assert req.index_map == [0, 2, 3, 4, 6, 1, 5, -1]
    assert [h.id for h in req.srcs] == [10, 12, 13, 14, 16]
    assert [h.id for h in req.dests] == [100, 101, 0] and req.tsid == 100
    assert req.length == RS_PIECE_LENGTH
    _, err = curator.reconstruct_request(CID, 5, hosts, [], lambda c: [])
    assert err == Error.ErrInvalidArgument
    _, err = curator.reconstruct_request(CID, 5, hosts, [10, 11, 12, 13], lambda c: [])
    assert err == Error.ErrAllocHost
    e = curator.encode_request(CID, hosts[:6], hosts[6:])
    assert e.index_map is None and e.tsid == 16 and len(e.srcs) == 6


class MemReader:
    """client mem tractserver talker: per-address piece bytes, optional failures."""

    def __init__(self, pieces, down=(), short=()):
        self.pieces, self.down, self.short = pieces, set(down), set(short)
        self.reads = []

    def read(self, addr, tid, version, length, off):
        self.reads.append(addr)
        if addr in self.down:
            return None, Error.ErrRPC
        b = self.pieces[addr][off:off + length]
        if addr in self.short:
            b = b[:-1]
        return b.copy(), (Error.ErrEOF if off + length >= len(self.pieces[addr]) else Error.NoError)

    def read_into(self, addr, tid, version, b, off):
        if addr in self.down:
            return 0, Error.ErrRPC
        src = self.pieces[addr][off:off + len(b)]
        b[:len(src)] = src
        return len(src), Error.NoError


def rs_tract(n, m, target, hosts=None, length=TRACT_LENGTH, offset=0):
    hosts = hosts or [f"ts{i}" for i in range(n + m)]
    cls = {(6, 3): StorageClass.RS_6_3, (8, 3): StorageClass.RS_8_3, (10, 3): StorageClass.RS_10_3,
           (12, 5): StorageClass.RS_12_5}[(n, m)]
    return TractPointer(chunk=CID.add(target), host=hosts[target], tsid=100 + target, offset=offset,
                        length=length, cls=cls, base_chunk=CID, other_hosts=list(hosts),
                        other_tsids=[100 + i for i in range(n + m)])


def test_client_reconstruct_control_paths():
    n, m = 6, 3
    pieces = {f"ts{i}": np.zeros(64, np.uint8) for i in range(9)}
    tr = rs_tract(n, m, 2, length=64)
    # disabled -> the direct read's error comes back
    cli = Client(MemReader(pieces, down={"ts2"}), ReconstructBehavior(enabled=False))
    assert cli.read_one_tract_rs(tr, np.zeros(64, np.uint8), 0).err == Error.ErrRPC
    # TSID not among OtherTSIDs -> ErrInvalidArgument
    cli = Client(MemReader(pieces, down={"ts2"}))
    bad = rs_tract(n, m, 2, length=64)
    bad.tsid = 999
    assert cli.read_one_tract_rs(bad, np.zeros(64, np.uint8), 0).err == Error.ErrInvalidArgument
    # fewer than n other hosts known -> ErrHostNotExist
    hosts = [f"ts{i}" for i in range(9)]
    hosts[0] = hosts[1] = hosts[3] = ""
    tr2 = rs_tract(n, m, 2, hosts=hosts, length=64)
    assert cli.read_one_tract_rs(tr2, np.zeros(64, np.uint8), 0).err == Error.ErrHostNotExist
    # wrong number of OtherHosts -> no reconstruction attempted
    tr3 = rs_tract(n, m, 2, length=64)
    tr3.other_hosts = tr3.other_hosts[:5]
    assert not cli.should_reconstruct(tr3)
    # direct read OK with short tract: zero pad + EOF
    ok = rs_tract(n, m, 2, length=40)
    buf = np.full(64, 7, np.uint8)
    r = Client(MemReader(pieces)).read_one_tract_rs(ok, buf, 0)
    assert r.err == Error.ErrEOF and r.read == 40 and not buf[40:].any()


# ------------------------------------------------------------------ GPU: full caller paths

@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [False, True])
def test_store_rsencode_like_TestRSEncode(pipeline, oracle_lib):
    """store_test.go:749-815: RS(3,2), B=12000, EncodeIncrementSize=5000."""
    N, M, B = 3, 2, 12000
    t = MemTractserverTalker()
    s = Store(t, encode_increment_size=5000, pipeline=pipeline)
    a = addrs(N + M)
    rng = np.random.default_rng(97531)
    data = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(N)]
    for lo, hi in [(0, 5000), (5000, 10000), (10000, 12000)]:
        for i in range(N):
            t.add_ctl_read_reply(a[i].host, data[i][lo:hi], Error.ErrEOF)
        for i in range(N, N + M):
            t.add_ctl_write_reply(a[i].host, Error.NoError)
    assert s.rs_encode(CID, B, a[:N], a[N:], None) == Error.NoError
    full = list(data)
    for i in range(N, N + M):
        parts = []
        for (tid, ver, b, off) in t.ctl_write_calls[a[i].host]:
            assert tid == CID.add(i).to_tract_id() and ver == RS_CHUNK_VERSION
            assert off == sum(len(p) for p in parts)
            parts.append(b)
        full.append(np.concatenate(parts))
    assert oracle_lib.verify(N, M, full)
    from blb_amd import reedsolomon
    assert reedsolomon.New(N, M).Verify(full)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [False, True])
def test_store_reconstruct_like_TestRSReconstruct(pipeline, oracle_lib):
    """store_test.go:817-879: RS(3,2), B=20000, missing 1 (data) and 3 (parity),
    indexMap [0,2,4,1,3]; reconstructAndVerify then CtlWrite of both."""
    N, M, B = 3, 2, 20000
    rng = np.random.default_rng(97532)
    data = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(N)] + [np.zeros(B, np.uint8)] * 0
    data += [np.zeros(B, np.uint8) for _ in range(M)]
    oracle_lib.encode(N, M, data)
    t = MemTractserverTalker()
    s = Store(t, encode_increment_size=8192, pipeline=pipeline)  # several windows
    a = addrs(N + M)
    for lo in range(0, B, 8192):
        hi = min(B, lo + 8192)
        for i in (0, 2, 4):
            t.add_ctl_read_reply(a[i].host, data[i][lo:hi], Error.ErrEOF)
        for i in (1, 3):
            t.add_ctl_write_reply(a[i].host, Error.NoError)
    err = s.rs_encode(CID, B, [a[0], a[2], a[4]], [a[1], a[3]], [0, 2, 4, 1, 3])
    assert err == Error.NoError
    for i in (1, 3):
        got = np.concatenate([b for (_, _, b, _) in t.ctl_write_calls[a[i].host]])
        assert np.array_equal(got, data[i])


@pytest.mark.gpu
def test_store_concurrent_rpcs_with_batcher(oracle_lib):
    """Concurrent RSEncode RPCs (encode and indexMap recovery, half of them pipelined) on
    Stores sharing one Batcher: every RPC writes the oracle's bytes, and the increments of
    different RPCs share launches."""
    import threading

    from blb_amd import reedsolomon
    N, M, B, inc, R = 6, 3, 150_000, 32768, 12
    # A 2 ms window: the RPCs' Python-side gathers and scatters hold the GIL between calls,
    # so without one, calls rarely meet (sharing is what this test checks).
    b = reedsolomon.Batcher(max_batch=64, window_us=2000)
    jobs = []
    for r in range(R):
        rng = np.random.default_rng(1000 + r)
        data = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(N)] + [np.zeros(B, np.uint8) for _ in range(M)]
        oracle_lib.encode(N, M, data)
        t = MemTractserverTalker()
        a = addrs(N + M)
        recover = r % 3 == 2
        srcs = [i for i in range(N + M) if i not in (1, 7)][:N] if recover else list(range(N))
        dsts = [1, 7] if recover else list(range(N, N + M))
        for lo in range(0, B, inc):
            for i in srcs:
                t.add_ctl_read_reply(a[i].host, data[i][lo:lo + inc], Error.ErrEOF)
            for i in dsts:
                t.add_ctl_write_reply(a[i].host, Error.NoError)
        imap = srcs + dsts if recover else None
        jobs.append((Store(t, encode_increment_size=inc, pipeline=r % 2 == 1, batcher=b), t, a, data, srcs, dsts, imap))
    errs = [None] * R
    start = threading.Barrier(R)

    def rpc(r):
        s, t, a, data, srcs, dsts, imap = jobs[r]
        start.wait()
        errs[r] = s.rs_encode(CID, B, [a[i] for i in srcs], [a[i] for i in dsts], imap)

    th = [threading.Thread(target=rpc, args=(r,)) for r in range(R)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert errs == [Error.NoError] * R
    for r, (s, t, a, data, srcs, dsts, imap) in enumerate(jobs):
        for i in dsts:
            got = np.concatenate([w[2] for w in t.ctl_write_calls[a[i].host]])
            assert np.array_equal(got, data[i]), (r, i)
    reqs, launches = b.stats()
    assert launches < reqs, (reqs, launches)
    b.close()


@pytest.mark.gpu
def test_store_reconstruct_verify_failure_is_unknown(oracle_lib):
    """reconstructAndVerify (store.go:1132-1142): with exactly k sources the rebuilt stripe
    is always a codeword, so Verify can only fail when an extra present shard disagrees;
    that failure maps to ErrUnknown (store.go:1102-1107)."""
    from blb_amd import reedsolomon
    N, M, B = 6, 3, 4096
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(N)] + [np.zeros(B, np.uint8) for _ in range(M)]
    oracle_lib.encode(N, M, data)
    s = Store(MemTractserverTalker())
    enc = reedsolomon.New(N, M)
    cur = [d.copy() for d in data]
    cur[1] = None
    cur[8][17] ^= 1                      # a present parity that disagrees
    assert s._code(enc, cur, False, list(range(N + M)), N, B) == Error.ErrUnknown
    cur = [d.copy() for d in data]
    cur[1] = None
    assert s._code(enc, cur, False, list(range(N + M)), N, B) == Error.NoError
    assert np.array_equal(cur[1], data[1])


@pytest.mark.gpu
@pytest.mark.parametrize("off,length", [(4000, 123000), (TRACT_LENGTH - 56789, 98765)])
def test_client_degraded_read_like_TestRSRecovery(off, length):
    """test_rs_recovery.go: kill the tractserver holding a piece, then read windows of it;
    the client reconstructs from n other pieces into the caller's buffer."""
    from blb_amd import reedsolomon
    n, m, target = 6, 3, 2
    rng = np.random.default_rng(off)
    S = max(TRACT_LENGTH, off + length + 4096)  # RS pieces hold several packed tracts
    shards = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(n)] + [np.empty(S, np.uint8) for _ in range(m)]
    reedsolomon.New(n, m).Encode(shards)
    pieces = {f"ts{i}": shards[i] for i in range(n + m)}
    reader = MemReader(pieces, down={"ts2", "ts4"}, short={"ts7"})
    cli = Client(reader)
    tr = rs_tract(n, m, target)
    buf = np.full(length, 0xEE, np.uint8)
    r = cli.read_one_tract_rs(tr, buf, off)
    assert r.err == Error.NoError and r.read == length, r
    assert np.array_equal(buf, shards[target][off:off + length])
    # a tract shorter than the caller's buffer: reconstruct its bytes, zero-pad, ErrEOF
    tr_short = rs_tract(n, m, target, length=5000)
    buf2 = np.full(6000, 0xEE, np.uint8)
    r2 = cli.read_one_tract_rs(tr_short, buf2, 0)
    assert r2.err == Error.ErrEOF and r2.read == 5000, r2
    assert np.array_equal(buf2[:5000], shards[target][:5000]) and not buf2[5000:].any()
    assert cli.reconstructs == 2
