"""PackTracts: the curator's first-fit-decreasing packer
(internal/curator/pack_tracts.go:124-169), checkTractSpec and Store.PackTracts
(internal/tractserver/store.go:922-1009), with the byte assembly on the GPU
(blbrs_pack_dev) checked bit-exact against oracle/rs_numpy.pack_piece.  The golden bytes
of test_store_pack_tracts are the reference's own (store_test.go:703-746)."""
import numpy as np
import pytest

from blb_amd import pack
from blb_amd.blbcore import (RS_CHUNK_VERSION, Error, RSChunkID, TSAddr, TractID,
                             blob_id_from_parts, tract_id_from_parts)
from blb_amd.tractserver import MemTractserverTalker, Store
from blb_amd.hostcopy import to_device, to_numpy
from oracle import rs_numpy as N

gpu = pytest.mark.gpu
CID = RSChunkID(0x80000555, 5555)
ADDRS = [TSAddr(1, "a1"), TSAddr(2, "a2"), TSAddr(3, "a3")]
TID = tract_id_from_parts(blob_id_from_parts(1, 1), 0)


def _spec(tid=TID, frm=ADDRS, version=1, offset=0, length=0):
    return pack.PackTractSpec(tid, list(frm), version, offset, length)


# ---- curator packer (CPU) ----

def test_pack_tracts_first_fit_decreasing():
    P = pack.PAD_TO_LENGTH
    target = 10 * P
    lens = [9 * P, 3 * P - 5, P + 1, 2 * P, 1, P, -1, 4 * P]
    tracts = [_spec(tract_id_from_parts(blob_id_from_parts(1, i + 1), 0), length=n) for i, n in enumerate(lens)]
    chunks = pack.pack_tracts(tracts, target)
    # FFD by hand (largest first, first chunk with room): 9P->c0; 4P->c1; 3P-5 (pads to 3P)
    # ->c1@4P; 2P->c1@7P; P+1 (pads to 2P) fits nowhere -> c2; P->c0@9P; 1 (pads to P)->c1@9P
    got = sorted((c.length, sorted((t.length, t.offset) for t in c.tracts)) for c in chunks)
    want = sorted([
        (10 * P, sorted([(9 * P, 0), (P, 9 * P)])),
        (10 * P, sorted([(4 * P, 0), (3 * P - 5, 4 * P), (2 * P, 7 * P), (1, 9 * P)])),
    ])
    assert got == want
    # c2 (2P) is < 90 % full and waits for the next round; the unstattable tract is skipped
    placed = {id(t) for c in chunks for t in c.tracts}
    assert all(id(t) not in placed for t in tracts if t.length in (P + 1, -1))


def test_pack_tracts_properties():
    rng = np.random.default_rng(5)
    target = 64 << 20
    tracts = [_spec(tract_id_from_parts(blob_id_from_parts(1, i + 1), 0), length=int(n))
              for i, n in enumerate(rng.integers(-1000, 8 << 20, 300))]
    chunks = pack.pack_tracts(tracts, target)
    slop = int(np.float32(target) * np.float32(pack.ACCEPT_SLOP))
    assert [c.length for c in chunks] == sorted((c.length for c in chunks), reverse=True)
    for c in chunks:
        assert target - c.length <= slop and c.length <= target
        end = 0
        for t in sorted(c.tracts, key=lambda t: t.offset):
            assert t.length >= 0 and t.offset % pack.PAD_TO_LENGTH == 0 and t.offset >= end
            end = t.offset + pack.padded_length(t.length)
        assert end == c.length


def test_check_tract_spec_invalid_cases():
    """store_test.go:647-680 TestPackTractsInvalid, as Store.pack_tracts return values."""
    s = Store(MemTractserverTalker())
    cases = [
        (-100, []),                                                          # negative length
        (1000, [_spec(tid=TractID(0, 0), offset=0, length=500)]),           # invalid tract id
        (1000, [_spec(frm=[], offset=0, length=500)]),                       # no from
        (1000, [_spec(offset=0, length=1500)]),                              # too long
        (1000, [_spec(offset=1500, length=500)]),                            # starting too high
        (1000, [_spec(offset=700, length=200), _spec(offset=100, length=200)]),  # out of order
    ]
    for length, srcs in cases:
        assert s.pack_tracts(length, srcs, CID) == Error.ErrInvalidArgument, (length, srcs)
    assert s.pack_tracts(1000, [], RSChunkID(0, 5)) == Error.ErrInvalidArgument   # bad dest


def test_store_pack_tracts_rpc_error():
    """store_test.go:682-701: no read replies -> ErrRPC, nothing stored."""
    s = Store(MemTractserverTalker())
    t1 = tract_id_from_parts(blob_id_from_parts(1, 2), 0)
    t2 = tract_id_from_parts(blob_id_from_parts(1, 7), 0)
    err = s.pack_tracts(1000, [_spec(t1, offset=100, length=200), _spec(t2, offset=700, length=200)], CID)
    assert err == Error.ErrRPC
    assert s.read(CID.to_tract_id(), RS_CHUNK_VERSION, 1000, 0)[1] == Error.ErrNoSuchTract


def test_oracle_pack_piece_golden():
    got = N.pack_piece(49, [(b"this is some data", 2), (b"this is some more data", 22)])
    assert got == b"\x00\x00this is some data\x00\x00\x00this is some more data\x00\x00\x00\x00\x00"
    assert N.pack_piece(1000, []) == b""


# ---- GPU ----

def _torch():
    return pytest.importorskip("torch")


@gpu
def test_store_pack_tracts():
    """store_test.go:703-746 TestPackTracts: replica fallback, holes and pad, read back."""
    tt = MemTractserverTalker()
    s = Store(tt)
    t1 = tract_id_from_parts(blob_id_from_parts(1, 2), 0)
    t2 = tract_id_from_parts(blob_id_from_parts(1, 7), 0)
    data1, data2 = b"this is some data", b"this is some more data"
    u8 = lambda b: np.frombuffer(b, np.uint8)  # noqa: E731
    tt.add_ctl_read_reply("a1", u8(b"oops"), Error.ErrRPC)          # tract 1: first fails
    tt.add_ctl_read_reply("a2", u8(data1), Error.ErrEOF)            #   second is good
    tt.add_ctl_read_reply("a1", u8(b"wrong length"), Error.ErrEOF)  # tract 2: wrong length
    tt.add_ctl_read_reply("a2", np.zeros(0, np.uint8), Error.ErrCorruptData)  # corrupt
    tt.add_ctl_read_reply("a3", u8(data2), Error.ErrEOF)            #   third is ok
    err = s.pack_tracts(len(data1) + len(data2) + 10, [
        _spec(t1, offset=2, length=len(data1)),
        _spec(t2, offset=len(data1) + 5, length=len(data2)),
    ], CID)
    assert err == Error.NoError
    b, err = s.read(CID.to_tract_id(), RS_CHUNK_VERSION, 1000, 0)
    assert err == Error.ErrEOF
    assert bytes(b) == b"\x00\x00this is some data\x00\x00\x00this is some more data\x00\x00\x00\x00\x00"
    assert [c[2] for c in tt.ctl_read_calls["a1"]] == [8 << 20, 8 << 20]  # CtlRead of TractLength


def _random_extents(rng, npieces, piece_len, pool_len):
    ext = []
    for p in range(npieces):
        off = int(rng.integers(0, 40))
        while off < piece_len:
            ln = int(rng.integers(0, min(piece_len - off, 300000) + 1))
            src = int(rng.integers(0, pool_len - ln + 1))
            ext.append((src, off, ln, p))
            off += ln + int(rng.choice([0, 0, 1, 3, 4, 17, 65532, 100000]))
    return ext


@gpu
@pytest.mark.parametrize("piece_len", [1, 15, 16, 4096, 65536, 65537, 1_000_003, 8 << 20])
def test_gpu_pack_pieces_vs_oracle(piece_len):
    torch = _torch()
    rng = np.random.default_rng(piece_len)
    npieces = 3
    pool = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    dpool = to_device(pool)
    ext = _random_extents(rng, npieces, piece_len, pool.size)
    stride = piece_len + int(rng.integers(0, 33))
    dst = torch.full((npieces, stride), 0xA5, dtype=torch.uint8, device="cuda")  # stale bytes
    pack.PackPieces(dst, piece_len, [(dpool[s:], off, ln, p) for s, off, ln, p in ext])
    got = to_numpy(dst)
    for p in range(npieces):
        want = N.pack_piece(piece_len, [(pool[s:s + ln].tobytes(), off) for s, off, ln, q in ext if q == p])
        want = want.ljust(piece_len, b"\0")  # a piece with no extents still spans piece_len
        assert got[p, :piece_len].tobytes() == want, p
        assert (got[p, piece_len:] == 0xA5).all()  # nothing written past the piece


@gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_pack_kernel_edges_vs_oracle(seed):
    """pack_kernel (pack.hip) against the oracle: random extents, plus regions whose 16-byte
    chunk count sits at the wave and workgroup edges the DPP neighbour exchange depends on (0, 1,
    63-65, 255-257, 1023-1025 chunks), from every source misalignment 0..15 and destination
    offsets that leave heads and tails."""
    torch = _torch()
    rng = np.random.default_rng(1006 + seed)
    pool = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
    dpool = to_device(pool)
    piece_len = 1_000_003
    ext = _random_extents(rng, 2, piece_len, pool.size)
    p, off = 2, 0
    for chunks in (0, 1, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025):
        for mis in range(16):
            ln = 16 * chunks + int(rng.integers(0, 16))
            head = int(rng.integers(0, 16))
            if off + head + ln > piece_len:
                p, off = p + 1, 0
            src = 16 * int(rng.integers(0, (pool.size - ln - 32) // 16)) + mis
            ext.append((src, off + head, ln, p))
            off += head + ln
    npieces = p + 1
    dst = torch.full((npieces, piece_len), 0xA5, dtype=torch.uint8, device="cuda")
    pack.PackPieces(dst, piece_len, [(dpool[s:], o, ln, q) for s, o, ln, q in ext])
    got = to_numpy(dst)
    for q in range(npieces):
        want = N.pack_piece(piece_len, [(pool[s:s + ln].tobytes(), o) for s, o, ln, r in ext if r == q])
        assert got[q].tobytes() == want.ljust(piece_len, b"\0"), q


@gpu
def test_gpu_pack_pinned_sources_and_destination():
    torch = _torch()
    rng = np.random.default_rng(9)
    piece_len = 300_001
    pool = torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8)).pin_memory()
    ext = _random_extents(rng, 2, piece_len, pool.numel())
    for dst in (torch.full((2, piece_len), 7, dtype=torch.uint8).pin_memory(),
                torch.full((2, piece_len), 7, dtype=torch.uint8, device="cuda")):
        pack.PackPieces(dst, piece_len, [(pool[s:], off, ln, p) for s, off, ln, p in ext])
        torch.cuda.synchronize()
        got = to_numpy(dst)
        for p in range(2):
            want = N.pack_piece(piece_len, [(pool[s:s + ln].numpy().tobytes(), off)
                                            for s, off, ln, q in ext if q == p]).ljust(piece_len, b"\0")
            assert got[p].tobytes() == want


@gpu
def test_gpu_pack_rejects_bad_extents():
    torch = _torch()
    src = torch.zeros(100, dtype=torch.uint8, device="cuda")
    dst = torch.zeros((2, 1000), dtype=torch.uint8, device="cuda")
    bad = [
        [(src, 10, 50, 0), (src, 40, 10, 0)],    # overlap
        [(src, 500, 10, 0), (src, 100, 10, 0)],  # out of order
        [(src, 995, 10, 0)],                      # past the piece
        [(src, 0, 10, 1), (src, 0, 10, 0)],      # pieces out of order
        [(src, 0, 10, 2)],                        # no such piece
        [(np.zeros(10, np.uint8), 0, 10, 0)],    # pageable host source
    ]
    for ext in bad:
        with pytest.raises(pack.ErrInvalidArgument):
            pack.PackPieces(dst, 1000, ext)


@gpu
def test_gpu_pack_then_encode_matches_oracle():
    """curator packTracts -> device PackTracts of k pieces -> RS encode == oracle."""
    torch = _torch()
    from blb_amd import reedsolomon
    rng = np.random.default_rng(21)
    k, m, piece_len = 6, 3, 4 << 20
    tracts, blobs = [], {}
    for i in range(90):  # ~45 MiB of tracts: enough for k chunks >= 90 % full
        n = int(rng.integers(1, 1 << 20))
        t = _spec(tract_id_from_parts(blob_id_from_parts(1, i + 1), 0), length=n)
        blobs[id(t)] = to_device(rng.integers(0, 256, n, dtype=np.uint8))
        tracts.append(t)
    chunks = pack.pack_tracts(tracts, piece_len)[:k]
    assert len(chunks) == k
    stripe = torch.empty((k + m, piece_len), dtype=torch.uint8, device="cuda")
    ext = [(blobs[id(t)], t.offset, t.length, p) for p, c in enumerate(chunks)
           for t in sorted(c.tracts, key=lambda t: t.offset)]
    pack.PackPieces(stripe[:k], piece_len, ext)
    enc = reedsolomon.New(k, m)
    enc.EncodeBatch(stripe.view(1, k + m, piece_len))
    got = to_numpy(stripe)
    data = [np.frombuffer(N.pack_piece(piece_len, [(to_numpy(blobs[id(t)]).tobytes(), t.offset)
                                                   for t in c.tracts]).ljust(piece_len, b"\0"), np.uint8)
            for c in chunks]
    for i in range(k):
        assert np.array_equal(got[i], data[i]), i
    par = N.encode(k, m, [d[:65536] for d in data])  # sampled columns: oracle is pure numpy
    for j in range(m):
        assert np.array_equal(got[k + j, :65536], par[j]), j


def _long_extents(rng, npieces, piece_len, pool_len):
    """Multi-MiB tracts at padToLength multiples (the packer's layout): most tiles lie inside
    one extent (the fused kernel's COPY path) with every source misalignment."""
    ext = []
    for p in range(npieces):
        off = 0
        while True:
            ln = int(rng.integers(1, min(piece_len, 3 << 20) + 1))
            if off + ln > piece_len:
                break
            src = int(rng.integers(0, pool_len - ln + 1))
            ext.append((src, off, ln, p))
            off += pack.padded_length(ln)
    return ext


@gpu
@pytest.mark.parametrize("k,m,S,layout", [(6, 3, 8 << 20, "long"), (6, 3, 1_000_003, "short"),
                                          (10, 4, 4 << 20, "long"), (12, 5, 65537, "short"),
                                          (3, 2, 20000, "short"), (5, 5, 70001, "short"),
                                          (6, 3, 4096, "long"), (8, 3, 3 << 20, "long")])
def test_gpu_pack_encode_fused_vs_oracle(oracle_lib, k, m, S, layout):
    """blbrs_pack_encode_dev: data shards == oracle pack_piece (tracts at offsets, zero
    holes and pad) and parity == oracle encode of those pieces; stale bytes everywhere
    before the call; (5,5) has no fused instantiation and runs pack then encode."""
    torch = _torch()
    from blb_amd import reedsolomon
    rng = np.random.default_rng(S + 7 * k + m)
    B = 3
    pool = rng.integers(0, 256, 12 << 20, dtype=np.uint8)
    dpool = to_device(pool)
    mk = _long_extents if layout == "long" else _random_extents
    ext = mk(rng, B * k, S, pool.size)
    st = torch.full((B, k + m, S), 0xEE, dtype=torch.uint8, device="cuda")
    enc = reedsolomon.New(k, m)
    pack.PackEncode(enc, st, [(dpool[s:], off, ln, p) for s, off, ln, p in ext])
    got = to_numpy(st)
    for b in range(B):
        data = []
        for j in range(k):
            p = b * k + j
            want = N.pack_piece(S, [(pool[s:s + ln].tobytes(), off) for s, off, ln, q in ext if q == p])
            want = np.frombuffer(want.ljust(S, b"\0"), np.uint8)
            assert np.array_equal(got[b, j], want), (b, j, "data")
            data.append(want.copy())
        sh = data + [np.zeros(S, np.uint8) for _ in range(m)]
        oracle_lib.encode(k, m, sh, use_avx2=True, threads=8)
        for j in range(m):
            assert np.array_equal(got[b, k + j], sh[k + j]), (b, j, "parity")


@gpu
def test_gpu_pack_encode_equals_pack_then_encode():
    """The fused call equals PackPieces over the data shards followed by EncodeBatch, at the
    BASELINE tract size."""
    torch = _torch()
    from blb_amd import reedsolomon
    rng = np.random.default_rng(5)
    k, m, B, S = 6, 3, 8, 8 << 20
    dpool = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device="cuda")
    ext = _long_extents(rng, B * k, S, dpool.numel())
    a = torch.full((B, k + m, S), 0x33, dtype=torch.uint8, device="cuda")
    b = a.clone()
    enc = reedsolomon.New(k, m)
    pack.PackEncode(enc, a, [(dpool[s:], off, ln, p) for s, off, ln, p in ext])
    flat = b.view(B * (k + m), S)
    rows = torch.arange(B * (k + m), device="cuda").view(B, k + m)[:, :k].reshape(-1)
    tmp = torch.empty((B * k, S), dtype=torch.uint8, device="cuda")
    pack.PackPieces(tmp, S, [(dpool[s:], off, ln, p) for s, off, ln, p in ext])
    flat[rows] = tmp
    enc.EncodeBatch(b)
    assert torch.equal(a, b)
