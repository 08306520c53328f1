"""Fused Encode + CRC-32C of the parity (blbrs_encode_crc_dev / Encoder.EncodeBatchCRC) vs the
oracle: parity bytes bit-exact vs the klauspost restatement, every block CRC equal to
crc32.Checksum(block, Castagnoli) of that parity (oracle), nothing written outside the
parity shards.  Covers the fused kernel's shapes (LC = 64 and 32 lane chunks, virtual-zero
segment prefixes of 65532-byte blocks, short tail blocks, whole-shard frames) and the
fallback (uninstantiated k, rows > 5, unaligned lengths)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from blb_amd import reedsolomon as rs  # noqa: E402
from blb_amd.hostcopy import to_device, to_numpy

MiB = 1 << 20


def run_case(O, k, m, S, block, B, pad=0, seed=0):
    rng = np.random.default_rng(seed + 131 * k + m + S)
    n = k + m
    host = rng.integers(0, 256, (B, n, S + pad), dtype=np.uint8)
    host[:, k:, :S] = 0xEE                       # un-zeroed output buffers
    dev_full = to_device(host)
    view = dev_full[:, :, :S]                    # strided shards when pad > 0
    enc = rs.New(k, m)
    crc = enc.EncodeBatchCRC(view, block)
    got = to_numpy(dev_full)
    blk = S if block <= 0 or block > S else block
    nblocks = (S + blk - 1) // blk
    assert tuple(crc.shape) == (m, B, nblocks)
    crc = to_numpy(crc).view(np.uint32)
    for b in range(B):
        sh = [host[b, i, :S].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        O.encode(k, m, sh, use_avx2=True, threads=8)
        for j in range(m):
            assert np.array_equal(got[b, k + j, :S], sh[k + j]), (k, m, S, block, b, j, "parity")
            want = O.crc32c_blocks(sh[k + j], blk)
            assert np.array_equal(crc[j, b], want), (k, m, S, block, b, j, "crc")
        # data shards and the padding after every shard untouched
        assert np.array_equal(got[b, :k], host[b, :k]), (k, m, S, block, b, "data")
        if pad:
            assert np.array_equal(got[b, :, S:], host[b, :, S:]), (k, m, S, block, b, "pad")


@pytest.mark.parametrize("block", [65532, 0, 4096, 65536, 1 << 20])
def test_encode_crc_rs63_tract(oracle_lib, block):
    run_case(oracle_lib, 6, 3, 8 * MiB, block, B=2)


@pytest.mark.parametrize("k,m", [(6, 3), (8, 3), (10, 3), (12, 5), (10, 4), (3, 2), (4, 2), (8, 4), (6, 1)])
def test_encode_crc_shapes(oracle_lib, k, m):
    # 4128704 = the tractserver's last RSEncode increment (67,043,264 % 4 MiB)
    for S, block in ((4128704, 65532), (1 * MiB, 0), (200004, 65532)):
        run_case(oracle_lib, k, m, S, block, B=2, seed=1)


def test_encode_crc_prefix_and_tail_cases(oracle_lib):
    """Segment prefixes inside row 0, several whole virtual rows, tiny blocks, and strided
    shards whose neighbours must not be touched by the masked first-row stores."""
    cases = [(65532, 65532 * 3), (65532, 65532 * 2 + 512), (4, 64), (8, 4100), (60000, 180004),
             (4100, 65536 + 4), (0, 4), (0, 4092), (0, 4096 + 4), (0, 65532), (0, 65536 + 65532),
             (131072, 131072 + 12), (2048, 10000), (12, 300)]
    for i, (block, S) in enumerate(cases):
        run_case(oracle_lib, 6, 3, S, block, B=3, pad=4 * (i % 5), seed=i)
        run_case(oracle_lib, 10, 4, S, block, B=2, pad=4 * ((i + 2) % 5), seed=i)


def test_encode_crc_fallback_shapes(oracle_lib):
    """No fused instantiation (k = 5, 7; rows > 5) or unaligned lengths: coding pass + CRC
    kernel, same results."""
    for k, m, S, block in ((5, 5, 70000, 65532), (7, 3, 65532 * 2, 0), (4, 6, 100000, 4096),
                           (6, 3, 98765, 65532), (6, 3, 12001, 0)):
        run_case(oracle_lib, k, m, S, block, B=2, seed=3)


def test_encode_crc_matches_separate_passes():
    """The fused call equals EncodeBatch followed by ChecksumBatch of each parity row, at the
    BASELINE shard size."""
    from blb_amd import checksum
    k, m, B, S = 6, 3, 16, 8 * MiB
    a = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device="cuda")
    b = a.clone()
    enc = rs.New(k, m)
    crc = enc.EncodeBatchCRC(a, 65532)
    enc.EncodeBatch(b)
    assert torch.equal(a, b)
    for j in range(m):
        sep = checksum.ChecksumBatch(b[:, k + j, :], 65532)
        assert torch.equal(crc[j], sep), j


def test_encode_crc_tile_grid_cases(oracle_lib, knob):
    """Shapes the tile-grid kernel (encode_crc_tile.hip) takes: rows <= 4, S a whole number
    of 8 KiB tiles, 16-byte aligned strides, block >= tile.  Block boundaries at many dword
    phases inside a tile (block = tile, tile + 4, 2*tile - 4, 65532), whole-shard frames,
    blocks longer than S, and the last short block; each case is also run on the persistent
    segment kernel (knob BLBRS_EC_PERSISTENT)."""
    T = 8192
    cases = [(6, 3, 128 * T, 65532, 3, 0), (6, 3, 16 * T, T, 2, 16), (6, 3, 16 * T, T + 4, 2, 32),
             (6, 3, 12 * T, 2 * T - 4, 2, 48), (6, 3, 8 * T, 0, 3, 0), (6, 3, 8 * T, 20 * T, 2, 16),
             (3, 2, 10 * T, 65532, 2, 0), (4, 2, 6 * T, T + 12, 2, 16), (6, 1, 8 * T, 65532, 2, 0),
             (8, 3, 8 * T, 65532, 2, 0), (10, 4, 16 * T, 65532, 2, 16), (10, 4, 6 * T, T, 2, 0),
             (12, 4, 8 * T, T + 4, 2, 0), (10, 3, 5 * T, 0, 2, 0), (12, 5, 8 * T, 65532, 2, 0)]
    for i, (k, m, S, block, B, pad) in enumerate(cases):
        run_case(oracle_lib, k, m, S, block, B=B, pad=pad, seed=100 + i)
        knob("BLBRS_EC_PERSISTENT", 1)
        run_case(oracle_lib, k, m, S, block, B=B, pad=pad, seed=200 + i)
        knob("BLBRS_EC_PERSISTENT", 0)


def _expected_blocks_at(O, buf, block, phase, seed):
    """crc32.Update chain of a file window: buffer byte 0 sits `phase` bytes into block 0."""
    out, pos, i = [], 0, 0
    while pos < buf.size or (i == 0 and buf.size == 0):
        end = min(buf.size, (i + 1) * block - phase)
        out.append(O.crc32c(buf[pos:end], seed if i == 0 else 0))
        pos, i = end, i + 1
    return np.array(out, np.uint32)


def test_encode_crc_piece_in_increment_windows(oracle_lib):
    """rsEncodeOne's real schedule (store.go:1028-1037,1115): a 67,043,264-byte RS piece
    (curator RSPieceLength) is encoded in EncodeIncrementSize = 4 MiB windows (the last one
    4,128,704 bytes), each written at offset 4 MiB * i of the parity piece, whose receiver
    checksums FILE-aligned 65532-byte ChecksumFile blocks and chains appends with crc32.Update
    (pkg/disk/checksum_block.go:76-81).  Per window: EncodeBatchCRC(phase = offset mod 65532,
    seed = the previous window's last, partial block CRC).  The per-window outputs, combined,
    must equal the oracle's 65532-byte block CRCs of the whole parity piece; the same for
    ChecksumBatch(phase, seeds) over the parity rows."""
    from blb_amd import checksum
    O = oracle_lib
    k, m, B = 6, 3, 2
    L, inc, blk = 67043264, 4 << 20, 65532
    g = torch.Generator(device="cuda")
    g.manual_seed(97531)
    piece = torch.empty((B, k + m, L), dtype=torch.uint8, device="cuda")
    piece[:, :k].random_(0, 256, generator=g)
    piece[:, k:].fill_(0xEE)
    enc = rs.New(k, m)
    combined = [[[] for _ in range(B)] for _ in range(m)]
    combined2 = [[[] for _ in range(B)] for _ in range(m)]
    prev = prev2 = None
    off = 0
    while off < L:
        ln = min(inc, L - off)
        phase = off % blk
        win = piece[:, :, off:off + ln]
        seeds = prev if phase else None
        crc = enc.EncodeBatchCRC(win, blk, phase=phase, seeds=seeds)
        # the same windows through the plain CRC entry point, row by row
        crc2 = torch.stack([checksum.ChecksumBatch(win[:, k + j], blk, phase=phase,
                                                   seeds=None if not phase else prev2[j].contiguous())
                            for j in range(m)])
        assert tuple(crc.shape) == (m, B, (phase + ln + blk - 1) // blk)
        last_partial = (off + ln) % blk != 0 and off + ln < L
        for c, acc in ((crc, combined), (crc2, combined2)):
            h = to_numpy(c).view(np.uint32)
            for j in range(m):
                for b in range(B):
                    acc[j][b].extend(h[j, b, :-1] if last_partial else h[j, b])
        prev = crc[:, :, -1].contiguous()
        prev2 = crc2[:, :, -1]
        off += ln
    host = to_numpy(piece)
    for b in range(B):
        sh = [host[b, i] for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
        O.encode(k, m, sh, use_avx2=True, threads=8)
        for j in range(m):
            assert np.array_equal(host[b, k + j], sh[k + j]), (b, j, "parity")
            want = O.crc32c_blocks(sh[k + j], blk)
            assert len(combined[j][b]) == want.size
            assert np.array_equal(np.array(combined[j][b], np.uint32), want), (b, j, "fused")
            assert np.array_equal(np.array(combined2[j][b], np.uint32), want), (b, j, "crc32c_dev_at")


@pytest.mark.parametrize("k,m", [(6, 3), (10, 4), (5, 5), (12, 5)])
def test_encode_crc_phase_and_seed_shapes(oracle_lib, k, m):
    """Phase / seed on every path: the tile kernel (aligned phases, partial last tiles), the
    2-pass fallback (k = 5, rows = 5, unaligned phases or lengths)."""
    O = oracle_lib
    rng = np.random.default_rng(k * 100 + m)
    enc = rs.New(k, m)
    cases = [(4128704, 65532, 256), (1 << 20, 65532, 65528), (200000, 4096, 4092), (8192 * 3 + 48, 8192, 4),
             (70001, 65532, 1000), (65536, 65532, 65531), (4096, 65532, 65000), (16, 65532, 0), (1 << 20, 0, 0),
             # blocks of > 64 tiles: the two-level tile fold (chunks of 32 tiles), with block
             # ends inside tiles, a partial last tile and a straddling first block
             ((3 << 20) + 16, 4 << 20, 12), (6 << 20, (2 << 20) + 4, 1000), ((2 << 20) + 48, 1 << 20, 0)]
    for S, block, phase in cases:
        B = 2
        host = rng.integers(0, 256, (B, k + m, S), dtype=np.uint8)
        host[:, k:] = 0x5A
        dev = to_device(host)
        seeds_h = rng.integers(0, 1 << 32, (m, B), dtype=np.uint64).astype(np.uint32)
        seeds = to_device(seeds_h.view(np.int32)) if block else None
        crc = to_numpy(enc.EncodeBatchCRC(dev, block, phase=phase, seeds=seeds)).view(np.uint32)
        got = to_numpy(dev)
        blk = block or S
        for b in range(B):
            sh = [host[b, i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
            O.encode(k, m, sh, use_avx2=True, threads=8)
            for j in range(m):
                assert np.array_equal(got[b, k + j], sh[k + j]), (k, m, S, block, phase, b, j, "parity")
                want = _expected_blocks_at(O, sh[k + j], blk, phase if block else 0,
                                           int(seeds_h[j, b]) if block else 0)
                assert np.array_equal(crc[j, b], want), (k, m, S, block, phase, b, j, "crc")


def test_encode_crc_at_rejects_bad_phase():
    enc = rs.New(6, 3)
    st = torch.zeros((1, 9, 8192), dtype=torch.uint8, device="cuda")
    with pytest.raises(rs.ErrInvalidArgument):
        enc.EncodeBatchCRC(st, 65532, phase=65532)


@pytest.mark.parametrize("k,m,lost,data_only", [(6, 3, (1,), True), (6, 3, (0, 7), False), (10, 4, (1, 7), False),
                                                (12, 5, (2, 5, 13, 16), False), (12, 5, (3, 15), True),
                                                (5, 5, (0, 6), False), (3, 2, (1, 3), False)])
def test_reconstruct_crc_vs_oracle(oracle_lib, k, m, lost, data_only):
    """blbrs_reconstruct_crc_dev_at: the recovery RPC rebuilds the missing pieces and the
    receiver checksums them (store.go:1110-1120, pkg/disk/checksum_block.go:76-81).  Rebuilt
    bytes equal the originals; each rebuilt shard's block CRCs (file-aligned phase, seeded
    first block) equal the oracle's; survivors untouched.  (5,5) has no fused instantiation
    and runs the two-pass fallback."""
    O = oracle_lib
    rng = np.random.default_rng(7 * k + m + len(lost))
    enc = rs.New(k, m)
    present = [i not in lost for i in range(k + m)]
    rows = [i for i in sorted(lost) if i < k or not data_only]
    for S, block, phase in ((4128704, 65532, 256), (1 << 20, 0, 0), (200000, 4096, 4092), (70001, 65532, 1000)):
        B = 2
        full = np.empty((B, k + m, S), np.uint8)
        for b in range(B):
            sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
            O.encode(k, m, sh, use_avx2=True, threads=8)
            full[b] = np.stack(sh)
        host = full.copy()
        host[:, list(lost)] = 0xC3
        dev = to_device(host)
        seeds_h = rng.integers(0, 1 << 32, (len(rows), B), dtype=np.uint64).astype(np.uint32)
        seeds = to_device(seeds_h.view(np.int32)) if block else None
        crc = enc.ReconstructBatchCRC(dev, present, block, data_only=data_only, phase=phase, seeds=seeds)
        crc = to_numpy(crc).view(np.uint32)
        got = to_numpy(dev)
        blk = block or S
        assert crc.shape[0] == len(rows)
        for b in range(B):
            for i in range(k + m):
                if i in lost and i not in rows:
                    assert (got[b, i] == 0xC3).all(), (k, m, S, b, i, "untouched parity")
                else:
                    assert np.array_equal(got[b, i], full[b, i]), (k, m, S, b, i, "bytes")
            for j, i in enumerate(rows):
                want = _expected_blocks_at(O, full[b, i], blk, phase if block else 0, int(seeds_h[j, b]) if block else 0)
                assert np.array_equal(crc[j, b], want), (k, m, S, block, phase, b, i, "crc")
    assert enc.ReconstructBatchCRC(torch.zeros((1, k + m, 64), dtype=torch.uint8, device="cuda"),
                                   [True] * (k + m), 65532) is None
