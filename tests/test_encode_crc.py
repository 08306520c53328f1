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

MiB = 1 << 20


def run_case(O, k, m, S, block, B, pad=0, seed=0):
    rng = np.random.default_rng(seed + 131 * k + m + S)
    n = k + m
    host = rng.integers(0, 256, (B, n, S + pad), dtype=np.uint8)
    host[:, k:, :S] = 0xEE                       # un-zeroed output buffers
    dev_full = torch.from_numpy(host).cuda()
    view = dev_full[:, :, :S]                    # strided shards when pad > 0
    enc = rs.New(k, m)
    crc = enc.EncodeBatchCRC(view, block)
    got = dev_full.cpu().numpy()
    blk = S if block <= 0 or block > S else block
    nblocks = (S + blk - 1) // blk
    assert tuple(crc.shape) == (m, B, nblocks)
    crc = crc.cpu().numpy().view(np.uint32)
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


def test_encode_crc_tile_grid_cases(oracle_lib):
    """Shapes the tile-grid kernel (encode_crc_tile.hip) takes: rows <= 4, S a whole number
    of 8 KiB tiles, 16-byte aligned strides, block >= tile.  Block boundaries at many dword
    phases inside a tile (block = tile, tile + 4, 2*tile - 4, 65532), whole-shard frames,
    blocks longer than S, and the last short block; each case is also run on the persistent
    segment kernel (BLBRS_EC_PERSISTENT, read per call)."""
    import os
    T = 8192
    cases = [(6, 3, 128 * T, 65532, 3, 0), (6, 3, 16 * T, T, 2, 16), (6, 3, 16 * T, T + 4, 2, 32),
             (6, 3, 12 * T, 2 * T - 4, 2, 48), (6, 3, 8 * T, 0, 3, 0), (6, 3, 8 * T, 20 * T, 2, 16),
             (3, 2, 10 * T, 65532, 2, 0), (4, 2, 6 * T, T + 12, 2, 16), (6, 1, 8 * T, 65532, 2, 0),
             (8, 3, 8 * T, 65532, 2, 0), (10, 4, 16 * T, 65532, 2, 16), (10, 4, 6 * T, T, 2, 0),
             (12, 4, 8 * T, T + 4, 2, 0), (10, 3, 5 * T, 0, 2, 0), (12, 5, 8 * T, 65532, 2, 0)]
    for i, (k, m, S, block, B, pad) in enumerate(cases):
        run_case(oracle_lib, k, m, S, block, B=B, pad=pad, seed=100 + i)
        os.environ["BLBRS_EC_PERSISTENT"] = "1"
        try:
            run_case(oracle_lib, k, m, S, block, B=B, pad=pad, seed=200 + i)
        finally:
            del os.environ["BLBRS_EC_PERSISTENT"]
