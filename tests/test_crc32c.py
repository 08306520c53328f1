"""CRC-32C (Castagnoli) of shard blocks: oracle pinning on CPU, GPU kernel bit-exact vs the
oracle.  The block sizes are blb's: 65532-byte ChecksumFile blocks
(pkg/disk/checksum_block.go:18-34) and whole-buffer bulk RPC frames (pkg/rpc/bulk_codec.go:47)."""
import numpy as np
import pytest

from oracle import rs_numpy as N
from blb_amd.hostcopy import to_device, to_numpy

CHECK = 0xE3069283  # CRC-32C("123456789"), the standard check value


def test_oracle_crc32c_pinned(oracle_lib):
    assert oracle_lib.crc32c(b"123456789") == CHECK
    assert N.crc32c(b"123456789") == CHECK
    assert oracle_lib.crc32c(b"") == 0
    rng = np.random.default_rng(7)
    for n in (1, 3, 100, 4099):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        assert oracle_lib.crc32c(d) == N.crc32c(d.tobytes())
        # crc32.Update chaining (checksumBlock.append, checksum_block.go:76-80)
        cut = n // 3
        assert oracle_lib.crc32c(d[cut:], oracle_lib.crc32c(d[:cut])) == oracle_lib.crc32c(d)
    blocks = oracle_lib.crc32c_blocks(np.arange(200000, dtype=np.uint32).view(np.uint8), 65532)
    assert blocks.size == (800000 + 65531) // 65532


gpu = pytest.mark.gpu


def _torch():
    return pytest.importorskip("torch")


@gpu
@pytest.mark.parametrize("block", [65532, 0, 4096, 1000, 1, 65536, 1 << 20])
def test_gpu_crc32c_vs_oracle(oracle_lib, block):
    from blb_amd import checksum
    torch = _torch()
    rng = np.random.default_rng(block + 1)
    for n in (1, 3, 4, 15, 65532, 65536, 98765, 3 * 65532 + 7, (8 << 20) + 13):
        if block == 1 and n > 5000:
            continue
        d = rng.integers(0, 256, n, dtype=np.uint8)
        want = oracle_lib.crc32c_blocks(d, block or n)
        got = checksum.Checksum(d, block)                          # host path (staged)
        assert np.array_equal(got, want), (n, block)
        t = to_device(d)
        got_d = checksum.as_uint32(checksum.Checksum(t, block))    # device path
        assert np.array_equal(got_d, want), (n, block, "dev")


@gpu
def test_gpu_crc32c_unaligned_and_pinned(oracle_lib):
    from blb_amd import checksum
    torch = _torch()
    rng = np.random.default_rng(3)
    base = rng.integers(0, 256, 300000, dtype=np.uint8)
    dbase = to_device(base)
    for off in (1, 2, 3, 5, 16):
        d = base[off:off + 200000]
        want = oracle_lib.crc32c_blocks(d, 65532)
        assert np.array_equal(checksum.as_uint32(checksum.Checksum(dbase[off:off + 200000], 65532)), want), off
    pinned = torch.from_numpy(base.copy()).pin_memory().numpy()
    assert np.array_equal(checksum.Checksum(pinned, 65532), oracle_lib.crc32c_blocks(base, 65532))


@gpu
def test_gpu_crc32c_batch_of_parity_shards(oracle_lib):
    """The use on the RS path: checksum every parity shard of a device-resident batch right
    after encoding it (ChecksumFile blocks and the whole-shard bulk-frame CRC)."""
    from blb_amd import checksum, reedsolomon
    torch = _torch()
    k, m, B, S = 6, 3, 8, (1 << 20) + 100
    enc = reedsolomon.New(k, m)
    st = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device="cuda")
    enc.EncodeBatch(st)
    parity = st[:, k:, :].reshape(B * m, S)           # strided rows
    crc_blocks = checksum.as_uint32(checksum.ChecksumBatch(parity, 65532))
    crc_whole = checksum.as_uint32(checksum.ChecksumBatch(parity, 0))
    host = to_numpy(parity)
    for r in range(B * m):
        assert np.array_equal(crc_blocks[r], oracle_lib.crc32c_blocks(host[r], 65532)), r
        assert int(crc_whole[r, 0]) == oracle_lib.crc32c(host[r]), r


@gpu
def test_gpu_crc32c_aligned_shapes(oracle_lib):
    """Dword-aligned lengths/blocks/strides take the streaming kernel: sweep the virtual
    zero-prefix cases (none, inside row 0, several whole rows) and strided batches."""
    from blb_amd import checksum
    torch = _torch()
    rng = np.random.default_rng(11)
    cases = [(65532, 4 * 65532), (65536, 65536 * 3), (4096, 4096 * 5 + 8), (4, 64), (8, 4100),
             (60000, 180004), (4100, 65536 + 4), (0, 4), (0, 4092), (0, 4096 + 4), (0, 65532),
             (0, 65536 + 65532), (131072, 131072 + 12)]
    for _ in range(12):
        blk = int(rng.integers(1, 40000)) * 4
        cases.append((blk, int(rng.integers(1, 80000)) * 4))
    for blk, n in cases:
        batch = int(rng.integers(1, 4))
        stride = n + 4 * int(rng.integers(0, 40))
        host = rng.integers(0, 256, (batch, stride), dtype=np.uint8)
        dev = to_device(host)
        got = checksum.as_uint32(checksum.ChecksumBatch(dev[:, :n], blk))
        for r in range(batch):
            want = oracle_lib.crc32c_blocks(host[r, :n], blk or n)
            assert np.array_equal(got[r], want), (blk, n, r)


def test_oracle_crc32c_hw_equals_table(oracle_lib):
    """The CPU-baseline restatement of Go's SSE4.2 path (three interleaved 8 KiB streams)
    returns exactly the table oracle's CRCs."""
    from oracle import oracle as O
    if not O.lib().rso_have_sse42():
        pytest.skip("no SSE4.2 on this host")
    rng = np.random.default_rng(17)
    for n, block in [(1, 1), (7, 0), (24575, 0), (24576, 0), (24577, 0), (3 * 65532 + 9, 65532),
                     (200_001, 4096), ((1 << 20) + 5, 0)]:
        d = rng.integers(0, 256, n, dtype=np.uint8)
        blk = block or n
        assert np.array_equal(O.crc32c_blocks_hw(d, blk, threads=3), oracle_lib.crc32c_blocks(d, blk)), (n, blk)
    assert O.crc32c_blocks_hw(np.frombuffer(b"123456789", np.uint8), 9)[0] == CHECK


@gpu
def test_gpu_crc32c_at_phase_and_seeds(oracle_lib):
    """blbrs_crc32c_dev_at: rows that are file windows starting `phase` bytes into a block,
    block 0 continuing a seed (crc32.Update, checksum_block.go:80); streaming kernel (dword
    phases and lengths) and segment kernel (odd phases, odd lengths, unaligned rows)."""
    from blb_amd import checksum
    torch = _torch()
    O = oracle_lib
    rng = np.random.default_rng(11)
    cases = [(65532, 256, 4194304), (65532, 65528, 1 << 20), (65532, 4, 65532), (65532, 65000, 4096),
             (65532, 1, 100003), (4096, 4092, 70000), (1000, 999, 12345), (65536, 12, 3 * 65536 + 8),
             (65532, 513, 7), (1 << 20, 4, 3 << 20)]
    for block, phase, n in cases:
        for lead in (0, 3):
            B = 3
            base = to_device(rng.integers(0, 256, (B, n + 16), dtype=np.uint8))
            rows = base[:, lead:lead + n]
            seeds_h = rng.integers(0, 1 << 32, B, dtype=np.uint64).astype(np.uint32)
            seeds = to_device(seeds_h.view(np.int32))
            got = checksum.as_uint32(checksum.ChecksumBatch(rows, block, phase=phase, seeds=seeds))
            host = to_numpy(rows)
            for b in range(B):
                want, pos, i = [], 0, 0
                while pos < n:
                    end = min(n, (i + 1) * block - phase)
                    want.append(O.crc32c(host[b, pos:end], int(seeds_h[b]) if i == 0 else 0))
                    pos, i = end, i + 1
                assert np.array_equal(got[b], np.array(want, np.uint32)), (block, phase, n, lead, b)
