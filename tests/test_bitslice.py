"""The compiled bit-plane encode network (gf_bitslice.hpp) against the oracle and against the
v_perm table path it replaces for encode passes.  The knob BLBRS_BITSLICE (blbrs_set_tuning) = 2
puts every compiled shape on the network (by default only k + m > 9), = 0 on the tables.

Every compiled shape (k in {3, 4, 6, 8, 10, 12}, m = 1..5) runs through the four kernels that
carry the network -- rs_code_kernel in store and verify mode, the fused encode+CRC tile kernel
and PackTracts + Encode -- on shard lengths that mix whole tiles (network) with a ragged last
tile (the per-lane table path inside the same launch).  Parity must equal the klauspost
restatement byte for byte, Verify must accept it and reject a one-byte corruption, and the
table path must write the same bytes.  Parity rows are the oracle's, not the library's: the
constexpr matrix is checked against reedsolomon.go buildMatrix's restatement on the CPU
(tests/test_capi.py) and here through the bytes it produces."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from blb_amd import pack  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402
from blb_amd.hostcopy import to_device, to_numpy

SHAPES = [(k, m) for k in (3, 4, 6, 8, 10, 12) for m in (1, 2, 3, 4, 5)]


def _oracle_parity(O, k, m, data):
    sh = [d.copy() for d in data] + [np.zeros(data[0].size, np.uint8) for _ in range(m)]
    O.encode(k, m, sh, use_avx2=True, threads=8)
    return sh[k:]


@pytest.mark.parametrize("k,m", SHAPES)
def test_network_encode_verify_vs_oracle_and_tables(oracle_lib, k, m, knob):
    # 3 whole 16 KiB tiles + a ragged tail: network tiles and table tiles in one launch
    S, B = 3 * 16384 + 4 * 1000 + 12, 3
    rng = np.random.default_rng(1000 * k + m)
    host = rng.integers(0, 256, (B, k + m, S), dtype=np.uint8)
    host[:, k:] = 0xEE
    knob("BLBRS_BITSLICE", 2)
    enc = rs.New(k, m)
    assert enc.compiled_network()["code"]
    st = to_device(host)
    enc.EncodeBatch(st)
    got = to_numpy(st)
    for b in range(B):
        want = _oracle_parity(oracle_lib, k, m, [host[b, i] for i in range(k)])
        for j in range(m):
            assert np.array_equal(got[b, k + j], want[j]), (k, m, b, j)
    assert bool(enc.VerifyBatch(st).all())
    bad = st.clone()
    bad[1, k + m - 1, 5] ^= 0x40           # inside the first (network) tile
    bad[2, k, S - 3] ^= 0x01               # inside the ragged tail (table path)
    assert to_numpy(enc.VerifyBatch(bad)).tolist() == [True, False, False]
    # the table path writes the same bytes and accepts the network's parity
    knob("BLBRS_BITSLICE", 0)
    assert not enc.compiled_network()["code"]
    tab = to_device(host)
    enc.EncodeBatch(tab)
    assert torch.equal(tab, st)
    assert bool(enc.VerifyBatch(st).all())
    assert to_numpy(enc.VerifyBatch(bad)).tolist() == [True, False, False]


@pytest.mark.parametrize("k,m", [(6, 3), (8, 3), (10, 4), (12, 5), (3, 2), (4, 1), (10, 5)])
def test_network_encode_crc_vs_oracle(oracle_lib, k, m, knob):
    """Fused encode + 65532-byte block CRCs: network and table kernels agree with the oracle
    on the parity and on every block CRC (a partial last tile: S % 8 KiB != 0)."""
    S, B = 4 * 65532 + 16 * 37, 2
    rng = np.random.default_rng(77 * k + m)
    host = rng.integers(0, 256, (B, k + m, S), dtype=np.uint8)
    host[:, k:] = 0xEE
    enc = rs.New(k, m)
    outs = {}
    for mode in ("2", "0"):
        knob("BLBRS_BITSLICE", int(mode))
        st = to_device(host)
        crc = to_numpy(enc.EncodeBatchCRC(st, 65532)).view(np.uint32)
        outs[mode] = (to_numpy(st), crc)
    assert np.array_equal(outs["2"][0], outs["0"][0]) and np.array_equal(outs["2"][1], outs["0"][1])
    got, crc = outs["2"]
    for b in range(B):
        want = _oracle_parity(oracle_lib, k, m, [host[b, i] for i in range(k)])
        for j in range(m):
            assert np.array_equal(got[b, k + j], want[j]), (k, m, b, j)
            assert np.array_equal(crc[j, b], oracle_lib.crc32c_blocks(want[j], 65532)), (k, m, b, j)


@pytest.mark.parametrize("k,m", [(6, 3), (8, 3), (12, 5), (3, 2), (10, 4)])
def test_network_pack_encode_vs_tables(k, m, knob):
    """PackTracts + Encode with the network (U = 2 tiles for every k) equals the table kernel
    (U = 1 for k > 6) and Verify accepts the parity; misaligned sources, holes and a ragged
    last tile."""
    S, B = 5 * 8192 + 48, 3
    rng = np.random.default_rng(31 * k + m)
    dpool = torch.randint(0, 256, (1 << 20,), dtype=torch.uint8, device="cuda")
    ext = []
    for p in range(B * k):
        off = int(rng.integers(0, 3)) * 16
        while True:
            ln = int(rng.integers(1, 20000))
            if off + ln > S:
                break
            src = int(rng.integers(0, dpool.numel() - ln))
            ext.append((dpool[src:], off, ln, p))
            off += ln + int(rng.integers(0, 3000))
    enc = rs.New(k, m)
    res = {}
    for mode in ("2", "0"):
        knob("BLBRS_BITSLICE", int(mode))
        st = torch.full((B, k + m, S), 0x5C, dtype=torch.uint8, device="cuda")
        pack.PackEncode(enc, st, ext)
        res[mode] = st
    assert torch.equal(res["2"], res["0"])
    knob("BLBRS_BITSLICE", 1)
    assert bool(enc.VerifyBatch(res["2"]).all())
