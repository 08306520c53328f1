"""Published known-answer vectors (tests/golden/published_kat.json) against both oracle
restatements (CPU) and the HIP engine (GPU).

These are fixed expected outputs from the test suites of the libraries blb's path calls:
klauspost/reedsolomon@925cb01d6510 (galois_test.go TestGalois, matrix_test.go
TestMatrixMultiply / TestMatrixInverse[2], reedsolomon_test.go TestOneEncode) and Go's
hash/crc32 golden table (Castagnoli column).  TestOneEncode pins absolute parity bytes of
Encode, which blb's own tests never do (store_test.go:810-814 only round-trips via Verify).
"""
import json
import os

import numpy as np
import pytest

from oracle import rs_numpy as N
from blb_amd.hostcopy import to_device, to_numpy

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "published_kat.json")))
RS = KAT["reedsolomon"]


def test_kat_galois(oracle_lib):
    L = oracle_lib.lib()
    for a, b, want in RS["galMultiply"]["cases"]:
        assert L.rso_gal_mul(a, b) == want
        assert N.gf_mul(a, b) == want
    for a, n, want in RS["galExp"]["cases"]:
        assert L.rso_gal_exp(a, n) == want
        assert N.gf_exp(a, n) == want


def test_kat_matrix(oracle_lib):
    mm = RS["matrixMultiply"]
    got = N.gf_matmul(np.array(mm["a"], np.uint8), np.array(mm["b"], np.uint8))
    assert got.tolist() == mm["want"]
    for case in RS["matrixInverse"]["cases"]:
        m = np.array(case["m"], np.uint8)
        assert oracle_lib.invert(m).tolist() == case["want"]
        assert N.gf_inv_matrix(m).tolist() == case["want"]


def _one_encode():
    e = RS["encode"]
    return e["k"], e["m"], [np.array(d, np.uint8) for d in e["data"]], [np.array(p, np.uint8) for p in e["parity"]]


def test_kat_one_encode_oracle(oracle_lib):
    k, m, data, parity = _one_encode()
    sh = [d.copy() for d in data] + [np.zeros(2, np.uint8) for _ in range(m)]
    oracle_lib.encode(k, m, sh)
    assert [s.tolist() for s in sh[k:]] == [p.tolist() for p in parity]
    sh2 = [d.copy() for d in data] + [np.zeros(2, np.uint8) for _ in range(m)]
    oracle_lib.encode(k, m, sh2, use_avx2=True)
    assert [s.tolist() for s in sh2[k:]] == [p.tolist() for p in parity]
    assert [p.tolist() for p in N.encode(k, m, data)] == [p.tolist() for p in parity]


def test_kat_crc32c_oracle(oracle_lib):
    for s, want in KAT["crc32c"]["cases"]:
        assert oracle_lib.crc32c(s.encode()) == int(want, 16), s
        assert N.crc32c(s.encode()) == int(want, 16), s


gpu = pytest.mark.gpu


@gpu
def test_kat_one_encode_gpu():
    torch = pytest.importorskip("torch")
    from blb_amd import reedsolomon as rs
    k, m, data, parity = _one_encode()
    enc = rs.New(k, m)
    sh = [d.copy() for d in data] + [np.full(2, 0xEE, np.uint8) for _ in range(m)]
    enc.Encode(sh)                                             # host-memory Encoder.Encode
    assert [s.tolist() for s in sh[k:]] == [p.tolist() for p in parity]
    assert enc.Verify(sh)
    # device-resident batch, a multiple of the wave width so full and ragged paths both run
    B = 70
    host = np.full((B, k + m, 2), 0x33, np.uint8)
    host[:, :k] = np.stack(data)
    st = to_device(host)
    enc.EncodeBatch(st)
    got = to_numpy(st)
    for b in range(B):
        assert got[b, k:].tolist() == [p.tolist() for p in parity], b
    # every 5-of-10 erasure pattern that loses data recovers TestOneEncode's data
    full = [d.copy() for d in data] + [p.copy() for p in parity]
    for lost in ([0], [4], [0, 1, 2, 3, 4], [1, 3, 5, 7, 9], [2, 6]):
        shards = [np.empty(0, np.uint8) if i in lost else full[i].copy() for i in range(k + m)]
        enc.Reconstruct(shards)
        assert [s.tolist() for s in shards] == [f.tolist() for f in full], lost


@gpu
def test_kat_crc32c_gpu():
    pytest.importorskip("torch")
    from blb_amd import checksum
    for s, want in KAT["crc32c"]["cases"]:
        if not s:
            continue
        got = checksum.Checksum(np.frombuffer(s.encode(), np.uint8).copy(), 0)
        assert int(got[0]) == int(want, 16), s
