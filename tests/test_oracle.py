"""CPU tests of the oracle (test infrastructure) against the committed golden vectors,
the Appendix A anchors and the algebraic properties klauspost's construction guarantees.

Parity bytes are pinned by two independent restatements (C + numpy), not by reference
output: the reference's own RS tests only round-trip through Verify
(internal/tractserver/store_test.go:810-814,875-878) and its RS library is un-vendored Go.
"""
import itertools

import numpy as np
import pytest

from oracle import rs_numpy as N


def test_anchor_rs42_backblaze(oracle_lib):
    # klauspost ported Backblaze JavaReedSolomon; its 4+2 parity rows are well known.
    mat = oracle_lib.build_matrix(4, 2)
    assert bytes(mat[4]).hex() == "1b1c1214"
    assert bytes(mat[5]).hex() == "1c1b1412"


def test_gf_field_laws(oracle_lib):
    L = oracle_lib.lib()
    for a in range(256):
        assert L.rso_gal_mul(a, 1) == a
        assert L.rso_gal_mul(a, 0) == 0
        assert L.rso_gal_mul(a, 2) == N.gf_mul(a, 2)
    rng = np.random.default_rng(1)
    for a, b in rng.integers(0, 256, size=(500, 2)):
        assert L.rso_gal_mul(int(a), int(b)) == N.gf_mul(int(a), int(b))
    # galExp edge cases (galois.go): n==0 -> 1 even for a==0; a==0 -> 0
    assert L.rso_gal_exp(0, 0) == 1 and L.rso_gal_exp(0, 3) == 0
    assert L.rso_gal_exp(2, 8) == 0x1D  # x^8 = x^4+x^3+x^2+1 under 0x11D


@pytest.mark.parametrize("k,m", [(1, 1), (3, 2), (4, 2), (6, 3), (8, 3), (10, 3), (10, 4), (12, 5),
                                 (17, 3), (30, 10)])
def test_matrix_systematic_and_mds(oracle_lib, k, m):
    mat = oracle_lib.build_matrix(k, m)
    assert np.array_equal(mat, N.build_matrix(k, m))
    assert np.array_equal(mat[:k], np.eye(k, dtype=np.uint8))
    for row in mat[k:]:
        assert np.bitwise_xor.reduce(row) == 1  # Lagrange-basis rows sum to 1
    # MDS: every k-row submatrix invertible (exhaustive for small shapes)
    from math import comb
    if comb(k + m, k) <= 400:
        combos = list(itertools.combinations(range(k + m), k))
    else:
        rng = np.random.default_rng(k * 1000 + m)
        combos = [sorted(rng.choice(k + m, k, replace=False).tolist()) for _ in range(400)]
    for rows in combos:
        oracle_lib.invert(mat[list(rows)])


def test_new_errors(oracle_lib):
    with pytest.raises(oracle_lib.OracleError) as e:
        oracle_lib.build_matrix(0, 2)
    assert e.value.name == "ErrInvShardNum"
    with pytest.raises(oracle_lib.OracleError) as e:
        oracle_lib.build_matrix(3, 0)
    assert e.value.name == "ErrInvShardNum"
    with pytest.raises(oracle_lib.OracleError) as e:
        oracle_lib.build_matrix(200, 57)
    assert e.value.name == "ErrMaxShardNum"
    oracle_lib.build_matrix(200, 56)  # k+m == 256 allowed


def test_golden_encode(oracle_lib, golden):
    for (k, m), g in golden.items():
        assert np.array_equal(oracle_lib.build_matrix(k, m), g["matrix"])
        i = 0
        while f"S{i}" in g:
            data, parity = g[f"data{i}"], g[f"parity{i}"]
            for avx2, threads in [(False, 1), (True, 1), (True, 4)]:
                shards = [data[j].copy() for j in range(k)] + [np.full(data.shape[1], 0xEE, np.uint8)
                                                               for _ in range(m)]
                oracle_lib.encode(k, m, shards, use_avx2=avx2, threads=threads)
                for j in range(m):
                    assert np.array_equal(shards[k + j], parity[j]), (k, m, i, j, avx2)
            assert oracle_lib.verify(k, m, [data[j] for j in range(k)] + [parity[j] for j in range(m)])
            i += 1


def test_golden_reconstruct(oracle_lib, golden):
    for (k, m), g in golden.items():
        shards_full = [g["data0"][j] for j in range(k)] + [g["parity0"][j] for j in range(m)]
        p = 0
        while f"pattern{p}" in g:
            pat = list(g[f"pattern{p}"])
            present = [i not in pat for i in range(k + m)]
            valid = [i for i in range(k + m) if present[i]][:k]
            assert valid == list(g[f"valid{p}"])
            mat = g["matrix"]
            assert np.array_equal(oracle_lib.invert(mat[valid]), g[f"decode{p}"])
            for data_only in (False, True):
                sh = [None if i in pat else shards_full[i].copy() for i in range(k + m)]
                out = oracle_lib.reconstruct(k, m, sh, data_only)
                for i in range(k + m):
                    if i < k or not data_only:
                        assert np.array_equal(out[i], shards_full[i]), (k, m, pat, i, data_only)
                    elif i in pat:
                        assert out[i] is None
            p += 1


def test_reconstruct_semantics(oracle_lib):
    k, m, S = 3, 2, 100
    rng = np.random.default_rng(5)
    sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8)] * 0
    sh += [np.zeros(S, np.uint8) for _ in range(m)]
    oracle_lib.encode(k, m, sh)
    # all present: nothing to do
    out = oracle_lib.reconstruct(k, m, [s.copy() for s in sh], False)
    assert all(np.array_equal(a, b) for a, b in zip(out, sh))
    # too few
    with pytest.raises(oracle_lib.OracleError) as e:
        oracle_lib.reconstruct(k, m, [sh[0], None, None, sh[3], None], False)
    assert e.value.name == "ErrTooFewShards"
    # size mismatch
    with pytest.raises(oracle_lib.OracleError) as e:
        oracle_lib.reconstruct(k, m, [sh[0], sh[1][:50], None, sh[3], sh[4]], False)
    assert e.value.name == "ErrShardSize"
    # no data
    with pytest.raises(oracle_lib.OracleError) as e:
        oracle_lib.reconstruct(k, m, [None] * 5, False)
    assert e.value.name == "ErrShardNoData"


def test_numpy_restatement_roundtrip():
    k, m, S = 6, 3, 64
    rng = np.random.default_rng(2)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    par = N.encode(k, m, data)
    full = data + par
    assert N.verify(k, m, full)
    sh = list(full)
    sh[1] = None
    sh[7] = None
    out = N.reconstruct(k, m, sh, data_only=False)
    assert all(np.array_equal(a, b) for a, b in zip(out, full))
