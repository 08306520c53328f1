"""Independent numpy restatement of klauspost/reedsolomon @925cb01d6510 (go.mod:20).

TEST INFRASTRUCTURE ONLY -- the second, independent CPU restatement used to cross-check
oracle/rs_oracle.c.  It deliberately shares no code and no table
construction with the C oracle: field products come from a carry-less
shift-and-reduce multiply (polynomial 0x11D), not from log/exp tables, and matrix
inversion is a separate Gauss-Jordan over those products.

Follows (algorithm of the pinned module):
  galois.go    galMultiply / galExp           -> gf_mul, gf_exp
  matrix.go    vandermonde / Invert / Multiply -> vandermonde, gf_inv_matrix, gf_matmul
  reedsolomon.go buildMatrix / Encode / reconstruct / Verify -> build_matrix, encode, ...
Caller semantics: internal/tractserver/store.go:1014-1142, client/blb/reconstruct.go:65-195.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D


def gf_mul(a: int, b: int) -> int:
    """Carry-less multiply reduced by x^8+x^4+x^3+x^2+1 (galois.go, 'generating polynomial 29')."""
    r = 0
    a &= 0xFF
    b &= 0xFF
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= POLY
    return r


def _build_mul_table() -> np.ndarray:
    t = np.zeros((256, 256), dtype=np.uint8)
    for a in range(256):
        for b in range(256):
            t[a, b] = gf_mul(a, b)
    return t


MUL = _build_mul_table()


def gf_pow(a: int, n: int) -> int:
    r = 1
    for _ in range(n):
        r = gf_mul(r, a)
    return r


def gf_exp(a: int, n: int) -> int:
    """galois.go galExp: 1 if n == 0, 0 if a == 0, else a**n in the field."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return gf_pow(a, n)


def gf_inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError("gf_inv(0)")
    for b in range(1, 256):
        if gf_mul(a, b) == 1:
            return b
    raise AssertionError("no inverse")


def vandermonde(rows: int, cols: int) -> np.ndarray:
    """matrix.go vandermonde: V[r][c] = galExp(byte(r), c)."""
    v = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        for c in range(cols):
            v[r, c] = gf_exp(r & 0xFF, c)
    return v


def gf_matmul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], b.shape[1]), dtype=np.uint8)
    for i in range(a.shape[0]):
        acc = np.zeros(b.shape[1], dtype=np.uint8)
        for j in range(a.shape[1]):
            acc ^= MUL[a[i, j]][b[j]]
        out[i] = acc
    return out


class SingularMatrix(Exception):
    pass


def gf_inv_matrix(m: np.ndarray) -> np.ndarray:
    """Gauss-Jordan inverse (any pivoting gives the same unique inverse)."""
    n = m.shape[0]
    a = np.concatenate([m.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for col in range(n):
        piv = next((r for r in range(col, n) if a[r, col]), None)
        if piv is None:
            raise SingularMatrix()
        if piv != col:
            a[[col, piv]] = a[[piv, col]]
        a[col] = MUL[gf_inv(int(a[col, col]))][a[col]]
        for r in range(n):
            if r != col and a[r, col]:
                a[r] ^= MUL[a[r, col]][a[col]]
    return a[:, n:].copy()


def build_matrix(k: int, m: int) -> np.ndarray:
    """reedsolomon.go New() checks + buildMatrix: M = V * inv(V[0:k])."""
    if k <= 0 or m <= 0:
        raise ValueError("ErrInvShardNum")
    if k + m > 256:
        raise ValueError("ErrMaxShardNum")
    v = vandermonde(k + m, k)
    return gf_matmul(v, gf_inv_matrix(v[:k]))


def code(rows: np.ndarray, inputs: list[np.ndarray]) -> list[np.ndarray]:
    """codeSomeShards: out_r = XOR_c rows[r][c] * inputs[c] (byte-wise)."""
    outs = []
    for r in range(rows.shape[0]):
        acc = np.zeros_like(inputs[0])
        for c, x in enumerate(inputs):
            acc ^= MUL[rows[r, c]][x]
        outs.append(acc)
    return outs


def encode(k: int, m: int, data: list[np.ndarray]) -> list[np.ndarray]:
    mat = build_matrix(k, m)
    return code(mat[k:], data)


def decode_rows(k: int, m: int, present: list[bool]) -> tuple[list[int], np.ndarray]:
    """reedsolomon.go reconstruct: valid = first k present indices ascending;
    returns (valid, inv(M[valid]))."""
    mat = build_matrix(k, m)
    valid = [i for i, p in enumerate(present) if p][:k]
    return valid, gf_inv_matrix(mat[valid])


def reconstruct(k: int, m: int, shards: list[np.ndarray | None], data_only: bool) -> list[np.ndarray]:
    """Encoder.Reconstruct / ReconstructData; missing = None or empty.  Returns a new list."""
    n = k + m
    shards = [None if (s is None or len(s) == 0) else s for s in shards]
    present = [s is not None for s in shards]
    if all(present):
        return list(shards)
    if sum(present) < k:
        raise ValueError("ErrTooFewShards")
    valid, dec = decode_rows(k, m, present)
    sub = [shards[i] for i in valid]
    out = list(shards)
    for i in range(k):
        if out[i] is None:
            out[i] = code(dec[i:i + 1], sub)[0]
    if not data_only:
        mat = build_matrix(k, m)
        for i in range(k, n):
            if out[i] is None:
                out[i] = code(mat[i:i + 1], out[:k])[0]
    return out


def verify(k: int, m: int, shards: list[np.ndarray]) -> bool:
    par = encode(k, m, shards[:k])
    return all(np.array_equal(p, s) for p, s in zip(par, shards[k:]))


def crc32c(data: bytes, crc: int = 0) -> int:
    """Bitwise CRC-32C (reflected polynomial 0x82F63B78), independent of the C table."""
    crc = ~crc & 0xFFFFFFFF
    for b in bytes(data):
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return ~crc & 0xFFFFFFFF


def pack_piece(length: int, srcs: list[tuple[bytes, int]]) -> bytes:
    """The packed chunk file Store.PackTracts leaves (internal/tractserver/store.go:922-994):
    each (tract bytes, Offset) written at its offset (t.write, :957), zero holes (a fresh
    sparse file reads 0), then zeros up to `length` when there are sources (:974-980).
    With no sources the file stays empty."""
    if not srcs:
        return b""
    out = bytearray(max(length, max(off + len(b) for b, off in srcs)))
    for b, off in srcs:
        out[off:off + len(b)] = b
    return bytes(out)
