"""ctypes front-end for the C restatement oracle/rs_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  The product package blb_amd/ never imports this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "librs_oracle.so")

ERRORS = {
    -1: "ErrInvShardNum",
    -2: "ErrMaxShardNum",
    -3: "ErrTooFewShards",
    -4: "ErrShardNoData",
    -5: "ErrShardSize",
    -6: "errSingular",
    -7: "alloc",
}


class OracleError(Exception):
    def __init__(self, code: int):
        super().__init__(ERRORS.get(code, f"rc={code}"))
        self.code = code
        self.name = ERRORS.get(code, f"rc={code}")


def build() -> str:
    """Compile the oracle with gcc (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.rso_build_matrix.argtypes = [ctypes.c_int, ctypes.c_int, P]
        L.rso_invert.argtypes = [ctypes.c_int, P, P]
        L.rso_gal_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.rso_gal_mul.restype = ctypes.c_uint8
        L.rso_gal_exp.argtypes = [ctypes.c_uint8, ctypes.c_int]
        L.rso_gal_exp.restype = ctypes.c_uint8
        L.rso_code.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_size_t,
                               ctypes.c_int, ctypes.c_int]
        L.rso_code.restype = None
        L.rso_encode.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int, ctypes.c_int]
        L.rso_verify.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P]
        L.rso_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int]
        L.rso_crc32c_update.argtypes = [ctypes.c_uint32, P, ctypes.c_size_t]
        L.rso_crc32c_update.restype = ctypes.c_uint32
        L.rso_crc32c_blocks.argtypes = [P, ctypes.c_size_t, ctypes.c_size_t, P]
        L.rso_crc32c_blocks.restype = None
        L.rso_crc32c_blocks_hw.argtypes = [P, ctypes.c_size_t, ctypes.c_size_t, P, ctypes.c_int]
        L.rso_crc32c_blocks_hw.restype = None
        L.rso_have_sse42.restype = ctypes.c_int
        L.rso_have_avx2.restype = ctypes.c_int
        L.rso_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[None if a is None else a.ctypes.data for a in arrs])


def _lens(arrs):
    return (ctypes.c_size_t * len(arrs))(*[0 if a is None else a.size for a in arrs])


def _check(rc: int):
    if rc != 0:
        raise OracleError(rc)


def build_matrix(k: int, m: int) -> np.ndarray:
    out = np.zeros((k + m) * k if 0 < k and 0 < m and k + m <= 256 else 1, dtype=np.uint8)
    _check(lib().rso_build_matrix(k, m, out.ctypes.data))
    return out.reshape(k + m, k)


def invert(mat: np.ndarray) -> np.ndarray:
    mat = np.ascontiguousarray(mat, dtype=np.uint8)
    out = np.zeros_like(mat)
    _check(lib().rso_invert(mat.shape[0], mat.ctypes.data, out.ctypes.data))
    return out


def code(rows: np.ndarray, inputs, outputs, use_avx2=False, threads=1):
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n = inputs[0].size
    lib().rso_code(rows.ctypes.data, rows.shape[1], rows.shape[0], _ptrs(inputs), _ptrs(outputs),
                   n, int(use_avx2), int(threads))


def encode(k: int, m: int, shards, use_avx2=False, threads=1):
    """Encoder.Encode on a list of k+m contiguous uint8 arrays (parity overwritten)."""
    _check(lib().rso_encode(k, m, _ptrs(shards), _lens(shards), int(use_avx2), int(threads)))


def verify(k: int, m: int, shards) -> bool:
    ok = ctypes.c_int(0)
    _check(lib().rso_verify(k, m, _ptrs(shards), _lens(shards), ctypes.byref(ok)))
    return bool(ok.value)


def reconstruct(k: int, m: int, shards, data_only: bool):
    """Encoder.Reconstruct[Data].  Missing entries: None or empty arrays.  Returns a new list
    with produced shards filled in (klauspost allocates when cap < size)."""
    n = k + m
    lens = [0 if s is None else s.size for s in shards]
    size = next((x for x in lens if x), 0)
    bufs = list(shards)
    for i in range(n):
        if lens[i] == 0 and size and (i < k or not data_only):
            bufs[i] = np.zeros(size, dtype=np.uint8)
    ptrs = (ctypes.c_void_p * n)(*[None if b is None or b.size == 0 else b.ctypes.data for b in bufs])
    L = (ctypes.c_size_t * n)(*lens)
    _check(lib().rso_reconstruct(k, m, ptrs, L, int(data_only)))
    return [bufs[i] if L[i] else (None if shards[i] is None or shards[i].size == 0 else shards[i])
            for i in range(n)]


def crc32c(data, crc: int = 0) -> int:
    """crc32.Update(crc, castagnoliTable, data) (Checksum when crc == 0)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                             dtype=np.uint8)
    return int(lib().rso_crc32c_update(crc, a.ctypes.data, a.size))


def crc32c_blocks(data: np.ndarray, block: int) -> np.ndarray:
    a = np.ascontiguousarray(data, dtype=np.uint8)
    nb = (a.size + block - 1) // block
    out = np.zeros(max(nb, 1), np.uint32)
    lib().rso_crc32c_blocks(a.ctypes.data, a.size, block, out.ctypes.data)
    return out[:nb]


def crc32c_blocks_hw(data: np.ndarray, block: int, threads: int = 1) -> np.ndarray:
    """Go's amd64 CRC-32C algorithm class (SSE4.2, three interleaved streams) over OpenMP
    threads: bench.py's CPU baseline for the CRC row.  Same output as crc32c_blocks."""
    a = np.ascontiguousarray(data, dtype=np.uint8)
    nb = (a.size + block - 1) // block
    out = np.zeros(max(nb, 1), np.uint32)
    lib().rso_crc32c_blocks_hw(a.ctypes.data, a.size, block, out.ctypes.data, int(threads))
    return out[:nb]
