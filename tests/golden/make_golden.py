"""Generate tests/golden/*.npz: RS golden vectors for the engine's parity tests.

The reference (blb) holds no RS golden vectors -- its tests only round-trip through the
same library's Verify (internal/tractserver/store_test.go:810-814,875-878) -- and its RS
arithmetic lives in the un-vendored Go module klauspost/reedsolomon@925cb01d6510
(go.mod:20), which cannot be built or run here (no Go toolchain).  The vectors are
therefore produced by TWO independent CPU restatements of that module's algorithm:
  * oracle/rs_oracle.c   (log/exp tables, klauspost's Gauss-Jordan, mulTable + AVX2 paths)
  * oracle/rs_numpy.py   (carry-less multiply, separate inversion)
and written only when both agree byte for byte, and when the matrices match the
survey-derived anchors (RS(4,2) = the Backblaze/klauspost matrix).

Shapes mirror the reference's tests and blb's classes: RS(3,2) lengths 12000/20000 with
erasures {1,3} (store_test.go:750-879), RS(6,3)/(8,3)/(10,3)/(12,5) (StorageClass.go:7-13),
RS(10,4) (BASELINE.json), odd lengths 1/15/17/4099, seed 97531*(stripe+1)
(test_storage_migration.go:27,45).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from oracle import rs_numpy as N  # noqa: E402

ANCHORS = {  # SURVEY.md Appendix A, parity rows
    (4, 2): ["1b1c1214", "1c1b1412"],
    (6, 3): ["070605040302", "060704050203", "a0dfdfb7fee8"],
    (10, 4): ["8196afb8d2c4fee80302", "9681b8afc4d2e8fe0203", "bfd6620a066fdfb70504",
              "d6bf0a626f06b7df0405"],
}

# (k, m, shard lengths, erasure patterns)
CASES = [
    (3, 2, [1, 15, 12000, 20000], [(1, 3), (0,), (3, 4), (0, 1)]),
    (4, 2, [17, 4099], [(0, 5), (2,), (4, 5)]),
    (6, 3, [1, 15, 4099], [(1,), (0, 2, 4), (6, 7, 8), (2, 7)]),
    (8, 3, [4099], [(0,), (3, 9, 10)]),
    (10, 3, [4099], [(1, 7), (10, 11, 12)]),
    (10, 4, [17, 4099], [(1, 7), (2, 11), (0, 1, 2, 3), (10, 11, 12, 13)]),
    (12, 5, [4099], [(0, 3, 6, 9, 12), (1, 2)]),
    (5, 3, [999], [(1, 5, 7)]),   # indexMap example [0,2,3,4,6,1,5,-1]
]


def stripe_data(k: int, S: int, stripe: int) -> np.ndarray:
    rng = np.random.default_rng(97531 * (stripe + 1))
    return rng.integers(0, 256, size=(k, S), dtype=np.uint8)


def main() -> None:
    O.build()
    for (k, m), rows in ANCHORS.items():
        mat = O.build_matrix(k, m)
        got = [bytes(r).hex() for r in mat[k:]]
        assert got == rows, f"anchor mismatch RS({k},{m}): {got}"
    written = 0
    for k, m, lengths, patterns in CASES:
        mat_c = O.build_matrix(k, m)
        mat_n = N.build_matrix(k, m)
        assert np.array_equal(mat_c, mat_n), (k, m)
        assert np.array_equal(mat_c[:k], np.eye(k, dtype=np.uint8)), "not systematic"
        for r in mat_c[k:]:
            x = 0
            for v in r:
                x ^= int(v)
            assert x == 1, "parity row does not XOR to 1"
        out = {"k": np.int32(k), "m": np.int32(m), "matrix": mat_c}
        for si, S in enumerate(lengths):
            data = stripe_data(k, S, si)
            shards = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
            O.encode(k, m, shards)
            shards_avx = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
            O.encode(k, m, shards_avx, use_avx2=True, threads=4)
            par_n = N.encode(k, m, [data[i] for i in range(k)])
            for i in range(m):
                assert np.array_equal(shards[k + i], par_n[i]), (k, m, S, i)
                assert np.array_equal(shards[k + i], shards_avx[k + i]), (k, m, S, i, "avx2")
            out[f"S{si}"] = np.int64(S)
            out[f"data{si}"] = data
            out[f"parity{si}"] = np.stack(shards[k:])
        for pi, pat in enumerate(patterns):
            present = [i not in pat for i in range(k + m)]
            valid_c = [i for i in range(k + m) if present[i]][:k]
            sub = mat_c[valid_c]
            dec_c = O.invert(sub)
            valid_n, dec_n = N.decode_rows(k, m, present)
            assert valid_c == valid_n and np.array_equal(dec_c, dec_n), (k, m, pat)
            out[f"pattern{pi}"] = np.array(pat, dtype=np.int32)
            out[f"decode{pi}"] = dec_c
            out[f"valid{pi}"] = np.array(valid_c, dtype=np.int32)
        path = os.path.join(HERE, f"rs_{k}_{m}.npz")
        np.savez_compressed(path, **out)
        written += 1
        print(f"wrote {os.path.relpath(path, ROOT)}")
    print(f"{written} fixtures; C and numpy restatements agree on every vector")


if __name__ == "__main__":
    main()
