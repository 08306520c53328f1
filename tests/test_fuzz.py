"""Seeded random sweep over the engine's entry points against the oracle (bit-exact).

Each case draws a shape (k data + m parity shards, k outside the compiled instantiations
and m above five included, so the runtime-k and wide-row kernels run too), a shard length
(ragged, unaligned to 16), a buffer kind (pageable, pinned or device) and an operation:
Encode / Verify with one corrupted byte / Reconstruct / ReconstructData with up to m
erasures, including parity-only and mixed patterns.  Outputs start as stale bytes.  The
expected bytes come from the C oracle (encode) or are the original shards (reconstruct);
klauspost's decode rule (first k present shards) only changes which survivors are read, so
identity with the original is the bar.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from blb_amd import reedsolomon as rs  # noqa: E402
from blb_amd.hostcopy import to_device, to_numpy

CASES = 160


def _draw(rng):
    k = int(rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 16, 17, 20, 24, 40]))
    m = int(rng.integers(1, 11 if k < 40 else 21))
    S = int(rng.choice([1, 15, 16, 17, 4095, 4096, 4097, 65532, 65536 + 3, int(rng.integers(1, 300_000))]))
    kind = str(rng.choice(["pageable", "pinned", "device"]))
    op = str(rng.choice(["encode", "verify", "reconstruct", "reconstruct_data"]))
    return k, m, S, kind, op


def _oracle_stripe(O, rng, k, m, S):
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    sh = [d.copy() for d in data] + [np.zeros(S, np.uint8) for _ in range(m)]
    O.encode(k, m, sh, use_avx2=True, threads=8)
    return sh


def test_random_sweep_vs_oracle(oracle_lib):
    rng = np.random.default_rng(20261017)
    dev = torch.device("cuda:0")
    seen = set()
    for case in range(CASES):
        k, m, S, kind, op = _draw(rng)
        seen.add((kind, op))
        n = k + m
        full = _oracle_stripe(oracle_lib, rng, k, m, S)
        enc = rs.New(k, m)
        tag = (case, k, m, S, kind, op)
        if kind == "device":
            B = int(rng.integers(1, 4))
            st = to_device(np.stack([np.stack(full)] * B), dev)
            if op == "encode":
                st[:, k:] = 0xEE
                enc.EncodeBatch(st)
                assert np.array_equal(to_numpy(st), np.stack([np.stack(full)] * B)), tag
            elif op == "verify":
                bad = int(rng.integers(0, B))
                shard, pos = int(rng.integers(0, n)), int(rng.integers(0, S))
                st[bad, shard, pos] ^= 0x01
                ok = to_numpy(enc.VerifyBatch(st))
                assert not ok[bad] and ok.sum() == B - 1, tag
            else:
                e = int(rng.integers(1, m + 1))
                lost = sorted(int(x) for x in rng.choice(n, e, replace=False))
                want = st.clone()
                st[:, lost] = 0xC3
                data_only = op == "reconstruct_data"
                enc.ReconstructBatch(st, [i not in lost for i in range(n)], data_only=data_only)
                for i in range(n):
                    if i in lost and data_only and i >= k:
                        assert bool((st[:, i] == 0xC3).all()), tag + (i,)
                    else:
                        assert torch.equal(st[:, i], want[:, i]), tag + (i,)
            continue
        mk = (lambda a: torch.from_numpy(a.copy()).pin_memory().numpy()) if kind == "pinned" else (lambda a: a.copy())
        if op == "encode":
            sh = [mk(full[i]) for i in range(k)] + [mk(np.full(S, 0xEE, np.uint8)) for _ in range(m)]
            enc.Encode(sh)
            for i in range(n):
                assert np.array_equal(sh[i], full[i]), tag + (i,)
        elif op == "verify":
            sh = [mk(x) for x in full]
            assert enc.Verify(sh), tag
            shard, pos = int(rng.integers(0, n)), int(rng.integers(0, S))
            sh[shard][pos] ^= 0x80
            assert not enc.Verify(sh), tag
        else:
            e = int(rng.integers(1, m + 1))
            lost = set(int(x) for x in rng.choice(n, e, replace=False))
            sh = [None if i in lost else mk(full[i]) for i in range(n)]
            data_only = op == "reconstruct_data"
            (enc.ReconstructData if data_only else enc.Reconstruct)(sh)
            for i in range(n):
                if i in lost and data_only and i >= k:
                    assert sh[i] is None, tag + (i,)
                else:
                    assert np.array_equal(sh[i], full[i]), tag + (i,)
    assert len(seen) >= 8, seen
