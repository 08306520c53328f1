"""A/B of the PackTracts kernel variants (BLBRS_PACK_VARIANT, read per launch; pack.hip):
bench.py's pack_tracts workload -- k columns of B 8 MiB pieces filled with tracts of random
length (64 KiB..8 MiB) from a 4 GiB device pool at padToLength offsets -- timed per variant,
interleaved in one process on the same buffers.  Every variant's pieces must equal
variant 0's byte for byte (the GPU tests pin variant outputs to the oracle)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import pack  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=6)
p.add_argument("--m", type=int, default=3)
p.add_argument("--batch", type=int, default=1024)
p.add_argument("--reps", type=int, default=3)
p.add_argument("--variants", default="0,6,8,10")
p.add_argument("--distinct", action="store_true",
               help="every tract its own source bytes (a pool as large as all tracts, in shuffled order)")
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
variants = [int(v) for v in a.variants.split(",")]
stripes = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
rng = np.random.default_rng(17)
lens = []  # per column: [(piece, offset, length)]
for j in range(k):
    col = []
    for b in range(B):
        off = 0
        while True:
            ln = int(rng.integers(64 << 10, (8 << 20) + 1))
            if off + ln > S:
                break
            col.append((b, off, ln))
            off += pack.padded_length(ln)
    lens.append(col)
read_bytes = sum(ln for col in lens for _, _, ln in col)
if a.distinct:  # sources laid end to end in a shuffled order, 256-byte aligned starts + a skew
    pool = torch.empty(read_bytes + 256 * sum(len(c) for c in lens) + 4096, dtype=torch.uint8, device=dev)
    pool.random_(0, 256)
    order = rng.permutation(sum(len(c) for c in lens))
    flat = [(j, i) for j, col in enumerate(lens) for i in range(len(col))]
    starts, pos = {}, 0
    for o in order:
        j, i = flat[o]
        starts[(j, i)] = pos + int(rng.integers(0, 16))
        pos += (lens[j][i][2] + 16 + 255) // 256 * 256
    per_col = [[(pool[starts[(j, i)]:], off, ln, b) for i, (b, off, ln) in enumerate(col)] for j, col in enumerate(lens)]
else:  # bench.py's layout: random offsets into a 4 GiB pool (sources overlap)
    pool = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
    per_col = []
    for col in lens:
        per_col.append([(pool[int(rng.integers(0, pool.numel() - ln)):], off, ln, b) for b, off, ln in col])
cols = [stripes[:, j, :] for j in range(k)]
nbytes = read_bytes + B * k * S


def run():
    for j in range(k):
        pack.PackPieces(cols[j], S, per_col[j])


def timed(v):
    rs.set_tuning("BLBRS_PACK_VARIANT", v)
    run()
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(400_000_000)  # host-side extent checks outside the window
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    run()
    e.record()
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e)


# Bit-exactness across variants: checksum every piece after each variant's pass.
sums = {}
for v in variants:
    stripes[:, :k].fill_(0xA5)
    rs.set_tuning("BLBRS_PACK_VARIANT", v)
    run()
    torch.cuda.synchronize(dev)
    sums[v] = stripes[:, :k].view(torch.int64).sum(dim=-1).cpu()
same = {v: bool(torch.equal(sums[v], sums[variants[0]])) for v in variants}
res = {v: [] for v in variants}
for _ in range(a.reps):
    for v in variants:
        res[v].append(timed(v))
print(json.dumps({"k": k, "B": B, "distinct": a.distinct, "bytes_read": read_bytes, "bytes_written": B * k * S,
                  "tracts": sum(len(e) for e in per_col), "same_as_first": same,
                  "ms": {v: [round(x, 3) for x in y] for v, y in res.items()},
                  "best_GBps": {v: round(nbytes / (min(y) * 1e-3) / 1e9, 1) for v, y in res.items()}}))
