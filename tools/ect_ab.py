"""A/B of the fused encode+CRC kernels on the BASELINE batch (RS(6,3) or --k/--m, B stripes
of 8 MiB, device-resident): plain encode, tile-grid kernel, persistent segment kernel, each
on 65532-byte blocks and whole-shard frames.  Interleaved reps in one process; run under
rocprofv3 --kernel-trace --stats for the per-kernel split (main kernel vs combine)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=6)
p.add_argument("--m", type=int, default=3)
p.add_argument("--batch", type=int, default=1024)
p.add_argument("--reps", type=int, default=2)
p.add_argument("--iters", type=int, default=5)
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
stripes = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device=dev)
enc = rs.New(k, m)
variants = [("tile", {}), ("persistent", {"BLBRS_EC_PERSISTENT": "1"})]


def timed(fn):
    fn()
    torch.cuda.synchronize(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e) / a.iters


res = {}
for rep in range(a.reps):
    res.setdefault("encode", []).append(timed(lambda: enc.EncodeBatch(stripes)))
    for name, env in variants:
        for blk_name, blk in (("b65532", 65532), ("whole", 0)):
            rs.use_knobs(env)
            try:
                ms = timed(lambda: enc.EncodeBatchCRC(stripes, blk))
            finally:
                rs.use_knobs({})
            res.setdefault(f"{name}_{blk_name}", []).append(ms)
    # file-aligned window (rsEncodeOne's parity window at 4 MiB: phase 256) with seeds
    seeds = torch.zeros((m, B), dtype=torch.int32, device=dev)
    res.setdefault("tile_b65532_phase256_seeded", []).append(
        timed(lambda: enc.EncodeBatchCRC(stripes, 65532, phase=256, seeds=seeds)))
out = {key: [round(v, 3) for v in vals] for key, vals in res.items()}
print(json.dumps({"k": k, "m": m, "B": B, "ms": out}))
