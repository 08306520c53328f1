"""Shard-stride padding A/B for the coding kernel: RS(k,m) encode / 1-erasure reconstruct of
B stripes of 8 MiB in a [B, k+m, S + pad] buffer (shard stride S + pad), device-resident.
One process per run; run several processes per pad (the physical placement differs per
process)."""
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
p.add_argument("--pad", type=int, default=0)
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
buf = torch.empty((B, k + m, S + a.pad), dtype=torch.uint8, device=dev)
st = buf[:, :, :S]
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
enc.EncodeBatch(st)
present = [i != 1 for i in range(k + m)]
res = {"encode": [], "reconstruct_data1": []}
for _ in range(a.reps):
    for n, fn in (("encode", lambda: enc.EncodeBatch(st)),
                  ("reconstruct_data1", lambda: enc.ReconstructBatch(st, present, data_only=True))):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize(dev)
        res[n].append(s.elapsed_time(e))
print(json.dumps({"pad": a.pad, "base_mod_2M": buf.data_ptr() % (2 << 20),
                  "ms": {n: round(float(np.median(v)), 3) for n, v in res.items()}}))
