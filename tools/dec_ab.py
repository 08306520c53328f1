"""A/B of the single-erasure ReconstructData launch (BASELINE config 3: RS(6,3), B=1024 x
8 MiB, data shard 1 missing): env variants read per launch (the BLBRS_DEC_U knob of the A/B build
behind profiles/r03/dec/ is not kept),
interleaved reps in one process on the same buffers; the rebuilt shard must equal the original
under every variant."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=6)
p.add_argument("--m", type=int, default=3)
p.add_argument("--batch", type=int, default=1024)
p.add_argument("--reps", type=int, default=5)
p.add_argument("--variants", default="shipped:",
               help="name:VAR=val+VAR=val;... (empty = defaults)")
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
variants = []
for item in a.variants.split(";"):
    name, _, env = item.partition(":")
    variants.append((name, dict(kv.split("=", 1) for kv in env.split("+") if kv)))
knobs = {key for _, env in variants for key in env}
st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
enc.EncodeBatch(st)
ref = st[:, 1].clone()
present = [i != 1 for i in range(k + m)]


def setenv(env):
    rs.use_knobs(env)  # library knobs (blbrs_set_tuning), read by the library once


ok, res = {}, {n: [] for n, _ in variants}
for name, env in variants:
    setenv(env)
    st[:, 1].fill_(0xA5)
    enc.ReconstructBatch(st, present, data_only=True)
    ok[name] = bool(torch.equal(st[:, 1], ref))
for _ in range(a.reps):
    for name, env in variants:
        setenv(env)
        enc.ReconstructBatch(st, present, data_only=True)
        torch.cuda.synchronize(dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        enc.ReconstructBatch(st, present, data_only=True)
        e.record()
        torch.cuda.synchronize(dev)
        res[name].append(s.elapsed_time(e))
nbytes = B * (k + 1) * S
print(json.dumps({"k": k, "m": m, "B": B, "restored": ok, "ms": {n: [round(x, 3) for x in v] for n, v in res.items()},
                  "best_GBps": {n: round(nbytes / (min(v) * 1e-3) / 1e9, 1) for n, v in res.items()}}))
