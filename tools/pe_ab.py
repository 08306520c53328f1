"""A/B of PackTracts + Encode: separate (PackPieces then EncodeBatch) vs fused (PackEncode),
RS(k,m) B stripes of 8 MiB with multi-MiB tracts at padToLength offsets (the packer's layout).
Interleaved reps in one process; run one process per library build (BLBRS_LIB_PATH)."""
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
p.add_argument("--variants", default="", help="fused-call env variants name:VAR=val+...;... (read per launch)")
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
pool = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
rng = np.random.default_rng(17)
ext, read_bytes = [], 0
for piece in range(B * k):
    off = 0
    while True:
        ln = int(rng.integers(64 << 10, (8 << 20) + 1))
        if off + ln > S:
            break
        src = int(rng.integers(0, pool.numel() - ln))
        ext.append((pool[src:], off, ln, piece))
        read_bytes += ln
        off += pack.padded_length(ln)
stripes = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
tmp = torch.empty((B, k, S), dtype=torch.uint8, device=dev)  # separate path: packed pieces
enc = rs.New(k, m)


def timed(fn):
    fn()
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(400_000_000)  # host-side extent checks outside the window
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e)


variants = [("fused", {})]
if a.variants:
    variants = []
    for item in a.variants.split(";"):
        name, _, env = item.partition(":")
        variants.append((name, dict(kv.split("=", 1) for kv in env.split("+") if kv)))
knobs = {key for _, env in variants for key in env}


def setenv(env):
    rs.use_knobs(env)  # library knobs (blbrs_set_tuning), read by the library once


res = {n: [] for n, _ in variants}
res.update({"pack": [], "encode": []})
ok = {}
for _ in range(a.reps):
    for n, env in variants:
        setenv(env)
        res[n].append(timed(lambda: pack.PackEncode(enc, stripes, ext)))
        ok[n] = bool(enc.VerifyBatch(stripes).all())
    setenv({})
    res["pack"].append(timed(lambda: pack.PackPieces(tmp.view(B * k, S), S, ext)))
    res["encode"].append(timed(lambda: enc.EncodeBatch(stripes)))
fused = min(min(res[n]) for n, _ in variants)
print(json.dumps({"k": k, "m": m, "B": B, "ms": {x: [round(v, 3) for v in y] for x, y in res.items()},
                  "fused_hbm_GBps": {n: round((read_bytes + B * (k + m) * S) / (min(res[n]) * 1e-3) / 1e9, 1) for n, _ in variants},
                  "bytes_read": read_bytes, "verify_ok": ok}))
