"""A/B of the compiled bit-plane encode network (gf_bitslice.hpp) against the v_perm table
path, in one process: BLBRS_BITSLICE=1 / 0 is read per launch, so the two alternate rep by
rep on the same device buffers.  Per shape: EncodeBatch, VerifyBatch and EncodeBatchCRC on
65532-byte blocks (ms per call, HIP events), B stripes of 8 MiB."""
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
p.add_argument("--shapes", default="6,3,1024;8,3,512;10,4,512;12,5,512")
p.add_argument("--reps", type=int, default=3)
p.add_argument("--iters", type=int, default=5)
p.add_argument("--ops", default="encode,verify,encode_crc")
# name:VAR=v+VAR2=w;... -- library knobs of each variant (rs.use_knobs / blbrs_set_tuning)
p.add_argument("--variants", default="net:BLBRS_BITSLICE=2;perm:BLBRS_BITSLICE=0;policy:BLBRS_BITSLICE=1")
a = p.parse_args()
dev = torch.device("cuda:0")
S = 8 << 20


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


for spec in a.shapes.split(";"):
    k, m, B = (int(v) for v in spec.split(","))
    stripes = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device=dev)
    enc = rs.New(k, m)
    ext = []
    if "pack_encode" in a.ops:
        # tracts of 64 KiB..8 MiB from a 4 GiB pool at padToLength-aligned piece offsets (bench.py)
        pool = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
        prng = np.random.default_rng(17)
        for piece in range(B * k):
            off = 0
            while True:
                ln = int(prng.integers(64 << 10, (8 << 20) + 1))
                if off + ln > S:
                    break
                ext.append((pool[int(prng.integers(0, pool.numel() - ln)):], off, ln, piece))
                off += pack.padded_length(ln)

    def pack_encode_ms():
        pack.PackEncode(enc, stripes, ext)
        torch.cuda.synchronize(dev)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(400_000_000)  # host-side extent checks outside the window
        s0.record()
        pack.PackEncode(enc, stripes, ext)
        s1.record()
        torch.cuda.synchronize(dev)
        return s0.elapsed_time(s1)

    ops = {"pack_encode": pack_encode_ms,
           "encode": lambda: enc.EncodeBatch(stripes),
           "verify": lambda: enc.VerifyBatch(stripes),
           "encode_crc": lambda: enc.EncodeBatchCRC(stripes, 65532)}
    variants = []
    for v in a.variants.split(";"):
        vname, _, envs = v.partition(":")
        variants.append((vname, dict(kv.split("=", 1) for kv in envs.split("+") if kv)))
    res = {}
    for rep in range(a.reps):
        for vname, env in variants:
            rs.use_knobs(env)
            for name in a.ops.split(","):
                ms = ops[name]() if name == "pack_encode" else timed(ops[name])
                res.setdefault(f"{name}_{vname}", []).append(round(ms, 3))
            rs.use_knobs({})
    # the two paths write the same parity
    enc.EncodeBatch(stripes)
    ok = bool(enc.VerifyBatch(stripes).all())
    rs.use_knobs({"BLBRS_BITSLICE": 0})
    ok_perm = bool(enc.VerifyBatch(stripes).all())
    rs.use_knobs({})
    gb = B * (k + m) * S / 1e9
    best = {key: min(v) for key, v in res.items()}
    print(json.dumps({"k": k, "m": m, "B": B, "GB": round(gb, 2), "verify_ok": [ok, ok_perm],
                      "compiled": enc.compiled_network(), "ms": res,
                      "TBps_best": {key: round(gb / v, 3) for key, v in best.items()}}), flush=True)
    del stripes, ext
    pool = None
    torch.cuda.empty_cache()
