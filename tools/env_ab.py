"""A/B of coding-kernel launch knobs read per launch (e.g. BLBRS_BITSLICE=0, gf_bitslice.hpp):
EncodeBatch, VerifyBatch and a 1-erasure ReconstructBatch of RS(k,m), B stripes of 8 MiB,
device-resident, every variant interleaved per rep in one process on the same buffers.
Parity under every variant must equal the first variant's; Verify must pass and the rebuilt
shard must equal the original."""
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
p.add_argument("--ops", default="encode,verify,reconstruct_data1")
p.add_argument("--variants", default="shipped:;tables:BLBRS_BITSLICE=0", help="name:VAR=val+VAR=val;...")
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
variants = []
for item in a.variants.split(";"):
    name, _, env = item.partition(":")
    variants.append((name, dict(kv.split("=", 1) for kv in env.split("+") if kv)))
knobs = {key for _, env in variants for key in env}


def setenv(env):
    rs.use_knobs(env)  # library knobs (blbrs_set_tuning), read by the library once


st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
present = [i != 1 for i in range(k + m)]
checks = {}
ref_par = None
for name, env in variants:
    setenv(env)
    st[:, k:].fill_(0xEE)
    enc.EncodeBatch(st)
    par = st[:, k:].view(torch.int64).sum(dim=-1)
    ref_par = par if ref_par is None else ref_par
    orig = st[:, 1].clone()
    st[:, 1].fill_(0xA5)
    enc.ReconstructBatch(st, present, data_only=True)
    checks[name] = {"parity_same": bool(torch.equal(par, ref_par)), "verify": bool(enc.VerifyBatch(st).all()),
                    "restored": bool(torch.equal(st[:, 1], orig))}
    del orig
ops = {"encode": lambda: enc.EncodeBatch(st), "verify": lambda: enc.VerifyBatch(st),
       "reconstruct_data1": lambda: enc.ReconstructBatch(st, present, data_only=True)}
ops = {n: ops[n] for n in a.ops.split(",")}
res = {f"{op}/{name}": [] for op in ops for name, _ in variants}
for _ in range(a.reps):
    for op, fn in ops.items():
        for name, env in variants:
            setenv(env)
            fn()
            torch.cuda.synchronize(dev)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize(dev)
            res[f"{op}/{name}"].append(round(s.elapsed_time(e), 3))
print(json.dumps({"k": k, "m": m, "B": B, "checks": checks, "ms": res,
                  "min_ms": {n: min(v) for n, v in res.items()}}))
