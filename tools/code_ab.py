"""A/B of the coding kernel's launch policy (tools/ect_variants.sh SRCS=rs_kernels builds under
BLBRS_LIB_PATH): EncodeBatch, VerifyBatch and a 1-erasure ReconstructBatch of RS(k,m), B stripes
of 8 MiB, device-resident, mean ms of interleaved reps."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=12)
p.add_argument("--m", type=int, default=5)
p.add_argument("--batch", type=int, default=512)
p.add_argument("--reps", type=int, default=3)
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
dev = torch.device("cuda:0")
st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
enc.EncodeBatch(st)
present = [i != 1 for i in range(k + m)]
ops = {"encode": lambda: enc.EncodeBatch(st), "verify": lambda: enc.VerifyBatch(st),
       "reconstruct_data1": lambda: enc.ReconstructBatch(st, present, data_only=True)}
res = {n: [] for n in ops}
for _ in range(a.reps):
    for n, fn in ops.items():
        fn()
        torch.cuda.synchronize(dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize(dev)
        res[n].append(s.elapsed_time(e))
ok = bool(enc.VerifyBatch(st).all())
print(json.dumps({"k": k, "m": m, "B": B, "ms": {n: round(float(np.mean(v)), 3) for n, v in res.items()},
                  "verify_ok": ok}))
