import json, torch, numpy as np, sys, os
sys.path.insert(0, os.getcwd())
from blb_amd import reedsolomon as rs
dev = torch.device("cuda:0")
k, m, B, S = 6, 3, 1024, 8 << 20
enc = rs.New(k, m)
bufs = []
for i in range(3):
    t = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    t[:, :k].random_(0, 256)
    bufs.append(t)
out = []
for rep in range(3):
    for i, t in enumerate(bufs):
        enc.EncodeBatch(t)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); enc.EncodeBatch(t); e.record(); torch.cuda.synchronize(dev)
        out.append((i, round(s.elapsed_time(e), 3)))
print(json.dumps({"ptrs_GB": [round(b.data_ptr() / 1e9, 1) for b in bufs], "ms": out}))
