"""Does a device sync between launches change a launch's time?  pmc_prod.py syncs after every
launch (one dispatch at a time under the counters), bench.py records events around launches
issued back to back.  RS(6,3) B=1024: encode and verify, per-launch HIP-event times, both ways,
interleaved, in one process.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

k, m, B, S = 6, 3, 1024, 8 << 20
st = torch.empty((B, k + m, S), dtype=torch.uint8, device="cuda")
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
enc.EncodeBatch(st)
ops = {"encode": lambda: enc.EncodeBatch(st), "verify": lambda: enc.VerifyBatch(st)}
res = {}
for rnd in range(3):
    for name, fn in ops.items():
        for mode in ("back_to_back", "sync_each"):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
            for s, e in evs:
                s.record()
                fn()
                e.record()
                if mode == "sync_each":
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            res.setdefault(f"{name}_{mode}", []).extend(round(s.elapsed_time(e), 3) for s, e in evs)
print(json.dumps({"median": {kk: sorted(v)[len(v) // 2] for kk, v in res.items()}, "ms": res}), flush=True)
