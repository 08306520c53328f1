"""Exit with a default-knob background compile in flight (round 6: BLBRS_RTC = 1 is the default).

One RS(12,5) recovery-RPC-shaped ReconstructBatch on a small device batch requests the pass's
network (compiled on the library's background thread) and the process exits at once, while the
compile is still running: the library must join its compiler thread at exit, before comgr's
static destructors run (DESIGN §4h "Exit").  Prints one JSON line; run it in a loop
(tools/gpu_round.sh ab step or a shell loop), each run a fresh process."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blb_amd import reedsolomon as rs  # noqa: E402

k, m, S, B = 12, 5, 64 << 10, 8
st = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device="cuda")
enc = rs.New(k, m)
enc.EncodeBatch(st)
bad = int(sys.argv[1]) % (k + m) if len(sys.argv) > 1 else 1
good = [i for i in range(k + m) if i != bad]
present = [i in good[:k] for i in range(k + m)]
enc.ReconstructBatch(st, present)
torch.cuda.synchronize()
print(json.dumps({"bad": bad, "rtc": rs.rtc_stats()}), flush=True)
