"""PackTracts fused with Encode, timed per call (HIP events) on distinct tract sources
(tools/tract_layout.py): RS(6,3) B=1024 and RS(8,3) B=512, `--reps` calls each after one warm-up.
Run under `rocprofv3 --kernel-trace --stats` to split a call into its pre-pass
(pe_classify_kernel) and pack_encode_kernel.  One JSON line per shape."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import tract_layout as TL  # noqa: E402
from blb_amd import pack  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--reps", type=int, default=5)
p.add_argument("--bitslice", default="1", help="BLBRS_BITSLICE values to time in turn (1 = shipped)")
p.add_argument("--jitter", action="store_true", help="0-15 extra source misalignment (non-blb)")
a = p.parse_args()
dev = torch.device("cuda:0")
S = 8 << 20
g = torch.Generator(device=dev)
g.manual_seed(5)
for k, m, B in ((6, 3, 1024), (8, 3, 512)):
    st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    enc = rs.New(k, m)
    lay = TL.layout(B * k, S, np.random.default_rng(k))
    pool, starts = TL.distinct_sources(lay, dev, g, np.random.default_rng(k + 1), jitter=a.jitter)
    ext = TL.extents(lay, pool, starts)
    read = sum(ln for _, _, ln in lay)
    for bsl in [int(x) for x in a.bitslice.split(",")]:
        rs.set_tuning("BLBRS_BITSLICE", bsl)
        pack.PackEncode(enc, st, ext)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(200_000_000)  # the host-side extent checks stay outside the window
            e0.record()
            pack.PackEncode(enc, st, ext)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        ok = bool(enc.VerifyBatch(st).all())
        algo = read + B * (k + m) * S
        best = min(ms)
        print(json.dumps({"k": k, "m": m, "batch": B, "bitslice": bsl, "network": enc.compiled_network()["pack"],
                          "lib": os.environ.get("BLBRS_LIB_PATH", "shipped"), "ms": [round(x, 3) for x in ms],
                          "algorithmic_bytes": algo, "frac_of_8TBps_best": round(algo / (best * 1e-3) / 8e12, 4),
                          "verify_ok": ok}), flush=True)
    rs.set_tuning("BLBRS_BITSLICE", 1)
    del st, pool, ext
    torch.cuda.empty_cache()
