"""Copy-engine rates for BASELINE config 5's copy-engine form (round 6): pinned host <-> HBM
hipMemcpyAsync, by copy size, stream count and direction mix.  Prints one JSON line per case.
usage: python tools/dma_probe.py"""
import json
import time

import torch

GIB = 1 << 30
dev = torch.device("cuda:0")
N = 1 << 30
host = torch.empty(N, dtype=torch.uint8).pin_memory()
hout = torch.empty(N, dtype=torch.uint8).pin_memory()
d = torch.empty(N, dtype=torch.uint8, device=dev)
d2 = torch.empty(N, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()


def run(chunk, nstreams, mix):
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    n = N // chunk
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        s = streams[i % nstreams]
        with torch.cuda.stream(s):
            sl = slice(i * chunk, (i + 1) * chunk)
            d[sl].copy_(host[sl], non_blocking=True)
            if mix:
                hout[sl].copy_(d2[sl], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return round(N / GIB / dt, 2), (round(N / GIB / dt, 2) if mix else None)


for chunk in (8 << 20, 48 << 20):
    for ns in (1, 2, 4, 8):
        for mix in (False, True):
            run(chunk, ns, mix)  # warm
            h2d, d2h = run(chunk, ns, mix)
            print(json.dumps({"chunk_MiB": chunk >> 20, "streams": ns, "with_d2h": mix, "h2d_GiBps": h2d,
                              "d2h_GiBps": d2h}), flush=True)
