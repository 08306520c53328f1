"""Measure the host-memory (PCIe-inclusive) paths on one MI355X:
  * raw pinned H2D / D2H / bidirectional copy rates (the ceiling);
  * EncodeHostBatch (streaming, pinned) vs stream count;
  * per-call Encode on pageable numpy shards at the tractserver's EncodeIncrementSize
    (4 MiB, internal/tractserver/config.go:117) and at a full 8 MiB tract, next to the CPU
    oracle doing the same call.
Prints one JSON object."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blb_amd import reedsolomon as rs  # noqa: E402

GIB = float(1 << 30)
MIB = 1 << 20


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda:0")
    out = {}
    n = 512 * MIB
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    d2 = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    t = timeit(lambda: d.copy_(h, non_blocking=True), 5)
    out["h2d_GBps"] = round(n / t / 1e9, 2)
    t = timeit(lambda: h.copy_(d, non_blocking=True), 5)
    out["d2h_GBps"] = round(n / t / 1e9, 2)

    def bidir():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    t = timeit(bidir, 5)
    out["bidir_GBps_each"] = round(n / t / 1e9, 2)
    del h, h2, d, d2

    k, m, S = 6, 3, 8 * MIB
    enc = rs.New(k, m)
    nb = 24
    pinned = torch.empty((nb, k + m, S), dtype=torch.uint8).pin_memory()
    host = pinned.numpy()
    host[:, :k] = np.random.default_rng(1).integers(0, 256, (nb, k, S), dtype=np.uint8)
    lists = [[host[b, i] for i in range(k + m)] for b in range(nb)]
    res = {}
    for ns in (1, 2, 3, 4, 6, 8):
        enc.EncodeHostBatch(lists, nstreams=ns)
        t = time.perf_counter()
        enc.EncodeHostBatch(lists, nstreams=ns)
        el = time.perf_counter() - t
        res[ns] = round(nb * k * S / GIB / el, 2)
    out["stream_encode_GiBps_data_by_nstreams"] = res

    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS") or 16)
    rows = O.build_matrix(k, m)[k:]
    for S2 in (4 * MIB, 8 * MIB):
        rng = np.random.default_rng(2)
        sh = [rng.integers(0, 256, S2, dtype=np.uint8) for _ in range(k)] + [np.empty(S2, np.uint8) for _ in range(m)]
        enc.Encode(sh)
        reps = 20
        t = time.perf_counter()
        for _ in range(reps):
            enc.Encode(sh)
        gpu = reps * k * S2 / GIB / (time.perf_counter() - t)
        pin = [torch.from_numpy(x).pin_memory().numpy() for x in sh]
        enc.Encode(pin)
        t = time.perf_counter()
        for _ in range(reps):
            enc.Encode(pin)
        gpu_pin = reps * k * S2 / GIB / (time.perf_counter() - t)
        O.code(rows, sh[:k], sh[k:], use_avx2=True, threads=threads)
        t = time.perf_counter()
        for _ in range(reps):
            O.code(rows, sh[:k], sh[k:], use_avx2=True, threads=threads)
        cpu = reps * k * S2 / GIB / (time.perf_counter() - t)
        out[f"host_call_encode_{S2 // MIB}MiB"] = {"gpu_pageable_GiBps": round(gpu, 2),
                                                   "gpu_pinned_GiBps": round(gpu_pin, 2),
                                                   "cpu_oracle_avx2_GiBps": round(cpu, 2),
                                                   "cpu_threads": threads}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
