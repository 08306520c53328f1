"""Measure the host-memory (PCIe-inclusive) paths on one MI355X:
  * raw pinned H2D / D2H / bidirectional copy rates (the ceiling);
  * EncodeHostBatch of pinned stripes (zero-copy);
  * per-call Encode on pageable numpy shards at the tractserver's EncodeIncrementSize
    (4 MiB, internal/tractserver/config.go:117) and at a full 8 MiB tract, next to the CPU
    oracle doing the same call;
  * per-call Encode / ReconstructData on shards from the pinned buffer pool
    (blbrs_buffer_get: library-owned pinned buffers, allocated once and reused -- not the
    registered caller memory the shipped rpc.GetBuffer drop-in hands out; bench.py's
    rpc_pool_extras measures that path, pkg/rpc/pool.go) from 1..16 concurrent threads, the
    way concurrent RSEncode RPCs (internal/tractserver/store.go:1099) and degraded reads
    (client/blb/reconstruct.go:173) call it, with and without a Batcher attached (concurrent
    calls share launches).
  * the client's degraded-read shape (client/blb/reconstruct.go:172-173): ReconstructData
    of one stripe whose k inputs are pool buffers and whose output is the user's pageable
    Blob.ReadAt buffer (blob.go:59), 1 and 8 MiB pieces from 1..16 threads.
Prints one JSON object.  `--pool-only` runs just the pool-call sections, `--client-only`
just the client shape (BLBRS_LIB_PATH = an older build gives the "before" numbers)."""
from __future__ import annotations

import json
import os
import sys
import threading
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
    if "--zc-sweep" in sys.argv:  # libraries before round 5 only (BLBRS_HOST_ZC was removed)
        # Zero-copy vs DMA staging of pinned shards (knob BLBRS_HOST_ZC), and the library's
        # default policy (-1), on the pool-buffer calls and the client shape.
        for mode in ("1", "0", "auto"):
            rs.set_tuning("BLBRS_HOST_ZC", -1 if mode == "auto" else int(mode))
            out[f"zc_{mode}"] = {"pool_calls": pool_calls(6, 3, seconds=1.0), "client_shape": client_shape(6, 3, 1.0)}
            print(json.dumps({mode: out[f"zc_{mode}"]}), file=sys.stderr, flush=True)
        rs.set_tuning("BLBRS_HOST_ZC", -1)
        print(json.dumps(out))
        return
    if "--client-only" in sys.argv:
        out["client_shape"] = client_shape(6, 3)
        out["lib"] = os.environ.get("BLBRS_LIB_PATH") or "blb_amd/libblbrs.so"
        print(json.dumps(out))
        return
    if "--pool-only" in sys.argv:
        out["pool_calls"] = pool_calls(6, 3)
        out["pool_calls_batched"] = pool_calls(6, 3, window_us=50)
        print(json.dumps(out))
        return
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
    enc.EncodeHostBatch(lists)
    t = time.perf_counter()
    enc.EncodeHostBatch(lists)
    el = time.perf_counter() - t
    out["host_batch_encode_pinned_GiBps_data"] = round(nb * k * S / GIB / el, 2)
    del lists, host, pinned

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
    out["pool_calls"] = pool_calls(k, m)
    out["pool_calls_batched"] = pool_calls(k, m, window_us=50)
    out["client_shape"] = client_shape(k, m)
    print(json.dumps(out))


def client_shape(k, m, seconds=1.5):
    """reconstructOneTract's call: data[i] = pool-buffer replies (library-owned
    pinned buffers from blbrs_buffer_get, standing in for rpc.GetBuffer's registered ones), data[target] = thisB[0:0:length], a slice of the user's
    pageable buffer; ReconstructData.  T threads, each its own stripe; GiB/s of data (k
    pieces per call)."""
    res = {}
    target = 2
    for S in (1 * MIB, 8 * MIB):
        enc = rs.New(k, m, devices=[0])
        for T in (1, 2, 4, 8, 16):
            stripes = []
            for t in range(T):
                sh = [rs.GetBuffer(S) for _ in range(k + m)]
                rng = np.random.default_rng(t)
                for i in range(k):
                    sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
                enc.Encode(sh)
                truth = sh[target].copy()
                thisB = np.empty(S + 4096, np.uint8)   # pageable, as Blob.ReadAt's p
                stripes.append((sh, truth, thisB))
            counts = [0] * T
            ok = [True] * T
            stop = time.perf_counter() + seconds

            def loop(t):
                sh, truth, thisB = stripes[t]
                while time.perf_counter() < stop:
                    work = list(sh)
                    work[target] = None
                    enc.ReconstructData(work, outs={target: thisB})
                    counts[t] += 1
                ok[t] = bool(np.array_equal(thisB[:S], truth))

            t0 = time.perf_counter()
            th = [threading.Thread(target=loop, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            el = time.perf_counter() - t0
            res[f"{S // MIB}MiB_T{T}_GiBps_data"] = round(sum(counts) * k * S / GIB / el, 2)
            res[f"{S // MIB}MiB_T{T}_calls_per_s"] = round(sum(counts) / el, 1)
            res[f"{S // MIB}MiB_T{T}_ok"] = all(ok)
            for sh, _, _ in stripes:
                for b in sh:
                    rs.PutBuffer(b)
    return res


def pool_calls(k, m, window_us=None, seconds=2.0):
    """Per-call host Encode / ReconstructData of one stripe of 4 MiB pool buffers per call,
    T threads each looping over its own stripe for ~2 s; with `window_us`, through a Batcher
    (max_batch 32) attached to the encoder."""
    res = {}
    S = 4 * MIB
    enc = rs.New(k, m, devices=[0])
    batcher = None
    if window_us is not None:
        batcher = rs.Batcher(max_batch=32, window_us=window_us, devices=[0])
        enc.SetBatcher(batcher)
        res["window_us"] = window_us
    for T in ((1, 2, 4, 8, 16) if batcher is None else (1, 4, 8, 16, 32)):
        stripes = []
        for t in range(T):
            sh = [rs.GetBuffer(S) for _ in range(k + m)]
            rng = np.random.default_rng(t)
            for i in range(k):
                sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
            enc.Encode(sh)
            stripes.append(sh)
        for op in ("encode", "reconstruct_data1"):
            counts = [0] * T
            stop = time.perf_counter() + seconds

            def loop(t):
                sh = stripes[t]
                out1 = sh[1]
                while time.perf_counter() < stop:
                    if op == "encode":
                        enc.Encode(sh)
                    else:
                        work = list(sh)
                        work[1] = None
                        enc.ReconstructData(work, outs={1: out1})
                    counts[t] += 1

            t0 = time.perf_counter()
            th = [threading.Thread(target=loop, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            el = time.perf_counter() - t0
            res[f"{op}_T{T}_GiBps_data"] = round(sum(counts) * k * S / GIB / el, 2)
            res[f"{op}_T{T}_calls_per_s"] = round(sum(counts) / el, 1)
        for sh in stripes:
            for b in sh:
                rs.PutBuffer(b)
    res["shard_bytes"] = S
    res["device_stats"] = rs.device_stats(0)
    if batcher is not None:
        res["batcher_requests"], res["batcher_launches"] = batcher.stats()
        enc.SetBatcher(None)
        batcher.close()
    return res


if __name__ == "__main__":
    main()
