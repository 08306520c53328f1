"""bench.py -- RS encode throughput on device-resident 8 MiB tracts (BASELINE.json metric).

Step = one batched RS(6,3) Encode of B=1024 stripes of 8 MiB tracts already resident in
HBM (BASELINE configs[1]); one kernel launch per step.  N GPUs: one process per GPU, each
encodes its own B stripes (weak scaling; stripes are independent, no collective on the
data path -- torch.distributed is used only for the barrier and the max-over-ranks time).

Prints ONE JSON line (rank 0).  `value` = data GiB/s over all ranks = N*B*k*S / t.
`roofline` prices the encode kernel by its algorithmic HBM bytes B*(k+m)*S per launch over
the launch time measured with HIP events on the launch stream.  `cpu_baseline` (rank 0,
N=1 only) times the CPU restatement oracle (klauspost's AVX2 nibble-table algorithm,
OpenMP) on a bounded sample -- a reported baseline, not the target.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from blb_amd import multigpu  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
import tract_layout as TL  # noqa: E402  (synthetic PackTracts extent sets)

GIB = float(1 << 30)
TRACT = 8 * 1024 * 1024          # core.TractLength (internal/core/constants.go:15)
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0            # MI355X_MICROARCH.md: 6.29 TB/s measured float4 copy
METRIC = "RS encode/decode GiB/s (device-resident 8MB tracts) at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--k", type=int, default=6)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--batch", type=int, default=1024, help="stripes per GPU (weak scaling)")
    p.add_argument("--total-batch", type=int, default=0,
                   help="if set: stripes for the whole job, split over ranks (strong scaling, "
                        "e.g. BASELINE config 4: --k 10 --m 4 --total-batch 4096)")
    p.add_argument("--shard", type=int, default=TRACT)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-extra", action="store_true", help="skip decode / PCIe side measurements")
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for the barrier/max-time collectives (nccl = RCCL); "
                        "'gloo' with ranks sharing a GPU is a rehearsal of the N>1 path on a 1-GPU box")
    return p.parse_args()


def lib_sha256():
    import hashlib
    from blb_amd import _lib
    return hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()


def pmc_traffic(k, m, batch, shard):
    """HBM bytes per launch of the encode kernel from a committed rocprofv3 --pmc summary
    (profiles/pmc_*.json, tools/pmc_prod.sh), used only when it was measured on THIS library
    build (same libblbrs.so sha256) for this exact workload; else None."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    sha = lib_sha256()
    for fn in sorted(os.listdir(pdir), reverse=True):
        if fn.startswith("pmc_") and fn.endswith(".json"):
            try:
                d = json.load(open(os.path.join(pdir, fn)))
            except (OSError, ValueError):
                continue
            w = d.get("workload", {})
            if (w.get("k"), w.get("m"), w.get("batch"), w.get("shard")) == (k, m, batch, shard) \
                    and d.get("lib_sha256") == sha:
                return d.get("hbm_bytes_per_launch"), fn
    return None, None


def cgroup_cpu_quota():
    """The job's CPU quota in cores from the cgroup (v2 cpu.max, else v1 cfs quota/period);
    None when unlimited or unreadable, with the raw text."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            raw = open(path).read().strip()
            q, per = raw.split()[:2]
            return (None if q == "max" else round(int(q) / int(per), 2)), f"{path}: {raw}"
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return (None if q < 0 else round(q / per, 2)), f"cgroup v1 cfs_quota_us={q} cfs_period_us={per}"
    except (OSError, ValueError):
        return None, "no cgroup cpu quota file"


def cpu_baseline(k, m, seconds):
    """klauspost's algorithm (AVX2 vpshufb nibble tables, OpenMP byte-range split like
    codeSomeShardsP) from the oracle restatement, on a bounded sample of the workload.  Records
    what bounds the thread count (affinity, OMP_NUM_THREADS, cgroup quota), the rate per thread
    and a 1/2/4/8/16-thread sweep up to the job's share, so the figure can be scaled to a whole
    host."""
    from oracle import oracle as O
    # Every core this process may run on (its affinity mask), capped by OMP_NUM_THREADS where
    # the GPU box sets it to the job's CPU share, and by the cgroup quota.
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)
    quota, quota_src = cgroup_cpu_quota()
    threads = max(1, min(affinity, omp) if omp else affinity)
    if quota is not None:
        threads = max(1, min(threads, int(quota)))
    cpu_model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu_model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nstripes = 4
    rng = np.random.default_rng(97531)
    rows = O.build_matrix(k, m)[k:]
    stripes = []
    for _ in range(nstripes):
        data = [rng.integers(0, 256, TRACT, dtype=np.uint8) for _ in range(k)]
        par = [np.empty(TRACT, np.uint8) for _ in range(m)]
        stripes.append((data, par))
    O.code(rows, stripes[0][0], stripes[0][1], use_avx2=True, threads=threads)  # warm
    done, t0 = 0, time.perf_counter()
    intervals, i_done, i_t0 = [], 0, t0   # ~1 s windows: a shared host's load shows up as spread
    while True:
        for data, par in stripes:
            O.code(rows, data, par, use_avx2=True, threads=threads)
        done += nstripes
        now = time.perf_counter()
        el = now - t0
        if now - i_t0 >= 1.0:
            intervals.append((done - i_done) * k * TRACT / GIB / (now - i_t0))
            i_done, i_t0 = done, now
        if el >= seconds:
            break
    gibps = done * k * TRACT / GIB / el
    intervals.sort()
    # Thread sweep (1.5 s per point) on the same stripes: how the rate scales with cores.
    sweep = {}
    for t in (1, 2, 4, 8, 16):
        if t > threads:
            break
        n, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < 1.5:
            data, par = stripes[n % nstripes]
            O.code(rows, data, par, use_avx2=True, threads=t)
            n += 1
        sweep[str(t)] = round(n * k * TRACT / GIB / (time.perf_counter() - t1), 2)
    out = {"value": round(gibps, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
           "per_thread_GiBps": round(gibps / threads, 3),
           "thread_sweep_GiBps": sweep,
           "interval_GiBps": {"min": round(intervals[0], 2), "median": round(intervals[len(intervals) // 2], 2),
                              "max": round(intervals[-1], 2), "windows": len(intervals)} if intervals else None,
           "scaling_note": "per_thread_GiBps x a host's cores is an upper bound; the sweep shows how far "
                           "from linear the rate already is at the job's share",
           "nproc": affinity, "os_cpu_count": os.cpu_count(), "omp_num_threads": omp or None,
           "cgroup_cpu_quota_cores": quota, "cgroup_cpu_quota_source": quota_src,
           "cpu_model": cpu_model, "avx2": bool(O.lib().rso_have_avx2()),
           "sample": f"RS({k},{m}) encode of {done} stripes x {k}x8MiB "
                     f"({done * k * TRACT / GIB:.1f} GiB data, {el:.1f} s) by the oracle's "
                     f"klauspost-AVX2 restatement, {threads} OpenMP threads"}
    # The other BASELINE rows on the same restatement (~2 s each).  Decode = the rows of
    # inv(M[first k present]) for the erased data shards, applied to the k survivors.
    def rate(kk, mm, missing, secs=2.0):
        mat = O.build_matrix(kk, mm)
        if missing:
            valid = [i for i in range(kk + mm) if i not in missing][:kk]
            rows_ = O.invert(mat[valid])[list(missing)]
        else:
            rows_ = mat[kk:]
        # 4 stripes in rotation, like the encode sample: the working set is not cache-resident
        sets = [([rng.integers(0, 256, TRACT, dtype=np.uint8) for _ in range(kk)],
                 [np.empty(TRACT, np.uint8) for _ in range(rows_.shape[0])]) for _ in range(4)]
        O.code(rows_, sets[0][0], sets[0][1], use_avx2=True, threads=threads)
        n, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < secs:
            ins, outs = sets[n % 4]
            O.code(rows_, ins, outs, use_avx2=True, threads=threads)
            n += 1
        return round(n * kk * TRACT / GIB / (time.perf_counter() - t1), 2)
    out["configs"] = {"unit": "GiB/s of data (k shards x 8 MiB per call)",
                      "rs63_reconstruct_data1": rate(6, 3, [1]),
                      "rs104_encode": rate(10, 4, []),
                      "rs104_reconstruct_data1_data7": rate(10, 4, [1, 7])}
    # CRC-32C row: Go's amd64 algorithm class (SSE4.2, 3 interleaved streams), 65532-byte
    # ChecksumFile blocks of m parity rows, ~3 s.
    if O.lib().rso_have_sse42():
        buf = rng.integers(0, 256, m * TRACT, dtype=np.uint8)
        O.crc32c_blocks_hw(buf, 65532, threads)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(3.0, seconds):
            O.crc32c_blocks_hw(buf, 65532, threads)
            done += 1
        el = time.perf_counter() - t0
        out["crc32c"] = {"value": round(done * buf.size / el / 1e9, 2), "unit": "GB/s", "cores": threads,
                         "kind": "port", "sample": f"{done} x CRC-32C of {m}x8MiB in 65532-byte blocks "
                                                   f"({el:.1f} s), SSE4.2 3-stream, {threads} OpenMP threads"}
    return out


def timed_all_ranks(fn, iters, dev, dist):
    """Wall time of `iters` calls of fn on every rank, bracketed by barrier + sync on both
    sides, max over ranks (the same clock discipline as the headline measurement)."""
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    return multigpu.max_over_ranks(time.perf_counter() - t0, dev)


def scale_extras(enc, k, m, S, world, rank, dev, dist):
    """BASELINE configs 4 and 5 at the job's N (run on every rank, aggregated over ranks):

    * config 4 -- RS(10,4) Encode, then Reconstruct of 2 erasures (data 1 + data 7), 512
      stripes per GPU: at N=8 that is exactly the batch=4096 split across 8 GPUs;
    * config 5 -- RS(k,m) Encode of pinned host-resident stripes (PCIe-inclusive: the kernel
      reads data and writes parity in host memory over PCIe), 24 stripes per GPU.

    Totals are all ranks' data bytes / the max-over-ranks wall time."""
    out = {}
    per = 512
    st = torch.empty((per, 14, S), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(97531 * (rank + 11))
    st[:, :10].random_(0, 256, generator=g)
    e104 = rs.New(10, 4)
    e104.EncodeBatch(st)
    ok = bool(e104.VerifyBatch(st).all())
    t_enc = timed_all_ranks(lambda: e104.EncodeBatch(st), 3, dev, dist)
    present = [i not in (1, 7) for i in range(14)]
    st[:, 1].fill_(0xA5)  # really erase: the timed reconstructs must restore these bytes
    st[:, 7].fill_(0x5A)
    e104.ReconstructBatch(st, present, data_only=False)
    t_rec = timed_all_ranks(lambda: e104.ReconstructBatch(st, present, data_only=False), 3, dev, dist)
    ok = ok and bool(e104.VerifyBatch(st).all())
    data_all = per * world * 10 * S * 3
    out["config4_rs104_encode_reconstruct2"] = {
        "stripes_total": per * world, "stripes_per_gpu": per,
        "encode_GiBps_data": round(data_all / GIB / t_enc, 1),
        "reconstruct2_GiBps_data": round(data_all / GIB / t_rec, 1),
        "encode_ms": round(t_enc / 3 * 1e3, 3), "reconstruct2_ms": round(t_rec / 3 * 1e3, 3),
        "verify_ok": ok}
    del st
    torch.cuda.empty_cache()

    nb = 24
    pinned = torch.empty((nb, k + m, S), dtype=torch.uint8).pin_memory()
    pinned[:, :k].copy_(torch.randint(0, 256, (nb, k, S), dtype=torch.uint8, device=dev, generator=g))
    host = pinned.numpy()
    lists = [[host[b, i] for i in range(k + m)] for b in range(nb)]
    enc.EncodeHostBatch(lists)
    t_host = timed_all_ranks(lambda: enc.EncodeHostBatch(lists), 2, dev, dist)
    parity = host[:, k:].copy()
    # The copy-engine form BASELINE config 5 names: hipMemcpyAsync H2D of the data shards into a
    # device ring, the kernel on HBM, hipMemcpyAsync D2H of the parity, over nstreams streams.
    dma = {}
    for ns in (2, 4, 8):
        host[:, k:] = 0xA5
        enc.EncodeHostBatch(lists, nstreams=ns)
        same = bool(np.array_equal(host[:, k:], parity))
        t = timed_all_ranks(lambda: enc.EncodeHostBatch(lists, nstreams=ns), 2, dev, dist)
        dma[f"nstreams_{ns}"] = {"GiBps_data": round(nb * world * k * S * 2 / GIB / t, 2), "parity_same_as_zero_copy": same}
    out["config5_pcie_inclusive_encode"] = {
        "GiBps_data": round(nb * world * k * S * 2 / GIB / t_host, 2), "stripes_per_gpu": nb,
        "copy_engines": dma,
        "note": "pinned host stripes; GiBps_data = coded in place over PCIe (zero copy: data read and "
                "parity written in host memory by the kernel, the shipped default nstreams = 0); "
                "copy_engines = hipMemcpyAsync H2D / kernel / D2H pipeline on a device ring; not the bench value"}
    del pinned
    return out


def host_call_extras(k, m, dev, threads=16, seconds=1.0):
    """The tractserver's real call shape (rank 0 at N=1): `threads` concurrent RSEncode RPCs,
    each calling Encode on one 4 MiB increment (EncodeIncrementSize, store.go:1099) of
    library-owned pinned buffers (blbrs_buffer_get, allocated once and reused, coded in place
    over PCIe), per call and through a Batcher (window 0).  `rpc_pool_churn` is the path blb
    would actually run (rpc_pool_extras).  PCIe-inclusive; never the bench value."""
    import threading
    S = 4 << 20
    out = {"threads": threads, "increment_bytes": S}
    stripes = []
    for t in range(threads):
        sh = [rs.GetBuffer(S) for _ in range(k + m)]
        g = np.random.default_rng(t)
        for i in range(k):
            sh[i][:] = g.integers(0, 256, S, dtype=np.uint8)
        stripes.append(sh)
    try:
        for mode in ("per_call", "batched"):
            enc = rs.New(k, m, devices=[dev.index])
            b = rs.Batcher(max_batch=64, window_us=0, devices=[dev.index]) if mode == "batched" else None
            if b is not None:
                enc.SetBatcher(b)
            for sh in stripes:
                enc.Encode(sh)
            counts = [0] * threads
            stop = time.perf_counter() + seconds

            def loop(t):
                while time.perf_counter() < stop:
                    enc.Encode(stripes[t])
                    counts[t] += 1

            t0 = time.perf_counter()
            th = [threading.Thread(target=loop, args=(t,)) for t in range(threads)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            el = time.perf_counter() - t0
            out[f"{mode}_GiBps_data"] = round(sum(counts) * k * S / GIB / el, 2)
            if b is not None:
                out["calls_per_launch"] = round(b.stats()[0] / max(1, b.stats()[1]), 2)
                enc.SetBatcher(None)
                b.close()
        ok = all(enc.Verify(sh) for sh in stripes[:2])
        out["verify_ok"] = bool(ok)
    finally:
        for sh in stripes:
            for x in sh:
                rs.PutBuffer(x)
    return out


def rpc_pool_extras(k, m, dev, threads=16, seconds=1.0, gc_every=(0, 64, 8)):
    """rpc.GetBuffer as blb's drop-in pool builds it (blb_amd/rpc.py = go/rsgpu's GetBuffer):
    caller-owned class buffers registered with the engine on creation and unregistered when
    collected.  Each of `threads` RPC threads takes k + m 4 MiB buffers per call with
    GetBuffer, Encodes, and PutBuffers them; every `gc_every` calls per thread it runs rpc.gc()
    (what a Go GC cycle does to a sync.Pool: the idle buffers are dropped, so later calls
    register fresh ones).  0 = no GC.  Reports GiB/s of data, the registrations and the mean
    hipHostRegister / hipHostUnregister wall time per 4 MiB buffer under concurrent coding."""
    import threading
    from blb_amd import rpc
    S = 4 << 20
    out = {"threads": threads, "increment_bytes": S}
    enc = rs.New(k, m, devices=[dev.index])
    g = np.random.default_rng(5)
    data = [g.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    for every in gc_every:
        rpc.gc()
        base = dict(rpc.stats)
        counts = [0] * threads
        stop = time.perf_counter() + seconds

        def loop(t):
            n = 0
            while time.perf_counter() < stop:
                sh = [rpc.GetBuffer(S) for _ in range(k + m)]
                for i in range(k):
                    sh[i][:] = data[i]
                enc.Encode(sh)
                for b in sh:
                    rpc.PutBuffer(b)
                n += 1
                if every and n % every == 0:
                    rpc.gc()
            counts[t] = n

        t0 = time.perf_counter()
        th = [threading.Thread(target=loop, args=(t,)) for t in range(threads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        el = time.perf_counter() - t0
        d = {key: rpc.stats[key] - base[key] for key in base}
        out[f"gc_every_{every or 'never'}"] = {
            "GiBps_data": round(sum(counts) * k * S / GIB / el, 2), "calls": sum(counts),
            "registrations": d["registered"] + d["reregistered"], "unregistrations": d["unregistered"],
            "refused": d["refused"],
            "register_ms_mean": round(1e3 * d["register_s"] / max(1, d["registered"] + d["reregistered"]), 3),
            "unregister_ms_mean": round(1e3 * d["unregister_s"] / max(1, d["unregistered"]), 3)}
    rpc.gc()
    return out


def wide_fused_extras(S, dev):
    """Fused encode+CRC (65532-byte ChecksumFile blocks) against the plain encode of the same
    stripes for blb's widest class RS(12,5) and the bench's RS(10,4), B=512 each, interleaved
    reps on one stream (rank 0 at N=1 only).  The shipped path runs the compiled bit-plane
    network; `tables` repeats both on the v_perm table path (knob BLBRS_BITSLICE=0)
    for comparison with round 2."""
    out = {}
    stream = torch.cuda.current_stream(dev)
    for k, m in ((12, 5), (10, 4)):
        st = torch.empty((512, k + m, S), dtype=torch.uint8, device=dev)
        st[:, :k].random_(0, 256)
        e = rs.New(k, m)
        e.EncodeBatch(st)
        e.EncodeBatchCRC(st, 65532)
        torch.cuda.synchronize(dev)
        times = {}
        for _ in range(3):
            for path, knobs in (("network", {}), ("tables", {"BLBRS_BITSLICE": 0})):
                with rs.tuning(**knobs):
                    for name, fn in (("encode", lambda: e.EncodeBatch(st)), ("fused", lambda: e.EncodeBatchCRC(st, 65532))):
                        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        s0.record(stream)
                        fn()
                        s1.record(stream)
                        torch.cuda.synchronize(dev)
                        times.setdefault((path, name), []).append(s0.elapsed_time(s1))
        ok = bool(e.VerifyBatch(st).all())
        ms = {key: float(np.mean(v)) for key, v in times.items()}
        nbytes = 512 * (k + m) * S
        out[f"encode_crc_fused_rs{k}_{m}_b512"] = {
            "encode_ms": round(ms[("network", "encode")], 3), "fused_ms": round(ms[("network", "fused")], 3),
            "ratio_to_encode": round(ms[("network", "fused")] / ms[("network", "encode")], 3),
            "fused_frac_of_8TBps": round(nbytes / (ms[("network", "fused")] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "compiled_network": e.compiled_network(),
            "tables": {"encode_ms": round(ms[("tables", "encode")], 3), "fused_ms": round(ms[("tables", "fused")], 3)},
            "block": 65532, "verify_ok": ok}
        del st
        torch.cuda.empty_cache()
    return out


def _ev_ms(fn, reps, stream, dev):
    """Mean HIP-event time (ms) of `reps` calls of fn on `stream` (one event pair per call)."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in evs:
        s.record(stream)
        fn()
        e.record(stream)
    torch.cuda.synchronize(dev)
    return float(np.mean([s.elapsed_time(e) for s, e in evs]))


def _stream_probe():
    """tools/_build/libstream_probe.so (the access-pattern probe), or None when not built."""
    import ctypes
    path = os.path.join(ROOT, "tools", "_build", "libstream_probe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.stream_probe.restype = ctypes.c_int
    lib.stream_probe.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] + [ctypes.c_size_t] * 4 + [ctypes.c_void_p]
    return lib


def recovery_extras(S, dev, reps=3, classes=((6, 3, 1024), (8, 3, 768), (10, 3, 640), (12, 5, 480))):
    """blb's real recovery call shapes for every storage class (rank 0 at N=1), B chosen so each
    batch is ~64-72 GiB of HBM:

    * rpc_{e}bad -- the curator's recovery RPC (internal/curator/reconstruct.go:51-79 ->
      internal/tractserver/store.go:1062-1102): the tractserver reads exactly the first k good
      pieces and Reconstruct rebuilds ALL m absent slots (the e bad pieces and the good parity
      pieces it did not read); the Verify after it has nothing left to compare.  e = 1 and m.
    * client_rows{r} -- the client's degraded read (client/blb/reconstruct.go:137-173): the
      first k good replies, ReconstructData of the r missing data slots (r = 1: every other
      data piece answered; r = m: the parity pieces answered first).

    Each row: the shipped path's HIP-event time under default knobs -- the v_perm tables, or on
    RS(12,5)-wide multi-row passes the run-time network, compiled in the background on first use
    (BLBRS_RTC = 1, default since round 6; timed once compiled, rs.rtc_wait) -- and there the
    tables beside it (BLBRS_RTC = 0), each checked bit-exact, algorithmic bytes B*(k+rows)*S and
    the fraction of 8 TB/s, and the trivial-XOR stream of the same reads and writes in the same
    layout and launch shape (tools/stream_probe.hip) at the kernel's U and at its best U."""
    probe = _stream_probe()
    stream = torch.cuda.current_stream(dev)
    out = {"note": "ms = median of interleaved reps; probe = trivial-XOR stream, same bytes/layout/launch"}
    for k, m, B in classes:
        n = k + m
        st = torch.empty((B, n, S), dtype=torch.uint8, device=dev)
        g = torch.Generator(device=dev)
        g.manual_seed(97531 + k)
        st[:, :k].random_(0, 256, generator=g)
        e = rs.New(k, m)
        e.EncodeBatch(st)
        spread = [1 + (i * k) // m for i in range(m)]
        rows = []
        for nbad in (1, m):
            good = [i for i in range(n) if i not in spread[:nbad]]
            rows.append((f"rpc_{nbad}bad", [i in good[:k] for i in range(n)], False, m))
        rows.append(("client_rows1", [i != 1 and i <= k for i in range(n)], True, 1))
        first_k = [j for j in range(n) if j not in spread][:k]
        rows.append((f"client_rows{m}", [i in first_k for i in range(n)], True, m))
        cls = {}
        for name, present, data_only, nrows in rows:
            targets = [i for i in range(n) if not present[i] and (i < k or not data_only)]
            ref = {i: st[:, i].clone() for i in targets if i < k}
            net = rs.rtc_eligible(k, nrows)   # the shipped default runs a run-time network
            knobs = {"shipped": {}}
            if net:
                knobs["tables"] = {"BLBRS_RTC": 0}
                e.ReconstructBatch(st, present, data_only=data_only)   # requests the network
                rs.rtc_wait(120000)                                     # compiled; the next launch loads it
            # Bit-exactness of every variant timed below.
            exact = {}
            for key, kn in knobs.items():
                for i in targets:
                    st[:, i].fill_(0xA5)
                with rs.tuning(**kn):
                    e.ReconstructBatch(st, present, data_only=data_only)
                torch.cuda.synchronize(dev)
                ok = all(bool(torch.equal(st[:, i], r)) for i, r in ref.items())
                if not data_only:
                    ok = ok and bool(e.VerifyBatch(st).all())
                exact[key] = ok
            del ref
            u = 4 if k + nrows <= 9 else 2
            run = lambda: e.ReconstructBatch(st, present, data_only=data_only)  # noqa: E731
            fns = {key: run for key in knobs}
            if probe is not None:
                for pu in (1, 2, 4):
                    fns[f"probe_u{pu}"] = (lambda pu=pu: probe.stream_probe(
                        k, nrows, pu, st.data_ptr(), S, n * S, B, S, stream.cuda_stream))
            times = {key: [] for key in fns}
            for _ in range(reps):
                for key, fn in fns.items():
                    with rs.tuning(**knobs.get(key, {})):
                        times[key].append(_ev_ms(fn, 1, stream, dev))
            e.EncodeBatch(st)  # the probe wrote garbage over parity shards [k, k + rows): restore them
            ms = {key: sorted(v)[len(v) // 2] for key, v in times.items()}
            nbytes = B * (k + nrows) * S
            row = {"rows": nrows, "present": [i for i in range(n) if present[i]], "algorithmic_bytes": nbytes,
                   "ms": round(ms["shipped"], 3), "frac_of_8TBps": round(nbytes / (ms["shipped"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "bit_exact": exact["shipped"], "kernel": "run-time network" if net else "tables"}
            if net:  # the v_perm tables beside the shipped network (BLBRS_RTC = 0)
                row["tables_ms"] = round(ms["tables"], 3)
                row["tables_bit_exact"] = exact["tables"]
            if probe is not None:
                best = min(ms[f"probe_u{pu}"] for pu in (1, 2, 4))
                row.update({"probe_ms_same_u": round(ms[f"probe_u{u}"], 3), "probe_ms_best_u": round(best, 3),
                            "ratio_to_probe": round(ms["shipped"] / best, 4)})
            cls[name] = row
        out[f"RS({k},{m})_B{B}"] = cls
        del st
        torch.cuda.empty_cache()
    out["rtc"] = rs.rtc_stats()
    return out


def cold_class_extras(S, dev, batch=512, reps=4):
    """blb's COLD transition class RS(8,3) (targetClass, internal/curator/
    storage_class_loop.go:41-44), B=512 stripes of 8 MiB (rank 0 at N=1): Encode, 1- and
    2-erasure Reconstruct, Encode fused with the ChecksumFile CRCs of a parity window at file
    offset 4 MiB (phase 256, seeded), and PackTracts fused with Encode.  Each row carries its
    algorithmic HBM bytes per launch and the fraction of the 8 TB/s spec."""
    from blb_amd import pack
    k, m = 8, 3
    n = k + m
    stream = torch.cuda.current_stream(dev)
    st = torch.empty((batch, n, S), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(8303)
    st[:, :k].random_(0, 256, generator=g)
    e = rs.New(k, m)
    out = {"workload": f"RS(8,3), batch={batch} stripes of {S >> 20} MiB", "compiled_network": e.compiled_network()}

    def row(name, ms, nbytes, **kw):
        gbs = nbytes / (ms * 1e-3) / 1e9
        out[name] = {"ms_per_launch": round(ms, 3), "hbm_GBps_algorithmic": round(gbs, 1),
                     "frac_of_8TBps": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": nbytes, **kw}

    e.EncodeBatch(st)
    torch.cuda.synchronize(dev)
    enc_ms = _ev_ms(lambda: e.EncodeBatch(st), reps, stream, dev)
    ok = bool(e.VerifyBatch(st).all())
    row("encode", enc_ms, batch * n * S, GiBps_data=round(batch * k * S / GIB / (enc_ms * 1e-3), 1), verify_ok=ok)
    ref = st[:, 1].clone()
    pres1 = [i != 1 for i in range(n)]
    st[:, 1].fill_(0xA5)
    e.ReconstructBatch(st, pres1, data_only=True)
    r1_ok = bool(torch.equal(st[:, 1], ref))
    r1_ms = _ev_ms(lambda: e.ReconstructBatch(st, pres1, data_only=True), reps, stream, dev)
    row("reconstruct_1_data_erasure", r1_ms, batch * (k + 1) * S, restored=r1_ok)
    pres2 = [i not in (1, 5) for i in range(n)]
    ref5 = st[:, 5].clone()
    st[:, 1].fill_(0x5A)
    st[:, 5].fill_(0xC3)
    e.ReconstructBatch(st, pres2)
    r2_ok = bool(torch.equal(st[:, 1], ref)) and bool(torch.equal(st[:, 5], ref5))
    r2_ms = _ev_ms(lambda: e.ReconstructBatch(st, pres2), reps, stream, dev)
    row("reconstruct_2_data_erasures", r2_ms, batch * (k + 2) * S, restored=r2_ok)
    del ref, ref5
    # rsEncodeOne's parity window 1 (file offset 4 MiB: phase 4 MiB mod 65532 = 256), seeded
    # with the CRC of the partial block window 0 left (crc32.Update, checksum_block.go:76-81).
    seeds = torch.randint(-2**31, 2**31 - 1, (m, batch), dtype=torch.int32, device=dev)
    e.EncodeBatchCRC(st, 65532, phase=256, seeds=seeds)
    torch.cuda.synchronize(dev)
    fc_ms = _ev_ms(lambda: e.EncodeBatchCRC(st, 65532, phase=256, seeds=seeds), reps, stream, dev)
    row("encode_crc_fused_b65532_phase256", fc_ms, batch * n * S, ratio_to_encode=round(fc_ms / enc_ms, 3),
        verify_ok=bool(e.VerifyBatch(st).all()))
    # PackTracts + Encode: tracts of 64 KiB..8 MiB at padToLength-aligned offsets into the B*k
    # data pieces, from distinct sources (the row's rate) and from one shared 4 GiB pool
    # (tools/tract_layout.py).
    lay = TL.layout(batch * k, S, np.random.default_rng(83))
    read_bytes = sum(ln for _, _, ln in lay)
    pe = {}
    for name, (pool, starts) in (("distinct", TL.distinct_sources(lay, dev, g, np.random.default_rng(84))),
                                 ("shared", TL.shared_sources(lay, 4 << 30, dev, np.random.default_rng(85)))):
        ext = TL.extents(lay, pool, starts)
        pack.PackEncode(e, st, ext)
        torch.cuda.synchronize(dev)
        torch.cuda._sleep(400_000_000)  # keeps the host-side extent checks outside the window
        pe[name] = (_ev_ms(lambda: pack.PackEncode(e, st, ext), 1, stream, dev), bool(e.VerifyBatch(st).all()))
        del pool, ext
    row("pack_encode_fused", pe["distinct"][0], read_bytes + batch * n * S, sources="distinct",
        shared_pool_ms=round(pe["shared"][0], 3), bytes_read=read_bytes, tracts=len(lay),
        verify_ok=pe["distinct"][1] and pe["shared"][1])
    del st
    torch.cuda.empty_cache()
    return out


def main():
    a = parse()
    r = multigpu.env_rank()
    world, rank, local = r.world, r.rank, r.local
    local = local % max(1, torch.cuda.device_count())  # identity on a node with >= N GPUs
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # NUMA: this rank's CPUs and future host pages on its GPU's node (2 sockets x 4 GPUs on an
    # 8-GPU host), before any pin_memory (config 5's pinned stripes, the pool buffers).
    numa = multigpu.bind_to_node(rs.device_numa_node(local))
    # One process per GPU: this rank's host-memory calls (config 5) stay on its own GPU
    # instead of spreading over every visible device (the library's in-process default).
    rs.set_default_devices([local])
    dist = None
    if world > 1:
        import torch.distributed as dist
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.backend)

    k, m, S = a.k, a.m, a.shard
    if a.total_batch:
        _, B = multigpu.stripe_range(a.total_batch, world, rank)
    else:
        B = a.batch
    enc = rs.New(k, m)
    stripes = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(97531 * (rank + 1))
    stripes[:, :k].random_(0, 256, generator=g)
    stream = torch.cuda.current_stream(dev)

    for _ in range(a.warmup):
        enc.EncodeBatch(stripes)
    torch.cuda.synchronize(dev)
    ok = bool(enc.VerifyBatch(stripes).all())
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        enc.EncodeBatch(stripes)
        e.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt_local = time.perf_counter() - t0
    dt = multigpu.max_over_ranks(dt_local, dev)
    value = multigpu.aggregate_gibps(float(B * k * S * a.steps), dt_local, dev)

    launch_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    algo_bytes = B * (k + m) * S
    achieved_gbs = algo_bytes / (launch_ms * 1e-3) / 1e9

    extra = {}
    cpu = None
    if rank == 0 and world == 1 and not a.no_extra:
        # BASELINE config 3: ReconstructData of data shard 1 over the same batch.
        present = [i != 1 for i in range(k + m)]
        enc.ReconstructBatch(stripes, present, data_only=True)
        torch.cuda.synchronize(dev)
        dev_evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(max(3, a.steps // 2))]
        for s, e in dev_evs:
            s.record(stream)
            enc.ReconstructBatch(stripes, present, data_only=True)
            e.record(stream)
        torch.cuda.synchronize(dev)
        dec_ms = float(np.mean([s.elapsed_time(e) for s, e in dev_evs]))
        extra["reconstruct_1_data_erasure"] = {
            "GiBps_data": round(B * k * S / GIB / (dec_ms * 1e-3), 2),
            "ms_per_launch": round(dec_ms, 3),
            "hbm_GBps_algorithmic": round(B * (k + 1) * S / (dec_ms * 1e-3) / 1e9, 1)}
        # The recovery write path: the same rebuild fused with the ChecksumFile CRCs of the
        # rebuilt shard (blbrs_reconstruct_crc_dev_at, 65532-byte blocks).
        enc.ReconstructBatchCRC(stripes, present, 65532, data_only=True)
        torch.cuda.synchronize(dev)
        for s, e in dev_evs:
            s.record(stream)
            enc.ReconstructBatchCRC(stripes, present, 65532, data_only=True)
            e.record(stream)
        torch.cuda.synchronize(dev)
        rc_ms = float(np.mean([s.elapsed_time(e) for s, e in dev_evs]))
        extra["reconstruct_crc_fused_1_data_erasure"] = {
            "ms_per_launch": round(rc_ms, 3), "ratio_to_reconstruct": round(rc_ms / dec_ms, 3), "block": 65532,
            "hbm_GBps_algorithmic": round(B * (k + 1) * S / (rc_ms * 1e-3) / 1e9, 1)}
        # Verify (reconstructAndVerify's parity recompute + compare, store.go:1136), fused.
        ver_evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(max(3, a.steps // 2))]
        flags_ok = True
        for s, e in ver_evs:
            s.record(stream)
            okv = enc.VerifyBatch(stripes)
            e.record(stream)
            flags_ok = flags_ok and bool(okv.all())
        torch.cuda.synchronize(dev)
        ver_ms = float(np.mean([s.elapsed_time(e) for s, e in ver_evs]))
        extra["verify"] = {"GiBps_data": round(B * k * S / GIB / (ver_ms * 1e-3), 2),
                           "ms_per_launch": round(ver_ms, 3), "all_ok": flags_ok,
                           "hbm_GBps_algorithmic": round(B * (k + m) * S / (ver_ms * 1e-3) / 1e9, 1)}
        # reconstructAndVerify (store.go:1132-1142) with all 8 survivors present: Reconstruct of
        # data shard 1 then Verify as two passes, against the one-pass store+verify kernel.  NOT
        # blb's RPC shape (the RPC passes exactly k survivors, so its Verify is vacuous):
        # `recovery_shapes` has that.
        rv_two = _ev_ms(lambda: (enc.ReconstructBatch(stripes, present), enc.VerifyBatch(stripes)),
                        max(3, a.steps // 4), stream, dev)
        rv_ok = bool(enc.ReconstructAndVerifyBatch(stripes, present).all())
        rv_one = _ev_ms(lambda: enc.ReconstructAndVerifyBatch(stripes, present), max(3, a.steps // 4), stream, dev)
        extra["reconstruct_and_verify_8_present_1_data_erasure"] = {
            "one_pass_ms": round(rv_one, 3), "two_pass_ms": round(rv_two, 3), "speedup": round(rv_two / rv_one, 3),
            "hbm_GBps_algorithmic_one_pass": round(algo_bytes / (rv_one * 1e-3) / 1e9, 1), "verify_ok": rv_ok}
        # CRC-32C of every parity shard in 65532-byte ChecksumFile blocks (§8f row 2).
        from blb_amd import checksum
        # Parity rows are strided (k+m)*S apart: checksum them as m strided batches of B rows.
        crc_evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        views = [stripes[:, k + j, :] for j in range(m)]
        for v in views:
            checksum.ChecksumBatch(v, checksum.CHECKSUM_BLOCK_DATA)
        torch.cuda.synchronize(dev)
        crc_evs[0].record(stream)
        for v in views:
            checksum.ChecksumBatch(v, checksum.CHECKSUM_BLOCK_DATA)
        crc_evs[1].record(stream)
        torch.cuda.synchronize(dev)
        crc_ms = crc_evs[0].elapsed_time(crc_evs[1])
        extra["crc32c_parity_blocks"] = {"GBps": round(B * m * S / (crc_ms * 1e-3) / 1e9, 1),
                                         "ms": round(crc_ms, 3), "bytes": B * m * S, "block": 65532}
        # The same two steps fused: parity checksummed in registers.  Default = the tile-grid
        # kernel (encode_crc_tile.hip); the persistent segment kernel (encode_crc.hip) is
        # timed beside it for the A/B (knob BLBRS_EC_PERSISTENT).
        def fused_ms(blk):
            enc.EncodeBatchCRC(stripes, blk)
            torch.cuda.synchronize(dev)
            f_evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                     for _ in range(max(3, a.steps // 4))]
            for s, e in f_evs:
                s.record(stream)
                enc.EncodeBatchCRC(stripes, blk)
                e.record(stream)
            torch.cuda.synchronize(dev)
            return float(np.mean([s.elapsed_time(e) for s, e in f_evs]))
        for blk_name, blk in (("blocks65532", checksum.CHECKSUM_BLOCK_DATA), ("whole_shard", 0)):
            f_ms = fused_ms(blk)
            with rs.tuning(BLBRS_EC_PERSISTENT=1):
                p_ms = fused_ms(blk)
            extra[f"encode_crc_fused_{blk_name}"] = {
                "ms_per_launch": round(f_ms, 3), "GiBps_data": round(B * k * S / GIB / (f_ms * 1e-3), 2),
                "ratio_to_encode": round(f_ms / launch_ms, 3),
                "hbm_GBps_algorithmic": round(algo_bytes / (f_ms * 1e-3) / 1e9, 1),
                "kernel": "encode_crc_tile_kernel + tile_combine_kernel",
                "persistent_segment_kernel_ms": round(p_ms, 3),
                "separate_encode_plus_crc_ms": round(launch_ms + crc_ms, 3) if blk else None}
        # PackTracts (§8f row 3): lay tracts of random length (64 KiB..8 MiB) at padToLength-
        # aligned offsets into the B*k data pieces, zero-filling holes and tails.  HBM bytes =
        # tract bytes read + piece bytes written.  Timed on two source sets over one layout
        # (tools/tract_layout.py): DISTINCT (every tract its own bytes -- the headline rate, every
        # byte read is a distinct HBM byte) and SHARED (windows of one 4 GiB pool, rounds 2-4;
        # overlapping windows can be served by L2 / MALL).
        from blb_amd import pack
        lay = TL.layout(B * k, S, np.random.default_rng(17))  # piece p = stripe p // k, shard p % k
        read_bytes = sum(ln for _, _, ln in lay)
        srcs = {"distinct": TL.distinct_sources(lay, dev, g, np.random.default_rng(18)),
                "shared": TL.shared_sources(lay, 4 << 30, dev, np.random.default_rng(19))}
        cols = [stripes[:, j, :] for j in range(k)]

        def pack_ms(pool, starts):
            ext = TL.extents(lay, pool, starts)
            per_col = [[(src, off, ln, p // k) for (src, off, ln, p) in ext if p % k == j] for j in range(k)]
            for j in range(k):
                pack.PackPieces(cols[j], S, per_col[j])
            torch.cuda.synchronize(dev)
            evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            torch.cuda._sleep(400_000_000)  # keeps the host-side extent checks outside the window
            evs[0].record(stream)
            for j in range(k):
                pack.PackPieces(cols[j], S, per_col[j])
            evs[1].record(stream)
            torch.cuda.synchronize(dev)
            return evs[0].elapsed_time(evs[1])

        def pack_encode_ms(pool, starts):
            # PackTracts fused with Encode (curator encPack -> encEncode in one pass): piece
            # b*k + j is data shard j of stripe b; parity encoded from registers.
            ext = TL.extents(lay, pool, starts)
            pack.PackEncode(enc, stripes, ext)
            torch.cuda.synchronize(dev)
            evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            torch.cuda._sleep(400_000_000)
            evs[0].record(stream)
            pack.PackEncode(enc, stripes, ext)
            evs[1].record(stream)
            torch.cuda.synchronize(dev)
            return evs[0].elapsed_time(evs[1]), bool(enc.VerifyBatch(stripes).all())

        pk = {name: pack_ms(*v) for name, v in srcs.items()}
        pe = {name: pack_encode_ms(*v) for name, v in srcs.items()}
        pk_bytes = read_bytes + B * k * S
        fe_bytes = read_bytes + B * (k + m) * S
        extra["pack_tracts"] = {"sources": "distinct", "ms": round(pk["distinct"], 3),
                                "hbm_GBps": round(pk_bytes / (pk["distinct"] * 1e-3) / 1e9, 1),
                                "frac_of_8TBps": round(pk_bytes / (pk["distinct"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "shared_pool_ms": round(pk["shared"], 3),
                                "pieces": B * k, "tracts": len(lay), "bytes_read": read_bytes, "bytes_written": B * k * S}
        extra["pack_encode_fused"] = {"sources": "distinct", "ms": round(pe["distinct"][0], 3),
                                      "hbm_GBps": round(fe_bytes / (pe["distinct"][0] * 1e-3) / 1e9, 1),
                                      "frac_of_8TBps": round(fe_bytes / (pe["distinct"][0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                      "shared_pool_ms": round(pe["shared"][0], 3),
                                      "separate_pack_plus_encode_ms": round(pk["distinct"] + launch_ms, 3),
                                      "bytes_read": read_bytes, "bytes_written": B * (k + m) * S,
                                      "verify_ok": pe["distinct"][1] and pe["shared"][1], "kernel": "pack_encode_kernel"}
        del srcs, cols

    if not a.no_extra and a.shard == TRACT:
        del stripes
        torch.cuda.empty_cache()
        extra.update(scale_extras(enc, k, m, S, world, rank, dev, dist))
        if world == 1:
            extra.update(wide_fused_extras(S, dev))
            extra["cold_class_rs83_b512"] = cold_class_extras(S, dev)
            extra["recovery_shapes"] = recovery_extras(S, dev)
            extra["host_calls_rs63_encode_4MiB_pool"] = host_call_extras(k, m, dev)
            extra["host_calls_rs63_encode_4MiB_rpc_pool_churn"] = rpc_pool_extras(k, m, dev)
    if rank == 0 and world == 1 and not a.no_extra:
        cpu = cpu_baseline(k, m, a.cpu_seconds)

    if rank == 0:
        traffic, traffic_src = pmc_traffic(k, m, B, S)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if a.total_batch else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded uniform random bytes, device-resident)",
            "config": {"workload": (f"RS({k},{m}) encode, batch={a.total_batch} stripes of {S // (1 << 20)} MiB "
                                    f"tracts split over {world} GPU(s)") if a.total_batch else
                                   f"RS({k},{m}) encode, batch={B} stripes of {S // (1 << 20)} MiB tracts per GPU",
                       "k": k, "m": m, "batch_per_gpu": B, "shard_bytes": S,
                       "parallelism": f"stripe-batch split x{world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "frac_vs_measured_copy": round(achieved_gbs / HBM_COPY_GBS, 4),
                         "kernel_ms": round(launch_ms, 3),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "traffic": traffic, "traffic_source": traffic_src},
            "cpu_baseline": cpu,
            "numa": numa,
            "verify_ok": ok,
        }
        if extra:
            line["extra"] = extra
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
