"""blb's real recovery call shapes on device-resident 8 MiB stripes, every storage class.

* RPC shape (curator reconstructChunk -> tractserver rsEncodeOne with an indexMap,
  internal/curator/reconstruct.go:51-79, internal/tractserver/store.go:1062-1102): the
  tractserver reads exactly the first k good pieces in index order, every other slot is nil,
  so Reconstruct rebuilds ALL m absent slots -- the e bad pieces and the m - e good parity
  pieces that were not read -- and the Verify that follows has nothing left to compare.
  e = 1..m bad data pieces.
* Client shape (client/blb/reconstruct.go:137-173): the first k good replies, then
  ReconstructData rebuilds the missing DATA slots only: the target alone (every other data
  piece answered; rows = 1) up to m missing data slots (rows = m).

Each row and variant (tables / run-time network): ms per launch (HIP events,
interleaved reps in one process), algorithmic HBM bytes B * (k + rows) * S, the fraction of
8 TB/s, and bit-exactness (erased shards restored, VerifyBatch of the whole batch).  Run the access-pattern probe beside it:
tools/_build/mix_probe rpc.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

S = 8 << 20
PEAK = 8000.0

p = argparse.ArgumentParser()
p.add_argument("--classes", default="6,3,1024;8,3,768;10,3,640;12,5,480")
p.add_argument("--reps", type=int, default=3)
p.add_argument("--out", default="")
a = p.parse_args()
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)


def ev_ms(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    fn()
    e.record(stream)
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e)


def bad_sets(k, m):
    """e = 1..m bad data pieces spread evenly over the data slots (1, 1 + k/m, ...)."""
    spread = [1 + (i * k) // m for i in range(m)]
    return [spread[:e] for e in range(1, m + 1)]


results = []
for item in a.classes.split(";"):
    k, m, B = (int(x) for x in item.split(","))
    n = k + m
    st = torch.empty((B, n, S), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(97531 + k)
    st[:, :k].random_(0, 256, generator=g)
    enc = rs.New(k, m)
    enc.EncodeBatch(st)
    torch.cuda.synchronize(dev)
    rows = [("encode", None, None, m)]
    for bad in bad_sets(k, m):
        good = [i for i in range(n) if i not in bad]
        present = [i in good[:k] for i in range(n)]
        rows.append((f"rpc_{len(bad)}bad", present, False, m))
    # client: target 1; best case every other data piece answered first; worst case the m
    # parity pieces answered and m - 1 other data pieces did not.
    pres = [i != 1 and i <= k for i in range(n)]
    rows.append(("client_rows1", pres, True, 1))
    miss = bad_sets(k, m)[-1]  # m data slots, the target among them
    first_k = [j for j in range(n) if j not in miss][:k]
    pres_w = [i in first_k for i in range(n)]
    rows.append((f"client_rows{m}", pres_w, True, m))
    # Variants (library knobs, blbrs_set_tuning): decode rows on the v_perm tables, on the
    # run-time network with shared XOR terms, and without; the encode row on the compiled
    # network, the run-time network (BLBRS_RTC_ENCODE) and the tables.
    dec_variants = [("tables", {"BLBRS_RTC": 0}), ("net", {}), ("net_nocse", {"BLBRS_RTC_CSE": 0})]
    enc_variants = [("compiled", {}), ("rtc", {"BLBRS_RTC_ENCODE": 1}),
                    ("rtc_nocse", {"BLBRS_RTC_ENCODE": 1, "BLBRS_RTC_CSE": 0}), ("tables", {"BLBRS_BITSLICE": 0})]

    def call(present, data_only):
        if present is None:
            enc.EncodeBatch(st)
        else:
            enc.ReconstructBatch(st, present, data_only=data_only)

    ok = {}
    for name, present, data_only, nrows in rows:
        for vname, knobs in (enc_variants if present is None else dec_variants):
            with rs.tuning(**knobs):
                call(present, data_only)   # requests the network
                rs.rtc_wait()
                if present is None:
                    ok[(name, vname)] = bool(enc.VerifyBatch(st).all())
                    continue
                targets = [i for i in range(n) if not present[i] and (i < k or not data_only)]
                ref = {i: st[:, i].clone() for i in targets if i < k}
                for i in targets:
                    st[:, i].fill_(0xA5)
                call(present, data_only)
                torch.cuda.synchronize(dev)
                good = all(torch.equal(st[:, i], r) for i, r in ref.items())
                if not data_only:
                    good = good and bool(enc.VerifyBatch(st).all())
                ok[(name, vname)] = good
                del ref
    times = {}
    for _ in range(a.reps):
        for name, present, data_only, nrows in rows:
            for vname, knobs in (enc_variants if present is None else dec_variants):
                with rs.tuning(**knobs):
                    times.setdefault((name, vname), []).append(ev_ms(lambda: call(present, data_only)))
    for name, present, data_only, nrows in rows:
        nbytes = B * (k + nrows) * S
        r = {"class": f"RS({k},{m})", "B": B, "row": name, "rows": nrows,
             "present": None if present is None else [i for i in range(n) if present[i]],
             "algorithmic_bytes": nbytes}
        for vname, _ in (enc_variants if present is None else dec_variants):
            v = times[(name, vname)]
            ms = sorted(v)[len(v) // 2]
            gbs = nbytes / (ms * 1e-3) / 1e9
            r[vname] = {"ms": round(ms, 3), "ms_all": [round(x, 3) for x in v], "GBps": round(gbs, 1),
                        "frac_of_8TBps": round(gbs / PEAK, 4), "bit_exact": ok[(name, vname)]}
        results.append(r)
        print(json.dumps(r), flush=True)
    del st
    torch.cuda.empty_cache()
results.append({"rtc_stats": rs.rtc_stats(), "lib": rs.version()})
print(json.dumps(results[-1]))
if a.out:
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)
