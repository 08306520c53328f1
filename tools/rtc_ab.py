"""A/B of recovery passes on the v_perm tables vs their run-time networks: blb's RPC
shape at RS(k,m) (each --patterns entry = the bad data pieces; the first k good pieces are read
and every absent slot rebuilt), B stripes of 8 MiB, every (pattern, variant) interleaved rep by
rep in ONE process on the same buffers -- placement of a 70 GB batch moves a launch by up to
8 % between processes, so only in-process ratios mean anything.  Variants (--variants, library
knobs via blbrs_set_tuning): tables, net (the shipped run-time network), net_cse (explicit
shared XOR temporaries), net_wpe4 (4 waves per SIMD requested); the encode on its compiled
network is timed beside them.  Prints one JSON line per (pattern, variant) and a summary."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=12)
p.add_argument("--m", type=int, default=5)
p.add_argument("--batch", type=int, default=480)
p.add_argument("--patterns", default="1;1,3,5,8,10")
p.add_argument("--reps", type=int, default=5)
p.add_argument("--variants", default="tables:BLBRS_RTC=0;net:;net_cse:BLBRS_RTC_CSE=1;net_wpe4:BLBRS_RTC_WPE=4",
               help="name:KNOB=v+KNOB=v;... (library knobs, blbrs_set_tuning)")
p.add_argument("--encode-variants", default="compiled:",
               help="the encode's variants, same syntax (e.g. rtc:BLBRS_RTC_ENCODE=1)")
a = p.parse_args()
k, m, B, S = a.k, a.m, a.batch, 8 << 20
n = k + m
dev = torch.device("cuda:0")
patterns = []
for item in a.patterns.split(";"):
    bad = [int(x) for x in item.split(",")]
    good = [i for i in range(n) if i not in bad]
    patterns.append((bad, [i in good[:k] for i in range(n)]))
def parse_variants(text):
    out = []
    for item in text.split(";"):
        name, _, env = item.partition(":")
        out.append((name, {kk: int(v) for kk, v in (kv.split("=", 1) for kv in env.split("+") if kv)}))
    return out


variants = parse_variants(a.variants)
enc_variants = parse_variants(a.encode_variants)
st = torch.empty((B, n, S), dtype=torch.uint8, device=dev)
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
enc.EncodeBatch(st)
rs.set_tuning("BLBRS_RTC", 2)  # compiled by the warm-up call
for _, present in patterns:
    for name, knobs in variants:
        with rs.tuning(**knobs):
            enc.ReconstructBatch(st, present)
for name, knobs in enc_variants:
    with rs.tuning(**knobs):
        enc.EncodeBatch(st)
ok = bool(enc.VerifyBatch(st).all())


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e), 3)


res = {}
for _ in range(a.reps):
    for pi, (_, present) in enumerate(patterns):
        for name, knobs in variants:
            with rs.tuning(**knobs):
                res.setdefault((pi, name), []).append(timed(lambda: enc.ReconstructBatch(st, present)))
    for name, knobs in enc_variants:
        with rs.tuning(**knobs):
            res.setdefault((-1, "encode_" + name), []).append(timed(lambda: enc.EncodeBatch(st)))
ok = ok and bool(enc.VerifyBatch(st).all())
summary = {}
for (pi, name), v in res.items():
    med = sorted(v)[len(v) // 2]
    bad = patterns[pi][0] if pi >= 0 else None
    print(json.dumps({"k": k, "m": m, "B": B, "bad": bad, "variant": name, "ms": v, "median": med,
                      "verify_ok": ok}), flush=True)
    summary[f"{bad}:{name}"] = med
for pi, (bad, _) in enumerate(patterns):
    t = summary[f"{bad}:tables"]
    summary[f"{bad}:net_over_tables"] = round(summary[f"{bad}:net"] / t, 4)
print(json.dumps({"summary": summary, "rtc": rs.rtc_stats()}))
