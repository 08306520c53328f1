"""Summarise tools/pmc_prod.sh (rocprofv3 --pmc passes over tools/pmc_prod.py, i.e. the
production libblbrs.so) into profiles/pmc_<tag>.json.

Calibration comes from the same process: torch's 8 GiB copy_ reads and writes exactly 8 GiB,
which gives the FETCH_SIZE and WRITE_SIZE scale factors (MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports 1/2 of wide streaming reads; measured, not assumed).  Per hot-path
op (tools/pmc_prod.py: one warm-up launch, then REPS launches): corrected HBM read / write
bytes next to the algorithmic bytes, the SQ counters and the kernel-trace duration, each the
mean over the REPS warm launches.  bench.py uses the encode's bytes
as roofline.traffic only while profiles/pmc_*.json's lib_sha256 equals the loaded library's.

usage: python tools/pmc_prod_summary.py OUTDIR TAG COMMIT
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys

GIB = 1 << 30


def rows(path):
    return list(csv.DictReader(open(path)))


def dispatches(d, counter=None):
    """[(dispatch_id, kernel_name, {counter: value})] in dispatch order."""
    out = {}
    for r in d:
        key = int(r["Dispatch_Id"])
        e = out.setdefault(key, [r["Kernel_Name"], {}])
        c = r["Counter_Name"]
        e[1][c] = e[1].get(c, 0.0) + float(r["Counter_Value"])
    return [(k, v[0], v[1]) for k, v in sorted(out.items())]


def csv_in(out, name, kind):
    hits = glob.glob(os.path.join(out, name, "**", f"*{kind}.csv"), recursive=True)
    if not hits:
        raise SystemExit(f"no {kind}.csv under {out}/{name}")
    return hits[0]


def main():
    out, tag, commit = sys.argv[1], sys.argv[2], sys.argv[3]
    meta = None
    for line in open(os.path.join(out, "trace.log")):
        if line.startswith("{"):
            meta = json.loads(line)
    fetch = dispatches(rows(csv_in(out, "fetch", "counter_collection")))
    write = dispatches(rows(csv_in(out, "write", "counter_collection")))
    sq = dispatches(rows(csv_in(out, "sq", "counter_collection")))
    sq2 = dispatches(rows(csv_in(out, "sq2", "counter_collection"))) if os.path.isdir(os.path.join(out, "sq2")) else None
    trace = sorted(rows(csv_in(out, "trace", "kernel_trace")), key=lambda r: int(r["Dispatch_Id"]))

    # calibration: the copy kernel that follows the fill (both 8 GiB)
    needles = {o["needle"] for o in meta["plan"]}
    big = [x for x in fetch if not any(n in x[1] for n in needles | {"tile_combine", "tile_chunk"})]
    copy_f = max(big, key=lambda x: x[2].get("FETCH_SIZE", 0.0))
    f_scale = 8 * GIB / (copy_f[2]["FETCH_SIZE"] * 1024.0)
    bigw = [x for x in write if x[0] == copy_f[0]]
    w_scale = 8 * GIB / (bigw[0][2]["WRITE_SIZE"] * 1024.0)

    def consume(seq, names, plan):
        """Walk the dispatches in order: each op takes the next `launches` whose kernel name
        contains its needle; the first is the warm-up.  Returns {label: [timed entries]}."""
        out, pos = {}, 0
        for o in plan:
            got = []
            while len(got) < o["launches"]:
                if pos >= len(seq):
                    raise SystemExit(f"ran out of dispatches at {o['label']}")
                if o["needle"] in names(seq[pos]):
                    got.append(seq[pos])
                pos += 1
            out[o["label"]] = got[1:]
        return out

    f_ops = consume(fetch, lambda x: x[1], meta["plan"])
    w_ops = consume(write, lambda x: x[1], meta["plan"])
    s_ops = consume(sq, lambda x: x[1], meta["plan"])
    s2_ops = consume(sq2, lambda x: x[1], meta["plan"]) if sq2 else {}
    t_ops = consume(trace, lambda r: r["Kernel_Name"], meta["plan"])

    def mean(vals):
        return sum(vals) / len(vals) if vals else None

    kernels = {}
    for o in meta["plan"]:
        if o.get("skip"):  # an untimed check launch between ops
            continue
        label, algo = o["label"], o["algorithmic_bytes"]
        rd = mean([x[2]["FETCH_SIZE"] for x in f_ops[label]]) * 1024.0 * f_scale
        wr = mean([x[2]["WRITE_SIZE"] for x in w_ops[label]]) * 1024.0 * w_scale
        counters = sorted({c for x in s_ops[label] for c in x[2]})
        sqv = {c: mean([x[2].get(c, 0.0) for x in s_ops[label]]) for c in counters}
        # the second SQ pass (wait and issue counters): its own SQ_WAVES / SQ_WAVE_CYCLES
        # normalise its counters, so they are kept apart under "sq2"
        sq2v = None
        if s2_ops:
            c2 = sorted({c for x in s2_ops[label] for c in x[2]})
            sq2v = {c: mean([x[2].get(c, 0.0) for x in s2_ops[label]]) for c in c2}
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in t_ops[label]]
        e = {"kernel": f_ops[label][0][1], "launches_averaged": len(ms),
             "hbm_read_bytes": round(rd), "hbm_write_bytes": round(wr),
             "hbm_bytes": round(rd + wr), "algorithmic_bytes": algo,
             "traffic_over_algorithmic": round((rd + wr) / algo, 6) if algo else None,
             "trace_ms": round(mean(ms), 4), "trace_ms_each": [round(x, 4) for x in ms], "sq": sqv}
        if sqv.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(sqv.get("SQ_LDS_BANK_CONFLICT", 0) / sqv["SQ_LDS_IDX_ACTIVE"], 4)
        if sqv.get("SQ_WAVES"):
            e["valu_insts_per_wave"] = round(sqv.get("SQ_INSTS_VALU", 0) / sqv["SQ_WAVES"], 1)
        if sq2v:
            e["sq2"] = sq2v
            if sq2v.get("SQ_WAVE_CYCLES"):
                wc = sq2v["SQ_WAVE_CYCLES"]
                e["wait_inst_any_frac_of_wave_cycles"] = round(sq2v.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
                e["wait_any_frac_of_wave_cycles"] = round(sq2v.get("SQ_WAIT_ANY", 0) / wc, 4)
                e["active_valu_frac_of_wave_cycles"] = round(sq2v.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4)
            if sq2v.get("SQ_WAVES"):
                e["salu_insts_per_wave"] = round(sq2v.get("SQ_INSTS_SALU", 0) / sq2v["SQ_WAVES"], 1)
                e["smem_insts_per_wave"] = round(sq2v.get("SQ_INSTS_SMEM", 0) / sq2v["SQ_WAVES"], 1)
        kernels[label] = e
    k, m, B, S = meta["k"], meta["m"], meta["batch"], meta["shard"]
    wide = meta.get("wide")
    res = {"tag": tag, "commit": commit, "lib_sha256": meta["lib_sha256"],
           "workload": {"k": k, "m": m, "batch": B, "shard": S, "wide": wide},
           "reps": meta.get("reps"), "rtc": meta.get("rtc"),
           "calibration": {"kernel": copy_f[1], "bytes_each_way": 8 * GIB,
                           "fetch_size_scale": round(f_scale, 4), "write_size_scale": round(w_scale, 4)},
           "hbm_bytes_per_launch": kernels["encode"]["hbm_bytes"],
           "kernels": kernels}
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", f"pmc_{tag}.json")
    json.dump(res, open(dst, "w"), indent=1)
    json.dump(res, open(os.path.join(out, f"pmc_{tag}.json"), "w"), indent=1)
    print(json.dumps({kk: {x: v[x] for x in ("hbm_bytes", "algorithmic_bytes", "traffic_over_algorithmic", "trace_ms")}
                      for kk, v in kernels.items()}))


if __name__ == "__main__":
    main()
