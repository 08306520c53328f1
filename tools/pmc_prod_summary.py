"""Summarise tools/pmc_prod.sh (rocprofv3 --pmc passes over tools/pmc_prod.py, i.e. the
production libblbrs.so) into profiles/pmc_<tag>.json.

Calibration comes from the same process: torch's 8 GiB copy_ reads and writes exactly 8 GiB,
which gives the FETCH_SIZE and WRITE_SIZE scale factors (MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports 1/2 of wide streaming reads; measured, not assumed).  Per hot-path
dispatch: corrected HBM read / write bytes next to the algorithmic bytes, the SQ counters of
the same dispatch, and the kernel-trace average duration.  bench.py uses the encode's bytes
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


def pick(ds, needle, nth=0):
    hits = [x for x in ds if needle in x[1]]
    if len(hits) <= nth:
        raise SystemExit(f"no dispatch #{nth} matching {needle!r}")
    return hits[nth]


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
    trace = rows(csv_in(out, "trace", "kernel_trace"))
    k, m, B, S = meta["k"], meta["m"], meta["batch"], meta["shard"]

    # calibration: the copy kernel that follows the fill (both 8 GiB)
    big = [x for x in fetch if not any(n in x[1] for n in ("rs_code", "encode_crc", "crc_stream", "pack_kernel"))]
    copy_f = max(big, key=lambda x: x[2].get("FETCH_SIZE", 0.0))
    f_scale = 8 * GIB / (copy_f[2]["FETCH_SIZE"] * 1024.0)
    bigw = [x for x in write if x[0] == copy_f[0]]
    w_scale = 8 * GIB / (bigw[0][2]["WRITE_SIZE"] * 1024.0)

    def durations(needle, nth=0):
        ts = [r for r in trace if needle in r["Kernel_Name"]]
        if len(ts) <= nth:
            return None
        r = ts[nth]
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # ms

    kernels = {}
    spec = [("encode", "rs_code_kernel", 0, B * (k + m) * S),
            ("reconstruct_data1", "rs_code_kernel", 1, B * (k + 1) * S),
            ("verify", "rs_code_kernel", 2, B * (k + m) * S),
            ("encode_crc_65532", "encode_crc_tile_kernel", 0, B * (k + m) * S),
            ("encode_crc_combine", "tile_combine_kernel", 0, None),
            ("crc32c_65532", "crc_stream_kernel", 0, B * S)]
    if meta.get("pack"):
        spec.append(("pack_tracts", "pack_kernel", 0, meta["pack"]["bytes_read"] + meta["pack"]["bytes_written"]))
    wide = meta.get("wide")
    if wide:  # RS(12,5) on the compiled network: dispatches after the RS(6,3) ones
        wb = wide["batch"] * (wide["k"] + wide["m"]) * S
        spec += [("encode_rs12_5_network", "rs_code_kernel", 3, wb),
                 ("encode_crc_rs12_5_network", "encode_crc_tile_kernel", 1, wb),
                 ("verify_rs12_5_network", "rs_code_kernel", 4, wb)]
    for label, needle, nth, algo in spec:
        f = pick(fetch, needle, nth)
        w = pick(write, needle, nth)
        s = pick(sq, needle, nth)
        rd = f[2]["FETCH_SIZE"] * 1024.0 * f_scale
        wr = w[2]["WRITE_SIZE"] * 1024.0 * w_scale
        e = {"kernel": f[1], "hbm_read_bytes": round(rd), "hbm_write_bytes": round(wr),
             "hbm_bytes": round(rd + wr), "algorithmic_bytes": algo,
             "traffic_over_algorithmic": round((rd + wr) / algo, 6) if algo else None,
             "trace_ms": durations(needle, nth), "sq": s[2]}
        sqv = s[2]
        if sqv.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(sqv.get("SQ_LDS_BANK_CONFLICT", 0) / sqv["SQ_LDS_IDX_ACTIVE"], 4)
        kernels[label] = e
    res = {"tag": tag, "commit": commit, "lib_sha256": meta["lib_sha256"],
           "workload": {"k": k, "m": m, "batch": B, "shard": S, "wide": wide},
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
