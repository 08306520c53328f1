"""Summarise tools/crc_pmc.sh: per library and op, HBM read bytes (FETCH_SIZE, scaled by the same
process's 8 GiB copy) over the algorithmic bytes, and the kernel-trace time (mean of the REPS
warm launches).  usage: python tools/crc_pmc_summary.py OUTDIR variant ..."""
import csv
import glob
import json
import os
import sys

GIB = 1 << 30


def csv_in(d, kind):
    hits = glob.glob(os.path.join(d, "**", f"*{kind}.csv"), recursive=True)
    if not hits:
        raise SystemExit(f"no {kind}.csv under {d}")
    return list(csv.DictReader(open(hits[0])))


def meta(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no plan in {log}")


def main():
    out, variants = sys.argv[1], sys.argv[2:]
    res = {}
    for v in variants:
        plan = meta(os.path.join(out, v, "trace.log"))
        fetch = {}
        for r in csv_in(os.path.join(out, v, "fetch"), "counter_collection"):
            e = fetch.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0])
            e[1] += float(r["Counter_Value"])
        fetch = [v_ for _, v_ in sorted(fetch.items())]
        copy = max((x for x in fetch if "crc" not in x[0]), key=lambda x: x[1])
        scale = 8 * GIB / (copy[1] * 1024.0)
        crc_f = [x[1] * 1024.0 * scale for x in fetch if "crc_stream_kernel" in x[0]]
        trace = sorted(csv_in(os.path.join(out, v, "trace"), "kernel_trace"), key=lambda r: int(r["Dispatch_Id"]))
        crc_t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace
                 if "crc_stream_kernel" in r["Kernel_Name"]]
        ops, pos = {}, 0
        for o in plan["plan"]:
            n = o["launches"]
            f, t = crc_f[pos + 1:pos + n], crc_t[pos + 1:pos + n]
            pos += n
            rd = sum(f) / len(f)
            ms = sum(t) / len(t)
            ops[o["label"]] = {"hbm_read_bytes": round(rd), "algorithmic_bytes": o["algorithmic_bytes"],
                               "read_over_algorithmic": round(rd / o["algorithmic_bytes"], 5),
                               "trace_ms": round(ms, 4), "GBps": round(o["algorithmic_bytes"] / ms / 1e6, 1)}
        res[v] = {"lib_sha256": plan["lib_sha256"], "fetch_size_scale": round(scale, 4), "ops": ops}
    json.dump(res, open(os.path.join(out, "crc_pmc.json"), "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
