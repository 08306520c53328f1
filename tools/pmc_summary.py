"""Summarise rocprofv3 --pmc runs of `tools/_build/tune pmc` (tools/pmc_run.sh) into
profiles/pmc_<tag>.json, which bench.py reads for roofline.traffic.

Calibration is measured in the same run, not assumed:
  * pattern_kernel<9,0,...> reads exactly B*9*S bytes -> FETCH_SIZE scale factor
    (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE reports 1/2 of wide streaming reads);
  * pattern_kernel<1,1,...> writes exactly B*S bytes -> WRITE_SIZE scale factor.
FETCH_SIZE / WRITE_SIZE are in KiB.  The corrected HBM bytes of the production kernel
rs_code_kernel<6,3,0,0,4,3> are reported per launch next to its algorithmic bytes.

usage: python tools/pmc_summary.py gpurun_out/pmc r01_rs63_encode
"""
from __future__ import annotations

import csv
import json
import os
import sys

S = 8 << 20
B = 1024


def load(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
    return out


def find(d, needle):
    hits = [v for (_, name), v in sorted(d.items()) if needle in name]
    if len(hits) != 1:
        raise SystemExit(f"expected one dispatch matching {needle!r}, got {len(hits)}")
    return hits[0]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    fetch = load(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    read_known = B * 9 * S
    write_known = B * S
    f_read = find(fetch, "pattern_kernel<9, 0") * 1024.0
    w_copy = find(write, "pattern_kernel<1, 1") * 1024.0
    f_scale = read_known / f_read
    w_scale = write_known / w_copy
    rs_fetch = find(fetch, "rs_code_kernel<6, 3, 0, 0") * 1024.0 * f_scale
    rs_write = find(write, "rs_code_kernel<6, 3, 0, 0") * 1024.0 * w_scale
    algo_read, algo_write = B * 6 * S, B * 3 * S
    out = {
        "tag": tag,
        "kernel": "rs_code_kernel<6, 3, 0, 0, 4, 3> (RS(6,3) encode, strided, U=4, nt)",
        "workload": {"k": 6, "m": 3, "batch": B, "shard": S},
        "fetch_scale_measured": round(f_scale, 6),
        "write_scale_measured": round(w_scale, 6),
        "hbm_read_bytes_per_launch": int(rs_fetch),
        "hbm_write_bytes_per_launch": int(rs_write),
        "hbm_bytes_per_launch": int(rs_fetch + rs_write),
        "algorithmic_bytes_per_launch": algo_read + algo_write,
        "traffic_over_algorithmic": round((rs_fetch + rs_write) / (algo_read + algo_write), 6),
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of tools/_build/tune pmc",
    }
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                       f"pmc_{tag}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
