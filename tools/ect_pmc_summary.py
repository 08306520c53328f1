"""Per-kernel SQ counters of tools/ect_pmc.sh's passes (rs_code_kernel vs the fused tile
kernel): python tools/ect_pmc_summary.py OUTDIR -> OUTDIR/summary.json."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
res = {}
for name in ("sq1", "sq2"):
    for path in glob.glob(os.path.join(out, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            kn = r["Kernel_Name"]
            key = "encode" if "rs_code_kernel" in kn else "tile" if "encode_crc_tile_kernel" in kn else None
            if key is None:
                continue
            d = res.setdefault(key, {"kernel": kn[:120], "vgpr": r.get("Arch_VGPR_Count"),
                                     "lds": r.get("LDS_Block_Size"), "scratch": r.get("Scratch_Size")})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for path in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        for key, needle in (("encode", "rs_code_kernel"), ("tile", "encode_crc_tile_kernel")):
            if needle in r["Name"] and key in res:
                res[key]["avg_ns"] = float(r["AverageNs"])
for d in res.values():
    w = d.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if c in d:
                d[c + "_frac"] = round(d[c] / w, 4)
    if d.get("SQ_WAVES"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM"):
            if c in d:
                d[c + "_per_wave"] = round(d[c] / d["SQ_WAVES"], 1)
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
