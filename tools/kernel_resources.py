"""Per-kernel register budget of a built HIP object: VGPR / AGPR / SGPR counts, spills, LDS.

Extracts the gfx950 code object from a hipcc .o (its .hip_fatbin bundle), reads the AMDGPU
metadata notes and prints one JSON object {kernel: {...}}.  Given two objects it prints only the
kernels whose budget differs -- the check that a change to rs_code.hpp left the coding kernels'
register allocation (and so their occupancy) alone.

usage: python tools/kernel_resources.py OBJ.o [OTHER.o]
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def resources(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = {}
    for ent in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        def f(key):
            m = re.search(rf"\.{key}:\s+(\S+)", ent)
            return m.group(1) if m else None
        out[f("name")] = {"vgpr": int(f("vgpr_count")), "agpr": int(ent.split("\n", 1)[0].strip(": ") or 0),
                          "sgpr": int(f("sgpr_count")), "vgpr_spill": int(f("vgpr_spill_count")),
                          "sgpr_spill": int(f("sgpr_spill_count")), "lds": int(f("group_segment_fixed_size")),
                          "kernarg": int(f("kernarg_segment_size")),
                          "scratch": int(f("private_segment_fixed_size"))}
    return out


def main():
    a = resources(sys.argv[1])
    if len(sys.argv) < 3:
        print(json.dumps(a, indent=1, sort_keys=True))
        return
    b = resources(sys.argv[2])
    diff = {k: {"a": a.get(k), "b": b.get(k)} for k in sorted(set(a) | set(b))
            if {x: y for x, y in (a.get(k) or {}).items() if x != "kernarg"} !=
            {x: y for x, y in (b.get(k) or {}).items() if x != "kernarg"}}
    print(json.dumps({"kernels_a": len(a), "kernels_b": len(b), "differ": diff}, indent=1))


if __name__ == "__main__":
    main()
