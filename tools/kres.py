"""Per-kernel VGPR / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
output on stdin: python tools/kres.py [name-regex] < remarks.txt"""
import re
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, r in rows.items():
    if pat and not pat.search(name):
        continue
    print(f"{name[:90]:90s} vgpr={r.get('VGPRs')} sgpr_spill={r.get('SGPRs Spill')} "
          f"vgpr_spill={r.get('VGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")
