"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel.
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [filter]"""
import re
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"vgpr {r.get('VGPRs','-'):>4} agpr {r.get('AGPRs','-'):>3} vspill {r.get('VGPRs Spill','-'):>3} "
              f"sspill {r.get('SGPRs Spill','-'):>3} occ {r.get('Occupancy [waves/SIMD]','-'):>2}  {r['name'][:90]}")
