"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel with VGPRs,
AGPRs, spills, LDS and occupancy.  Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 |
python scripts/kernel_resources.py [name-filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" ")[0] + ("_spill" if "Spill" in k else "")] = v
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    d = d.split("(")[0]
    if flt and flt not in d:
        continue
    print(f"{d:60s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} vspill={r.get('VGPRs_spill')} "
          f"sspill={r.get('SGPRs_spill')} occ={r.get('Occupancy')} lds={r.get('LDS')}")
