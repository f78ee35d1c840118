#!/usr/bin/env python3
"""Print the kernel sequence of one step from a rocprofv3 kernel_trace.csv (the step is located by
a kernel that runs once per step, e.g. the AdamW update), with per-kernel µs and grid sizes."""
import csv
import sys

path, marker = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "adamw_kernel"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[which - 1] + 1, idx[which] + 1
tot = 0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
    print(f"{d:8.1f}  wg={g:6d}  {r['Kernel_Name'][:110]}")
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"sum {tot:.1f} us, span {span:.1f} us, {b - a} kernels")
