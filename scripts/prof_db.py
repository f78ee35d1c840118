#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (``--kernel-trace`` output ``*_results.db``).

  prof_db.py <db> stats [steps] [top]       per-kernel totals (ms/step, %, calls, avg us, VGPR/LDS)
  prof_db.py <db> step [marker] [which]     kernel sequence of one step (start offset, duration; located
                                            by a kernel that runs once per step, default the AdamW update)
"""
import sqlite3
import sys


def rows(db):
    c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)  # never creates a file
    q = ("select name, start, end, grid_x*grid_y*grid_z, workgroup_x*workgroup_y*workgroup_z, "
         "lds_size, vgpr_count, accum_vgpr_count from kernels order by start")
    return list(c.execute(q))


def stats(db, steps=1.0, top=40):
    agg = {}
    for name, s, e, grid, wg, lds, vg, ag in rows(db):
        a = agg.setdefault(name, [0, 0, grid // max(1, wg), lds, vg, ag])
        a[0] += e - s
        a[1] += 1
    tot = sum(a[0] for a in agg.values())
    print(f"total GPU kernel time {tot / 1e6:.2f} ms  ({tot / 1e6 / steps:.3f} ms per step over {steps:g} steps)")
    print(f"{'ms/step':>8} {'%':>6} {'calls':>6} {'avg_us':>8} {'wgs':>7} {'lds':>6} {'vgpr':>5}  kernel")
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{a[0] / 1e6 / steps:8.3f} {100 * a[0] / tot:6.2f} {a[1]:6d} {a[0] / a[1] / 1e3:8.1f} {a[2]:7d} "
              f"{a[3]:6d} {a[4]:5d}  {name[:110]}")


def step(db, marker="adamw_kernel", which=-2):
    r = rows(db)
    idx = [i for i, x in enumerate(r) if marker in x[0]]
    a, b = idx[which - 1] + 1, idx[which] + 1
    tot = 0
    t0 = r[a][1]
    print(f"{'start_us':>9} {'dur_us':>8}")
    for name, s, e, grid, wg, lds, vg, ag in r[a:b]:
        tot += e - s
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  wg={grid // max(1, wg):6d}  {name[:110]}")
    print(f"sum {tot / 1e3:.1f} us, span {(r[b - 1][2] - r[a][1]) / 1e3:.1f} us, {b - a} kernels")


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1].startswith("-"):
        print(__doc__)
        sys.exit(0)
    db, mode = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "stats"
    if mode == "stats":
        stats(db, float(sys.argv[3]) if len(sys.argv) > 3 else 1.0, int(sys.argv[4]) if len(sys.argv) > 4 else 40)
    else:
        step(db, sys.argv[3] if len(sys.argv) > 3 else "adamw_kernel", int(sys.argv[4]) if len(sys.argv) > 4 else -2)
