"""Summarise a rocprofv3 --pmc database: per kernel (name filter) the mean of each counter over its
dispatches (counter values summed over the per-SE / per-XCD instances first).
Usage: python scripts/pmc_db.py <run_results.db> [name-substring ...]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
flts = sys.argv[2:]
c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)  # never creates a file
rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration, lds_block_size, vgpr_count, "
                 "accum_vgpr_count, scratch_size from counters_collection")
per = defaultdict(lambda: defaultdict(float))
meta = {}
for did, name, cn, v, dur, lds, vg, ag, scr in rows:
    short = name.split("(")[0]
    if flts and not any(f in short for f in flts):
        continue
    per[(short, did)][cn] += v
    meta[(short, did)] = (dur, lds, vg, ag, scr)
agg = defaultdict(lambda: defaultdict(list))
for (short, did), cnts in per.items():
    for cn, v in cnts.items():
        agg[short][cn].append(v)
    agg[short]["_dur_ns"].append(meta[(short, did)][0])
for short, cnts in agg.items():
    print(short)
    for cn in sorted(cnts):
        vals = cnts[cn]
        print(f"   {cn:28s} {sum(vals) / len(vals):16.1f}   (n={len(vals)})")
