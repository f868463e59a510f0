"""Summarise a rocprofv3 PMC database: per kernel, mean counters per dispatch and duration."""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration, vgpr_count, lds_block_size, grid_size, workgroup_size from counters_collection").fetchall()
agg = defaultdict(lambda: defaultdict(float))
meta = {}
disp = defaultdict(set)
for d, k, cn, v, dur, vg, lds, gs, ws in rows:
    if flt and flt not in k:
        continue
    agg[k][cn] += v
    disp[k].add(d)
    meta[k] = (vg, lds, gs, ws)
    agg[k]["__dur"] += 0
durs = defaultdict(float)
for d, k, dur in c.execute("select distinct dispatch_id, kernel_name, duration from counters_collection"):
    if flt and flt not in k:
        continue
    durs[k] += dur
for k in agg:
    n = len(disp[k])
    print(f"== {k[:90]}  dispatches={n} mean_dur_us={durs[k] / n / 1e3:.1f} vgpr={meta[k][0]} lds={meta[k][1]} grid={meta[k][2]} wg={meta[k][3]}")
    for cn, v in sorted(agg[k].items()):
        if cn.startswith("__"):
            continue
        print(f"   {cn:28s} {v / n:16.1f}")
