"""Summarise rocprofv3 --pmc databases: per kernel, mean counter value per dispatch and duration.

    python tools/pmc_summary.py <dir-or-db> [<dir-or-db> ...] [--filter substring]

Reads the rocpd SQLite output of ROCm 7 rocprofv3 (the `counters_collection` view when present,
else rocpd_pmc_event joined with rocpd_info_pmc and the kernel dispatches).
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def rows_of(db):
    c = sqlite3.connect(db)
    names = {r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")}
    if "counters_collection" in names:
        cols = [d[1] for d in c.execute("pragma table_info(counters_collection)")]
        kcol = "kernel_name" if "kernel_name" in cols else "name"
        vcol = "value" if "value" in cols else "counter_value"
        q = f"select dispatch_id, {kcol}, counter_name, {vcol}, duration from counters_collection"
        return c.execute(q).fetchall()
    raise SystemExit(f"{db}: no counters_collection view; tables: {sorted(names)}")


def main(args):
    flt = ""
    if "--filter" in args:
        i = args.index("--filter")
        flt = args[i + 1]
        args = args[:i] + args[i + 2:]
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    dur = defaultdict(dict)
    for a in args:
        dbs = glob.glob(os.path.join(a, "**", "*.db"), recursive=True) if os.path.isdir(a) else [a]
        for db in dbs:
            for d, k, cn, v, du in rows_of(db):
                if flt and flt not in k:
                    continue
                agg[k][cn] += v
                disp[k][cn].add((db, d))
                dur[k][(db, d)] = du
    for k in sorted(agg, key=lambda k: -sum(dur[k].values())):
        nd = len(dur[k])
        print(f"== {k[:110]}\n   dispatches={nd} mean_dur_us={sum(dur[k].values()) / max(nd, 1) / 1e3:.1f}")
        for cn, v in sorted(agg[k].items()):
            print(f"   {cn:28s} {v / max(len(disp[k][cn]), 1):18.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
