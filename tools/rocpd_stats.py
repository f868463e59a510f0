"""Kernel-trace summary (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/<round>_kernel_stats.csv

ROCm 7's rocprofv3 writes a rocpd database by default; this prints the same columns as the
`kernel_stats.csv` of `--output-format csv` (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev) plus the launch shape of each kernel.
"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x * grid_y * grid_z, workgroup_x * workgroup_y * workgroup_z, vgpr_count, lds_size from kernels").fetchall()
    durs = defaultdict(list)
    shape = {}
    for name, dur, gx, wx, vg, lds in rows:
        durs[name].append(dur)
        shape[name] = (gx // max(wx, 1), wx, vg, lds)
    total = sum(sum(v) for v in durs.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev",
                "Workgroups", "WorkgroupSize", "VGPR", "LDS"])
    for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        n = len(v)
        mean = sum(v) / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        w.writerow([name, n, sum(v), round(mean, 3), round(100.0 * sum(v) / total, 2), min(v), max(v),
                    round(sd, 3), *shape[name]])


if __name__ == "__main__":
    main(sys.argv[1])
