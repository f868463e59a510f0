"""Device-timeline gaps of one stream from a rocprofv3 CSV trace (--kernel-trace
--memory-copy-trace --output-format csv): where the GPU sits idle between a run's operations.

    python3 tools/timeline_gaps.py DIR/run [--match k_sv_tile_reg]

Every kernel and copy is an interval; consecutive intervals (sorted by start) leave a gap, which is
classified by the pair (previous op, next op) -- e.g. "copy D2H -> copy H2D" is the host's turn
between two evaluations (read-back, sync, planning the next one), "kernel -> kernel" the launch
gap.  Only the window from the first to the last op whose name contains --match is counted.
"""
import argparse
import collections
import csv
import json


def _rows(path):
    try:
        with open(path, newline="") as f:
            return list(csv.DictReader(f))
    except FileNotFoundError:
        return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--match", default="k_sv_tile_reg")
    args = ap.parse_args()
    ev = []
    for r in _rows(args.prefix + "_kernel_trace.csv"):
        name = r.get("Kernel_Name", "")
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", short))
    for r in _rows(args.prefix + "_memory_copy_trace.csv"):
        d = r.get("Direction", "copy")
        kind = "H2D" if "HOST_TO_DEVICE" in d.upper() or d.upper() == "H2D" else (
            "D2H" if "DEVICE_TO_HOST" in d.upper() or d.upper() == "D2H" else d)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", kind))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if args.match in e[3]]
    if not idx:
        raise SystemExit("no matching ops")
    ev = ev[idx[0]:idx[-1] + 1]
    busy = collections.Counter()
    gaps = collections.defaultdict(list)
    end = ev[0][0]
    prev = None
    for s, e, typ, name in ev:
        label = name if typ == "kernel" else "copy " + name
        busy[label] += e - s
        if prev is not None:
            gaps[(prev, label)].append(max(0, s - end))
        end = max(end, e)
        prev = label
    span = ev[-1][1] - ev[0][0]
    out = {"window_us": span / 1e3, "ops": len(ev),
           "busy_us": {k: round(v / 1e3, 1) for k, v in busy.most_common()},
           "idle_us": round((span - sum(busy.values())) / 1e3, 1),
           "gaps": sorted(({"between": f"{a} -> {b}", "n": len(v), "total_us": round(sum(v) / 1e3, 1),
                            "mean_us": round(sum(v) / len(v) / 1e3, 2)} for (a, b), v in gaps.items()),
                          key=lambda g: -g["total_us"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
