"""Summarise tools/ab_repeat.sh output: per tag, the step time and k_chain time of every repeat."""
import glob
import json
import os
import re
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
rows = {}
for f in sorted(glob.glob(os.path.join(out, "abr_*_*.json"))):
    m = re.match(r"abr_(.+)_(\d+)\.json", os.path.basename(f))
    try:
        d = json.load(open(f))
    except (ValueError, OSError):
        continue
    rows.setdefault(m.group(1), []).append((d["ms_per_step"], d["breakdown_ms"]["mps_chain"]))
for t, v in rows.items():
    st = [a for a, _ in v]
    ch = [b for _, b in v]
    print(f"{t:10s} step {' '.join(f'{x:6.2f}' for x in st)}  mean {sum(st)/len(st):6.2f} | "
          f"chain {' '.join(f'{x:6.2f}' for x in ch)}  mean {sum(ch)/len(ch):6.2f}")
