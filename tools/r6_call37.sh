#!/bin/bash
# round 6: host-side phase times of every batched apply in a 7-layer paper-setting compile
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AQC_HOST_TIMING=1 timeout -k 10 300 python3 -u tools/layer_profile.py --target graded --layers 7 --cpu-pairs 0 > gpurun_out/r6c37_layers.json 2> gpurun_out/r6c37_host.err
python3 - <<'PY' > gpurun_out/r6c37_host_summary.txt
import re, collections
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for line in open("gpurun_out/r6c37_host.err"):
    m = re.match(r"\[aqc host\] apply (\d+) states: validate ([\d.]+) ms, schedule ([\d.]+) ms, jobs\+launch ([\d.]+) ms", line)
    if m:
        a = agg[int(m.group(1))]
        a[0] += 1; a[1] += float(m.group(2)); a[2] += float(m.group(3)); a[3] += float(m.group(4))
for ns, (n, v, s, j) in sorted(agg.items()):
    print(f"states={ns:5d} calls={n:6d} validate={v:8.2f} ms schedule={s:8.2f} ms jobs+launch={j:8.2f} ms  per call: {(v+s+j)/n:.3f} ms")
PY
