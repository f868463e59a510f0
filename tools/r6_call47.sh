#!/bin/bash
# round 6: the default bench line with Python GC off in the timed steps (default) vs on
# (AQC_BENCH_GC=1), interleaved, twice each -- per-step times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in on off on off; do
  if [ "$t" = on ]; then g=1; else g=0; fi
  AQC_BENCH_GC=$g timeout -k 10 400 python3 bench.py --no-latency >> gpurun_out/r6c47_bench_gc$t.json 2>> gpurun_out/r6c47_bench_gc$t.err || exit $?
done
