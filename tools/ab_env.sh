#!/bin/bash
# Interleaved repeats of the short bench line under different environment settings (same build):
# for r in 1..R, for each "tag=VAR=value" argument: bench.py with that variable set ->
# gpurun_out/abr_<tag>_<r>.json (tools/ab_repeat_summary.py reads them).
# Usage (GPU box): AB_REPS=3 bash tools/ab_env.sh t8=AQC_HOST_THREADS=8 t1=AQC_HOST_THREADS=1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for r in $(seq 1 "${AB_REPS:-3}"); do
  for a in "$@"; do
    t=${a%%=*}
    kv=${a#*=}
    env "$kv" timeout -k 10 200 python3 bench.py $B > gpurun_out/abr_${t}_$r.json 2> gpurun_out/abr_${t}_$r.err
  done
done
