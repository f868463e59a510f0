#!/bin/bash
# Interleaved repeats of the short bench line for experiment builds (noise estimate for an A/B):
# for r in 1..R, for each tag: bench.py with AQC_LIB=<tag's library> -> gpurun_out/abr_<tag>_<r>.json
# Usage (GPU box): AB_REPS=3 bash tools/ab_repeat.sh <tag> [<tag> ...]   ("cur" = libaqchip.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for r in $(seq 1 "${AB_REPS:-3}"); do
  for t in "$@"; do
    if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 bench.py $B > gpurun_out/abr_${t}_$r.json 2> gpurun_out/abr_${t}_$r.err
  done
done
