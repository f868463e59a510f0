#!/bin/bash
# A/B of experiment builds of libaqchip (in-tree adaptaqc_amd/libaqchip_<tag>.so): for each tag the
# Gram-path phase probe (tools/svd32_probe.py) and a short bench line.  Every step has its own time
# limit; the chain stops at the first failure.
# Usage (GPU box): bash tools/ab_libs.sh <tag> [<tag> ...]     ("cur" = adaptaqc_amd/libaqchip.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps ${AB_STEPS:-10} --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for t in "$@"; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/ab_probe_$t.txt 2>&1
  AQC_LIB=$lib timeout -k 10 200 python3 bench.py $B > gpurun_out/ab_bench_$t.json 2> gpurun_out/ab_bench_$t.err
done
