#!/bin/bash
# round 6: S3 without per-column clock reads (default) vs with them (AQC_S3_TICKS=1, + range ticks):
# interleaved bench A/B, then the tick build's phase probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for t in cur ticks cur ticks; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 bench.py $B >> gpurun_out/r6c40_bench_$t.json 2>> gpurun_out/r6c40_bench_$t.err || exit $?
done
AQC_LIB=$PWD/adaptaqc_amd/libaqchip_ticks.so timeout -k 10 300 python3 tools/gram_phase_compile.py > gpurun_out/r6c40_phases_ticks.json 2> gpurun_out/r6c40_phases.err || exit $?
