#!/bin/bash
# round 6: S3 without per-column clock reads (cur) vs the committed S3 with them (orig): interleaved bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for t in orig cur orig cur orig cur; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 bench.py $B >> gpurun_out/r6c41_bench_$t.json 2>> gpurun_out/r6c41_bench_$t.err || exit $?
done
