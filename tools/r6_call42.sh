#!/bin/bash
# round 6: S3's last 32 columns in wave 0 alone (AQC_S3_TAIL): Gram-path parity suites, then an
# interleaved bench A/B against the same build without the tail
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_svd.py tests/test_gpu_headline.py tests/test_gpu_mps.py tests/test_gpu_threshold.py > gpurun_out/r6c42_tests.log 2>&1 || exit $?
B="--steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for t in notail cur notail cur; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 bench.py $B >> gpurun_out/r6c42_bench_$t.json 2>> gpurun_out/r6c42_bench_$t.err || exit $?
done
