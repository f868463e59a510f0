#!/bin/bash
# Round-5 GPU call 1: the GPU suite after the cleanup, the default bench line, then an interleaved
# A/B of the S6 precompute mapping (AQC_S6_TPRE_SKIP0) with its phase probe.  Each step has its own
# time limit; a fault, abort or time limit ends the call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5_tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || exit $?
for t in cur skip0; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/r5_probe_$t.txt 2>&1 || exit $?
done
AB_REPS=3 timeout -k 10 700 bash tools/ab_repeat.sh cur skip0 || exit $?
exit $rc
