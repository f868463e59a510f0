#!/bin/bash
# One GPU call: the GPU test suite, then (unless it crashed / timed out) A/B of experiment builds.
# Test failures (rc 1) do not stop the A/B; a fault, abort or time limit does.
# Usage (GPU box): bash tools/gpu_round_call.sh <ab-tag> ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 bash tools/ab_libs.sh "$@" || exit $?
fi
exit $rc
