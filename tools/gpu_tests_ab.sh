#!/bin/bash
# One GPU call: selected GPU test files (TESTS, default the whole gpu suite), then -- unless the
# tests crashed or timed out -- the A/B of experiment builds named on the command line.
# Usage (GPU box): TESTS="tests/test_gpu_svd.py ..." bash tools/gpu_tests_ab.sh <tag> ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TESTS:-tests}
timeout -k 10 800 python3 -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 bash tools/ab_libs.sh "$@" || exit $?
fi
exit $rc
