#!/bin/bash
# Round-5 GPU call 10: the tests the certificate fixes touch, then the round profile
# (tools/profile_round.sh: kernel-trace stats of the bench, the PMC passes, a full bench line, and
# configs 2 / 4 / 5 under the kernel trace).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mps.py tests/test_gpu_svd.py tests/test_gpu_threshold.py tests/test_gpu_headline.py \
  -q --timeout 300 --timeout-method thread > gpurun_out/r5c10_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c10.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUND=r5 SKIP_TESTS=1 bash tools/profile_round.sh || exit $?
exit $rc
