#!/bin/bash
# Round-5 GPU call 4: batched local / softened costs, the rank-deficiency certificate, then the
# unbounded profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_threshold.py tests/test_gpu_binding.py tests/test_gpu_compiler.py \
  tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r5c4_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c4_tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 tools/unbounded_profile.py > gpurun_out/r5c4_unbounded.json 2> gpurun_out/r5c4_unbounded.err || exit $?
exit $rc
