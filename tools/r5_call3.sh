#!/bin/bash
# Round-5 GPU call 3: the SVD / threshold / MPS suites with the wide-K Gram path, the unbounded
# profile again, and an interleaved bench A/B against the previous build (libaqchip_prev.so).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_threshold.py tests/test_gpu_headline.py \
  tests/test_gpu_mps.py tests/test_gpu_bigchi.py tests/test_gpu_gram_big.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5c3_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c3_tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 tools/unbounded_profile.py > gpurun_out/r5c3_unbounded.json 2> gpurun_out/r5c3_unbounded.err || exit $?
AB_REPS=3 timeout -k 10 700 bash tools/ab_repeat.sh cur prev || exit $?
exit $rc
