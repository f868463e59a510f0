#!/bin/bash
# Round-5 GPU call 2: the threshold-1e-8 parity tests and the SVD / MPS suites after the kept-count
# change, then the unbounded-workload profile and a short bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_threshold.py tests/test_gpu_headline.py tests/test_gpu_svd.py \
  tests/test_gpu_gram_big.py tests/test_gpu_mps.py tests/test_gpu_bigchi.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5c2_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c2_tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 tools/unbounded_profile.py > gpurun_out/r5_unbounded.json 2> gpurun_out/r5_unbounded.err || exit $?
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency > gpurun_out/r5c2_bench.json 2> gpurun_out/r5c2_bench.err || exit $?
exit $rc
