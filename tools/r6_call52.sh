#!/bin/bash
# round 6: ring-wide staging growth -- the MPS-side GPU tests, then the default bench line twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_mps.py tests/test_gpu_async_flags.py tests/test_gpu_zsum.py tests/test_gpu_headline.py \
  > gpurun_out/r6c52_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c52_bench_a.json 2> gpurun_out/r6c52_bench_a.err || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c52_bench_b.json 2> gpurun_out/r6c52_bench_b.err || exit $?
