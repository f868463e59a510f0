#!/bin/bash
# round 6: the batched overlap read-back carries the error flags (ring staging, no stream sync
# before its launch); async-flag tests, bench line, 11-layer profile (costs must be unchanged)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_async_flags.py tests/test_gpu_headline.py tests/test_gpu_zsum.py tests/test_gpu_binding.py tests/test_gpu_compiler.py tests/test_gpu_mps.py > gpurun_out/r6c50_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency > gpurun_out/r6c50_bench.json 2> gpurun_out/r6c50_bench.err || exit $?
timeout -k 10 600 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c50_layers.json 2> gpurun_out/r6c50_layers.err || exit $?
