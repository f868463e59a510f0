#!/bin/bash
# round 6: window kernel without scratch (generic steps); window parity tests, then the final
# 11-layer paper-setting profile with the like-for-like CPU column
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_zsum.py tests/test_gpu_binding.py > gpurun_out/r6c38_tests.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/layer_profile.py --target graded --cpu-budget 20 > gpurun_out/r6c38_layer_graded.json 2> gpurun_out/r6c38_layer_graded.err || exit $?
