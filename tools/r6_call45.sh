#!/bin/bash
# round 6: one circuit conversion per Rotoselect visit (patched in place)
# evaluator / compiler tests, then the 11-layer paper-setting profile (capacity growth exercised)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zsum.py tests/test_gpu_binding.py tests/test_gpu_compiler.py tests/test_gpu_threshold.py tests/test_host.py > gpurun_out/r6c45_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c45_layers.json 2> gpurun_out/r6c45_layers.err || exit $?
