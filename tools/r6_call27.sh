#!/bin/bash
# round 6: window kernel as two workgroups per state (parallel chains, coalesced right steps)
# costs, window jobs through pinned staging): the evaluator's GPU tests, then the layer profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_binding.py tests/test_gpu_compiler.py tests/test_gpu_zsum.py tests/test_gpu_threshold.py > gpurun_out/r6c27_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/layer_profile.py --target graded --layers 7 --cpu-pairs 0 > gpurun_out/r6c27_layers.json 2> gpurun_out/r6c27_layers.err || exit $?
