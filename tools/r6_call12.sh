#!/bin/bash
# round 6: the whole GPU suite, then the layer profile and its host profile
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r6c12_tests.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded --cpu-budget 40 > gpurun_out/r6c12_layer_graded.json 2> gpurun_out/r6c12_layer_graded.err || exit $?
