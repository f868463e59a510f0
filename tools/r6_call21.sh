#!/bin/bash
# round 6: window kernels v2 (vector steps, chains meeting in the middle): parity, per-gate timing, layer profile
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_zsum.py > gpurun_out/r6c21_zsum.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_binding.py > gpurun_out/r6c21_bind.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded --cpu-budget 20 > gpurun_out/r6c21_layer_graded.json 2> gpurun_out/r6c21_layer_graded.err || exit $?
