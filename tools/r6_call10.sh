#!/bin/bash
# round 6: capacity-1024 tests (goldens), two-rank tests, the graded-target layer profile with the
# like-for-like CPU column, and a kernel + copy trace of a short compile
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_bigchi.py -m gpu -k "above_512 or gram_side" > gpurun_out/r6c10_bigchi.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_comm.py -m gpu > gpurun_out/r6c10_comm.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded --cpu-budget 40 > gpurun_out/r6c10_layer_graded.json 2> gpurun_out/r6c10_layer_graded.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6c10_tl -o run -- python3 tools/layer_profile.py --target graded --layers 3 --cpu-pairs 0 > gpurun_out/r6c10_tl.log 2>&1 || exit $?
python3 tools/timeline_gaps.py gpurun_out/r6c10_tl/run --match k_ > gpurun_out/r6c10_layer_gaps.json
