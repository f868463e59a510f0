#!/bin/bash
# round 6: capacity-64 window steps (whole tile per thread, next tile prefetched): parity, layer kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_zsum.py tests/test_gpu_binding.py tests/test_gpu_compiler.py tests/test_gpu_threshold.py > gpurun_out/r6c29_tests.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c29_kt -o run -- python3 tools/layer_profile.py --target graded --layers 7 --cpu-pairs 0 > gpurun_out/r6c29_layers_kt.json 2> gpurun_out/r6c29_layers_kt.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c29_kt/run_results.db > gpurun_out/r6c29_kernel_stats.csv; rm -rf gpurun_out/r6c29_kt
timeout -k 10 400 python3 -u tools/layer_profile.py --target graded --layers 7 --cpu-pairs 0 > gpurun_out/r6c29_layers.json 2> gpurun_out/r6c29_layers.err || exit $?
