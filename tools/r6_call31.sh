#!/bin/bash
# round 6: the sweep's psi from the backend's cached base; compiler/gradient GPU tests, 11-layer
# paper-setting profile (Rotosolve at layer 10) and its kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime_order.py tests/test_gpu_compiler.py tests/test_gpu_grad.py tests/test_gpu_binding.py > gpurun_out/r6c31_tests.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c31_layers.json 2> gpurun_out/r6c31_layers.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c31_kt -o run -- python3 tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c31_layers_kt.json 2> gpurun_out/r6c31_layers_kt.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c31_kt/run_results.db > gpurun_out/r6c31_kernel_stats.csv; rm -rf gpurun_out/r6c31_kt
