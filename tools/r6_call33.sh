#!/bin/bash
# round 6: gram_big Gram-Schmidt block CGS2 with the second pass only when needed: parity suites, then the 11-layer
# paper-setting profile (Rotosolve at layer 10) with kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gram_big.py tests/test_gpu_threshold.py tests/test_gpu_bigchi.py tests/test_gpu_svd.py > gpurun_out/r6c33_tests.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c33_layers.json 2> gpurun_out/r6c33_layers.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c33_kt -o run -- python3 tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c33_layers_kt.json 2> gpurun_out/r6c33_layers_kt.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c33_kt/run_results.db > gpurun_out/r6c33_kernel_stats.csv; rm -rf gpurun_out/r6c33_kt
