#!/bin/bash
# round 6: k_gb_inv with a 32-row prefetch -- gram_big tests, the 11-layer
# compile (costs must be unchanged), and its kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py > gpurun_out/r6c59_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c59_layers.json 2> gpurun_out/r6c59_layers.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c59_kt -o run -- python3 tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c59_layers_kt.json 2> gpurun_out/r6c59_layers_kt.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c59_kt/run_results.db > gpurun_out/r6c59_layer_kernel_stats.csv && rm -rf gpurun_out/r6c59_kt || exit $?
