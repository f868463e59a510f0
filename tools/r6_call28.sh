#!/bin/bash
# round 6: kernel stats of a 7-layer paper-setting compile (layer_profile.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c28_kt -o run -- python3 tools/layer_profile.py --target graded --layers 7 --cpu-pairs 0 > gpurun_out/r6c28_layers.json 2> gpurun_out/r6c28_layers.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c28_kt/run_results.db > gpurun_out/r6c28_kernel_stats.csv; rm -rf gpurun_out/r6c28_kt
