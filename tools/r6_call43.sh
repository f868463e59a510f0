#!/bin/bash
# round 6: device timeline gaps of a 7-layer paper-setting compile on the current library, and the
# host profile of the same
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6c43_tl -o run -- python3 tools/layer_profile.py --target graded --layers 7 --cpu-pairs 0 > gpurun_out/r6c43_layers.json 2> gpurun_out/r6c43_layers.err || exit $?
python3 tools/timeline_gaps.py gpurun_out/r6c43_tl/run --match k_ > gpurun_out/r6c43_gaps.json
rm -rf gpurun_out/r6c43_tl
timeout -k 10 400 python3 -u tools/layer_cprofile.py > gpurun_out/r6c43_cprofile.txt 2> gpurun_out/r6c43_cprofile.err || exit $?
