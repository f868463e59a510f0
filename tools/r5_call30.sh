#!/bin/bash
# Round-5 GPU call 30: the unbounded-capacity workload and one compile layer of the paper setting
# (graded target) re-measured on the round's final library.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/unbounded_profile.py > gpurun_out/r5c30_unbounded.json 2> gpurun_out/r5c30_unbounded.err || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded > gpurun_out/r5c30_layer_graded.json 2> gpurun_out/r5c30_layer_graded.err || exit $?
exit 0
