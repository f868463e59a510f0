#!/bin/bash
# round 6: layer profile (graded target, like-for-like CPU column) and the bench after the windowed costs
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 500 python3 -u tools/layer_profile.py --target graded --cpu-budget 40 > gpurun_out/r6c20_layer_graded.json 2> gpurun_out/r6c20_layer_graded.err || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c20_bench.json 2> gpurun_out/r6c20_bench.err || exit $?
