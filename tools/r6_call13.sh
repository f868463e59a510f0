#!/bin/bash
# round 6: host profile and device timeline of a short compile after the evaluator changes; bench
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python3 -u tools/layer_cprofile.py > gpurun_out/r6c13_cprof.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6c13_tl -o run -- python3 tools/layer_profile.py --target graded --layers 6 --cpu-pairs 0 > gpurun_out/r6c13_tl.log 2>&1 || exit $?
python3 tools/timeline_gaps.py gpurun_out/r6c13_tl/run --match k_svd_gram > gpurun_out/r6c13_layer_gaps.json
timeout -k 10 400 python3 bench.py > gpurun_out/r6c13_bench.json 2> gpurun_out/r6c13_bench.err || exit $?
