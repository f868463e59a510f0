#!/bin/bash
# Round-4 closing check on the final tree: the whole GPU suite and a default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/close_suite.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/close_bench.json 2> gpurun_out/close_bench.err || exit $?
timeout -k 10 300 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/close_configs.log 2>&1 || exit $?
