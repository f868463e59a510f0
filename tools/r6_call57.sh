#!/bin/bash
# round 6 final tree: smoke() and the default bench line (the driver's round-end commands)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6c57_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c57_bench.json 2> gpurun_out/r6c57_bench.err || exit $?
