#!/bin/bash
# round 6: the default bench line (the driver's command), twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r6c51_bench_a.json 2> gpurun_out/r6c51_bench_a.err || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c51_bench_b.json 2> gpurun_out/r6c51_bench_b.err || exit $?
