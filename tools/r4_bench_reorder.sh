#!/bin/bash
# Round-4 call: the bench step with the chain's host preparation behind the sweep's kernels --
# two untraced runs, then the traced timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency --no-parity > gpurun_out/reo1.json 2> gpurun_out/reo1.err || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency --no-parity > gpurun_out/reo2.json 2> gpurun_out/reo2.err || exit $?
bash tools/r4_bench_timeline.sh
