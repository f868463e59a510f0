#!/bin/bash
# Round profiling on the GPU box: rocprofv3 kernel-trace stats of a bench run, the PMC passes
# (tools/pmc_bench.sh), then a full bench line.  Each step has its own time limit; the chain
# stops at the first failure.  Outputs under gpurun_out/ (copy the ones to keep into profiles/).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/ktrace_bench.json 2> gpurun_out/ktrace.err
find gpurun_out/ktrace -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
rm -rf gpurun_out/ktrace/*/*.db 2>/dev/null || true
timeout -k 10 900 bash tools/pmc_bench.sh
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
