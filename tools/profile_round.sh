#!/bin/bash
# Round profiling on the GPU box: the GPU tests, rocprofv3 kernel-trace stats of a bench run, the
# PMC passes (tools/pmc_bench.sh), a full bench line, and the other BASELINE configs with their
# kernel stats.  Each step has its own time limit; the chain stops at the first failure.  Outputs
# under gpurun_out/ (copy the ones to keep into profiles/).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/ktrace_bench.json 2> gpurun_out/ktrace.err
python3 tools/rocpd_stats.py gpurun_out/ktrace/run_results.db > gpurun_out/kernel_stats.csv
rm -rf gpurun_out/ktrace
timeout -k 10 900 bash tools/pmc_bench.sh
# the full bench line below reads this round's PMC results (copied back from gpurun_out/ locally)
cp gpurun_out/exec_k_chain.json profiles/${ROUND:-r3}_exec_k_chain.json
cp gpurun_out/traffic.json profiles/${ROUND:-r3}_traffic.json
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
if [ -z "$SKIP_CONFIGS" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kcfg -o run -- python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/configs.json 2> gpurun_out/configs.err
  python3 tools/rocpd_stats.py gpurun_out/kcfg/run_results.db > gpurun_out/configs_kernel_stats.csv
  rm -rf gpurun_out/kcfg
fi
