#!/bin/bash
# round 6 final library: configs 2/4/5 with kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c60_kcfg -o run -- python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r6c60_configs.json 2> gpurun_out/r6c60_configs.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c60_kcfg/run_results.db > gpurun_out/r6c60_configs_kernel_stats.csv && rm -rf gpurun_out/r6c60_kcfg || exit $?
timeout -k 10 300 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r6c60_configs_plain.json 2> gpurun_out/r6c60_configs_plain.err || exit $?
