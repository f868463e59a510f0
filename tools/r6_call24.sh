#!/bin/bash
# round 6: CPU-leg settle A/B, PMC passes of the bench (r6 traffic / executed work), configs 2/4/5 with kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--no-parity --no-latency"
timeout -k 10 300 python3 bench.py --no-cpu-baseline $B > gpurun_out/r6c24_nocpu.json 2> gpurun_out/r6c24_nocpu.err || exit $?
timeout -k 10 300 python3 bench.py $B > gpurun_out/r6c24_cpu0.json 2> gpurun_out/r6c24_cpu0.err || exit $?
timeout -k 10 300 python3 bench.py --cpu-settle 8 $B > gpurun_out/r6c24_cpu8.json 2> gpurun_out/r6c24_cpu8.err || exit $?
timeout -k 10 900 bash tools/pmc_bench.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c24_kcfg -o run -- python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r6c24_configs.json 2> gpurun_out/r6c24_configs.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c24_kcfg/run_results.db > gpurun_out/r6c24_configs_kernel_stats.csv; rm -rf gpurun_out/r6c24_kcfg
