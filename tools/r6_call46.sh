#!/bin/bash
# round 6 final library: the whole GPU suite, the default bench line, kernel-trace stats of the
# bench, configs 2/4/5 with kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6c46_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c46_bench.json 2> gpurun_out/r6c46_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c46_kt -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r6c46_ktrace_bench.json 2> gpurun_out/r6c46_ktrace.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c46_kt/run_results.db > gpurun_out/r6c46_bench_kernel_stats.csv; rm -rf gpurun_out/r6c46_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c46_kcfg -o run -- python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r6c46_configs.json 2> gpurun_out/r6c46_configs.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c46_kcfg/run_results.db > gpurun_out/r6c46_configs_kernel_stats.csv; rm -rf gpurun_out/r6c46_kcfg
