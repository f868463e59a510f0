#!/bin/bash
# round 6 final library (ring-wide staging growth): the whole GPU suite, the default bench line,
# kernel-trace stats of the bench, the PMC passes of k_chain
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6c54_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r6c54_bench.json 2> gpurun_out/r6c54_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c54_kt -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r6c54_ktrace_bench.json 2> gpurun_out/r6c54_ktrace.err || exit $?
python3 tools/rocpd_stats.py gpurun_out/r6c54_kt/run_results.db > gpurun_out/r6c54_bench_kernel_stats.csv && rm -rf gpurun_out/r6c54_kt || exit $?
bash tools/pmc_bench.sh || exit $?
