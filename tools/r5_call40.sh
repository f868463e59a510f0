#!/bin/bash
# Round-5 GPU call 40 (final library): the bench's kernel summary under the kernel trace and
# BASELINE configs 2 / 4 / 5 without it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r5c40_prof_bench.json 2> gpurun_out/r5c40_prof_bench.err || exit $?
db=$(find gpurun_out/r5prof -name "*.db" | head -1)
python3 tools/rocpd_stats.py "$db" > gpurun_out/r5c40_bench_kernel_stats.csv || exit $?
rm -rf gpurun_out/r5prof
timeout -k 10 400 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r5c40_configs.json 2> gpurun_out/r5c40_configs.err || exit $?
exit 0
