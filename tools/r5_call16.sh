#!/bin/bash
# Round-5 GPU call 16 (release candidate after the config-5 two-stage exchange, S6 in 3M form and
# the capacity-64 environment chains): the whole -m gpu suite, smoke(), the bench under rocprofv3
# --kernel-trace --stats (kernel summary for profiles/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5c16_gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc" > gpurun_out/r5c16.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c16_smoke.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r5_prof_bench.json 2> gpurun_out/r5_prof_bench.err || exit $?
find gpurun_out/r5prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r5_bench_kernel_stats.csv \;
find gpurun_out/r5prof -name "*.db" -delete 2>/dev/null; find gpurun_out/r5prof -name "*kernel_trace.csv" -delete 2>/dev/null
exit $rc
