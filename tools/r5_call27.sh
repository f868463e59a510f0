#!/bin/bash
# Round-5 GPU call 27 (release candidate after the XCD placements, the three-stream schedule and
# the 16-byte hand-off traffic): the whole -m gpu suite, smoke(), the default bench line, the bench's
# kernel summary, configs 2 / 4 / 5 without the trace, the local-cost latency.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5c27_gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc" > gpurun_out/r5c27.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c27_smoke.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py > gpurun_out/r5c27_bench.json 2> gpurun_out/r5c27_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r5c27_prof_bench.json 2> gpurun_out/r5c27_prof_bench.err || exit $?
db=$(find gpurun_out/r5prof -name "*.db" | head -1)
python3 tools/rocpd_stats.py "$db" > gpurun_out/r5c27_bench_kernel_stats.csv || exit $?
rm -rf gpurun_out/r5prof
timeout -k 10 400 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r5c27_configs.json 2> gpurun_out/r5c27_configs.err || exit $?
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
  -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c27_local.log 2>&1
exit $rc
