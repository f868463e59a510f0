#!/bin/bash
# Round-5 GPU call 39 (final library: pair-RDM chains grouped by state from 8 states up): the whole -m gpu suite, smoke(),
# config 5, the default bench line (with its single-evaluation latencies).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5c39_gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc" > gpurun_out/r5c39.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c39_smoke.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c39_c5.json 2> gpurun_out/r5c39_c5.err || exit $?
timeout -k 10 500 python3 bench.py > gpurun_out/r5c39_bench.json 2> gpurun_out/r5c39_bench.err || exit $?
exit $rc
