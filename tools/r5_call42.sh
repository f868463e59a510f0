#!/bin/bash
# Round-5 GPU call 42 (final library, with the transposed P_b closing traces): the whole -m gpu
# suite, smoke(), the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5c42_gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc" > gpurun_out/r5c42.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c42_smoke.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py > gpurun_out/r5c42_bench.json 2> gpurun_out/r5c42_bench.err || exit $?
exit $rc
