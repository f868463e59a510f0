#!/bin/bash
# Round-4 GPU call: the GPU tests, then (unless they crashed) the round-3 teardown repro under
# rocprofv3 (config 5) and a bench line.  Each step has its own limit; a fault / abort / time limit
# ends the call.  Outputs under gpurun_out/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${TESTS:-} > gpurun_out/tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" > gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$CFG5" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg5prof -o run -- python3 tools/configs_bench.py --configs 5 > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
  rc=$?
  echo "cfg5 rocprof rc=$rc" >> gpurun_out/steps.txt
  rm -rf gpurun_out/cfg5prof/*/*.db 2>/dev/null
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  echo "bench rc=$rc" >> gpurun_out/steps.txt
  exit $rc
fi
