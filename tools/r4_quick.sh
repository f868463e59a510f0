#!/bin/bash
# Round-4 quick GPU call: selected GPU tests (QUICK_TESTS, a pytest -k expression), then optional
# config runs (QUICK_CONFIGS=2,5 ...) and the single-state latency probe (QUICK_LATENCY=1).
# Every step has its own limit; any failure ends the call.  Outputs under gpurun_out/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/quick_steps.txt
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/quick_steps.txt
  return $rc
}
if [ -n "$QUICK_TESTS" ]; then
  step qtests 500 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$QUICK_TESTS" || exit $?
fi
if [ -n "$QUICK_CONFIGS" ]; then
  step qconfigs 400 python3 tools/configs_bench.py --configs "$QUICK_CONFIGS" || exit $?
fi
if [ -n "$QUICK_LATENCY" ]; then
  step qlatency 300 python3 tools/latency_probe.py || exit $?
fi
