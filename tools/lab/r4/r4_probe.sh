#!/bin/bash
# Phase probe of the chain(s) (+ optional tests).  PROBE_SIZES, PROBE_1024=1, PROBE_TESTS=<pytest -k expr>.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/probe_steps.txt
if [ -n "$PROBE_TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread -k "$PROBE_TESTS" > gpurun_out/probe_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" >> gpurun_out/probe_steps.txt
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python3 tools/chain256_probe.py 25 ${PROBE_SIZES:-32,512} > gpurun_out/probe256.jsonl 2> gpurun_out/probe256.err || exit $?
echo "probe256 rc=0" >> gpurun_out/probe_steps.txt
if [ -n "$PROBE_1024" ]; then
  AQC_CHAIN=1024 timeout -k 10 200 python3 tools/chain256_probe.py 25 ${PROBE_SIZES:-32,512} > gpurun_out/probe1024.jsonl 2> gpurun_out/probe1024.err || exit $?
fi
