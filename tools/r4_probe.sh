#!/bin/bash
# Phase probe of both chains + the new binding tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_binding.py -x -v -s --timeout 200 --timeout-method thread -k rotoselect > gpurun_out/binding.log 2>&1
echo "binding rc=$?" > gpurun_out/probe_steps.txt
timeout -k 10 200 python3 tools/chain256_probe.py 25 32,256,512,1024 > gpurun_out/probe256.jsonl 2> gpurun_out/probe256.err || exit $?
AQC_CHAIN=1024 timeout -k 10 200 python3 tools/chain256_probe.py 25 32,256,1024 > gpurun_out/probe1024.jsonl 2> gpurun_out/probe1024.err || exit $?
