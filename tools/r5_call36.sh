#!/bin/bash
# Round-5 GPU call 36: the two-round environment-chain test and the entanglement / z_all tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mps.py tests/test_gpu_ent.py -q --timeout 200 --timeout-method thread > gpurun_out/r5c36_tests.log 2>&1
exit $?
