#!/bin/bash
# Round-4 call: S6's compact-WY factors precomputed during S5 by idle waves (in-tree default,
# AQC_S6_TPRE=1) against the in-loop zlarft (libaqchip_tpre0.so): parity, then the lib A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py tests/test_gpu_mps.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tpre_tests.log 2>&1 || exit $?
AB_STEPS=10 bash tools/ab_libs.sh cur tpre0
