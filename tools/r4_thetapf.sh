#!/bin/bash
# Round-4 call: k_chain's theta with the next m chunk prefetched into registers (in-tree default,
# AQC_THETA_PF=1) against loads at the top of each step (libaqchip_thpf0.so): parity, then lib A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_headline.py tests/test_gpu_mps.py -x -q --timeout 200 --timeout-method thread > gpurun_out/thpf_tests.log 2>&1 || exit $?
AB_STEPS=10 bash tools/ab_libs.sh cur thpf0 cur thpf0
