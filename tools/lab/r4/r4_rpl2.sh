#!/bin/bash
# Round-4 call: S3 with two rows per lane (AQC_S3_RPL 2, the in-tree default) -- the SVD and headline
# parity tests, then the lib A/B (phase probe + short bench) against the one-row layout (rpl1) and
# the two-row layout with the v / p prefetch (rpl2p1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rpl2_tests.log 2>&1 || exit $?
AB_STEPS=10 bash tools/ab_libs.sh cur rpl1 rpl2p1 cur
