#!/bin/bash
# Round-4 call: S4 multisection shapes -- 4 lanes x 5-section x 12 rounds (in-tree default), 8 x 9 x 9
# (s4g8), 16 x 17 x 7 (s4g16): the SVD / headline parity tests with each, then the lib A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in s4g8 s4g16; do
  AQC_LIB=$PWD/adaptaqc_amd/libaqchip_$t.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s4_tests_$t.log 2>&1 || exit $?
done
AB_STEPS=10 bash tools/ab_libs.sh cur s4g8 s4g16 cur
