#!/bin/bash
# Config-5 A/B of the multi-workgroup Gram path's tridiagonalisation layouts (AQC_GB_RPL = 2 / 1) with
# the phase ticks, after the Gram-path tests.  Outputs under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rc=0; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gram_big.py -v --timeout 120 --timeout-method thread > gpurun_out/gb_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for R in 2 1; do
  AQC_GB_RPL=$R timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/gb_cfg5_rpl$R.json 2> gpurun_out/gb_cfg5_rpl$R.err
done
