#!/bin/bash
# Config-5 A/B of the multi-workgroup Gram path (an environment switch per variant, e.g.
# AQC_GB_OVERLAP / AQC_GB_RPL) after the Gram-path tests.  Outputs under gpurun_out/.
# Usage (GPU box): bash tools/gb_ab.sh "VAR=a" "VAR=b" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rc=0; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -v --timeout 200 --timeout-method thread > gpurun_out/gb_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
i=0
for v in "$@"; do
  env $v timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/gb_ab_$i.json 2> gpurun_out/gb_ab_$i.err
  i=$((i+1))
done
