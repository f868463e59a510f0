#!/bin/bash
# Multi-workgroup Gram path (gram_big.hip): its GPU tests, the big-chi tests, then config 5 with the
# Gram path and with the block Jacobi alone (AQC_BIG_GRAM=0), with kernel stats of the first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# test failures (rc 1) do not stop the call; a crash, abort or time limit does
rc=0; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gram_big.py -v --timeout 120 --timeout-method thread > gpurun_out/gb_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
rc=0; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bigchi.py -v --timeout 200 --timeout-method thread > gpurun_out/gb_bigchi.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/gb5 -o run -- python3 tools/configs_bench.py --configs 5 > gpurun_out/gb_cfg5.json 2> gpurun_out/gb_cfg5.err
python3 tools/rocpd_stats.py gpurun_out/gb5/run_results.db > gpurun_out/gb_cfg5_stats.csv
rm -rf gpurun_out/gb5
AQC_BIG_GRAM=0 timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/bj_cfg5.json 2> gpurun_out/bj_cfg5.err
