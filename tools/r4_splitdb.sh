#!/bin/bash
# Round-4 call: the standalone split GEMM with double-buffered k tiles (default) against single
# (libaqchip_sdb0.so): MPS / gram_big / headline tests, then config 5 and single-state latency A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mps.py tests/test_gpu_gram_big.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sdb_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/sdb_c5_on_$i.log 2>&1 || exit $?
  AQC_LIB=$PWD/adaptaqc_amd/libaqchip_sdb0.so timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/sdb_c5_off_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/latency_probe.py > gpurun_out/sdb_lat_on.log 2>&1 || exit $?
AQC_LIB=$PWD/adaptaqc_amd/libaqchip_sdb0.so timeout -k 10 300 python3 tools/latency_probe.py > gpurun_out/sdb_lat_off.log 2>&1 || exit $?
