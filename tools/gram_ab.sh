#!/bin/bash
# A/B of the Gram SVD against a saved baseline build (adaptaqc_amd/libaqchip_base.so): SVD/MPS/headline
# GPU tests on the current build, the phase ticks and accuracy probe, and a short bench on both.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_mps.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/ab_probe_new.txt 2>&1
AQC_LIB=$PWD/adaptaqc_amd/libaqchip_base.so timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/ab_probe_base.txt 2>&1
B="--steps 10 --warmup 3 --no-cpu-baseline --no-latency"
timeout -k 10 300 python3 bench.py $B > gpurun_out/ab_bench_new.json 2> gpurun_out/ab_bench_new.err
AQC_LIB=$PWD/adaptaqc_amd/libaqchip_base.so timeout -k 10 300 python3 bench.py $B > gpurun_out/ab_bench_base.json 2> gpurun_out/ab_bench_base.err
