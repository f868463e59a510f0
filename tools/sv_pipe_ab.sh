#!/bin/bash
# A/B of the SV path against a saved baseline build (adaptaqc_amd/libaqchip_base.so): SV GPU tests
# on the current build, then config 2 on both.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sv.py tests/test_gpu_compiler.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sv_tests.log 2>&1
timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_new.json 2> gpurun_out/sv_new.err
AQC_LIB=$PWD/adaptaqc_amd/libaqchip_base.so timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_base.json 2> gpurun_out/sv_base.err
timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_new2.json 2> gpurun_out/sv_new2.err
