#!/bin/bash
# Round-4 call: amp 0 handed off by the final SV pass -- the SV tests, then config 2 twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sv.py tests/test_gpu_binding.py -x -q --timeout 200 --timeout-method thread > gpurun_out/amp0_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/amp0_c2a.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/amp0_c2b.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/sv_compiler_path.py 3 > gpurun_out/amp0_svpath.log 2>&1 || exit $?
