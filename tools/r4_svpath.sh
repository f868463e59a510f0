#!/bin/bash
# Round-4 call: config 2 through the backend path (conversion memo vs fresh), plus the SV / binding tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sv.py tests/test_gpu_binding.py tests/test_gpu_compiler.py -x -q --timeout 200 --timeout-method thread > gpurun_out/svpath_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/sv_compiler_path.py 3 > gpurun_out/svpath.log 2>&1 || exit $?
