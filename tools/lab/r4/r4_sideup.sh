#!/bin/bash
# Round-4 call: SV plans of the later batches uploaded on a side stream (default) vs on the state's
# stream (AQC_SV_SIDE_UPLOAD=0): the SV tests, then config 2 alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sv.py tests/test_gpu_binding.py tests/test_gpu_compiler.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sideup_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sideup_on_$i.log 2>&1 || exit $?
  AQC_SV_SIDE_UPLOAD=0 timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sideup_off_$i.log 2>&1 || exit $?
done
