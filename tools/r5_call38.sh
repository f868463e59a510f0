#!/bin/bash
# Round-5 GPU call 38: the XCD grouping applied only from 8 jobs up (below 8, a job's blocks cycle
# over its share of the XCDs) and the pair-RDM chains on the grouped grid (libaqchip.so as built),
# against the library of the previous commit (libaqchip_head.so): parity of the kernels on the grid,
# ISL all-pair timing (1, 8, 32 states), single-state latency, unbounded-chi layers at 2 states.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py tests/test_gpu_gram_big.py tests/test_gpu_binding.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c38_tests.log 2>&1 || exit $?
for t in head cur head cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 tools/isl_timing.py >> gpurun_out/r5c38_isl_$t.txt 2>&1 || exit $?
  AQC_LIB=$lib timeout -k 10 200 python3 tools/latency_probe.py >> gpurun_out/r5c38_lat_$t.txt 2>&1 || exit $?
done
for t in head cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 300 python3 -u tools/unbounded_profile.py --states 2 > gpurun_out/r5c38_unb2_$t.json 2> gpurun_out/r5c38_unb2_$t.err || exit $?
done
exit 0
