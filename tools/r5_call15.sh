#!/bin/bash
# Round-5 GPU call 15: S6 of the 2 chi = 128 Gram path with 3M complex products (three real MFMAs
# per complex k step in Y^H V, T (Y^H V) and V -= Y W2; S6 is matrix-core-bound: libaqchip_s6m3.so):
# SVD / chain parity, lone-SVD phase ticks, then interleaved bench repeats against the library as built;
# the capacity-64 environment chains with the hand-off poll kept clear of the operand prefetch
# (libaqchip_env4.so): parity, step phases, local-cost latency.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_s6m3.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py tests/test_gpu_mps.py \
  tests/test_gpu_threshold.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c15_s6m3_tests.log 2>&1
rc=$?
echo "s6m3 tests rc=$rc" > gpurun_out/r5c15.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AQC_LIB=$L/libaqchip_env4.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py::test_z_all_batch_split_environments_vs_oracle \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c15_env4_tests.log 2>&1
r=$?
echo "env4 tests rc=$r" >> gpurun_out/r5c15.rc
if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
AQC_LIB=$L/libaqchip_env4.so timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c15_env4_probe.json 2>&1 || exit $?
AQC_LIB=$L/libaqchip_env4.so timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
  -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c15_local_env4.log 2>&1
r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
if [ $rc -ne 0 ]; then exit $rc; fi
for t in cur s6m3; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/r5c15_probe_$t.txt 2>&1 || exit $?
done
AB_REPS=2 timeout -k 10 400 bash tools/ab_repeat.sh cur s6m3 || exit $?
exit 0
