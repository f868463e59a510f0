#!/bin/bash
# Round-5 GPU call 24: gram_big parity on the three-stream schedule and the BASELINE configs 2 / 4 / 5
# without the kernel trace (the round's config numbers); the capacity-64 chains' hand-off traffic as
# 16-byte sc1 buffer loads / stores (libaqchip_b16.so): parity, step phases, local-cost latency.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c24_gb_tests.log 2>&1
rc=$?
echo "gb tests rc=$rc" > gpurun_out/r5c24.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r5c24_configs.json 2> gpurun_out/r5c24_configs.err || exit $?
AQC_LIB=$L/libaqchip_b16.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py::test_z_all_batch_split_environments_vs_oracle \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c24_b16_tests.log 2>&1
r=$?
echo "b16 tests rc=$r" >> gpurun_out/r5c24.rc
if [ $r -ne 0 ]; then exit $r; fi
for t in b16 cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c24_probe_$t.json 2>&1 || exit $?
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c24_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit $rc
