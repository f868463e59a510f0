#!/bin/bash
# Round-5 GPU call 12: the whole -m gpu suite on the library as built (certificate at 2 chi = 128,
# the fused / lock-step test aware of it), smoke, and where the environment chains' steps go.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5c12_gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc" > gpurun_out/r5c12.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c12_smoke.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c12_env_probe.json 2>&1 || exit $?
# experiment build: 3M products in the narrow chain GEMMs, T in the LDS at chi = 64
export AQC_LIB=$PWD/adaptaqc_amd/libaqchip_env2.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py::test_z_all_batch_split_environments_vs_oracle -q --timeout 120 --timeout-method thread > gpurun_out/r5c12_env2_tests.log 2>&1
r=$?; echo "env2 tests rc=$r" >> gpurun_out/r5c12.rc; if [ $r -gt 1 ]; then exit $r; fi
timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c12_env2_probe.json 2>&1 || exit $?
unset AQC_LIB
L=$PWD/adaptaqc_amd
# (call 13: config-5 exchange changes, local-cost latency)
AQC_LIB=$L/libaqchip_gb1.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c13_gb1_tests.log 2>&1
rc=$?
echo "gb1 tests rc=$rc" >> gpurun_out/r5c12.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur gb1; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c13_c5_${t}_$r.json 2> gpurun_out/r5c13_c5_${t}_$r.err || exit $?
  done
done
for t in env2 cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c13_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit $rc
