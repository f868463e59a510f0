#!/bin/bash
# Round-5 GPU call 13: config 5's exchange tridiagonalisation with wave 0 alone forming w, the new
# row, its norm and the next reflector after the reads (libaqchip_gb2.so: one barrier after the
# reads instead of three): gram_big parity, then an interleaved config-5 A/B with the phase ticks.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_gb2.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c13_gb2_tests.log 2>&1
rc=$?
echo "gb2 tests rc=$rc" > gpurun_out/r5c13.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur gb2; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c13_c5_${t}_$r.json 2> gpurun_out/r5c13_c5_${t}_$r.err || exit $?
  done
done
# (call 14: capacity-64 environment chains with resident operands)
AQC_LIB=$L/libaqchip_env3.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py::test_z_all_batch_split_environments_vs_oracle \
  "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c14_env3_tests.log 2>&1
rc=$?
echo "env3 tests rc=$rc" >> gpurun_out/r5c13.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AQC_LIB=$L/libaqchip_env3.so timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c14_env3_probe.json 2>&1 || exit $?
for t in env3 cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c14_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit 0
