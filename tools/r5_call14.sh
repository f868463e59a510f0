#!/bin/bash
# Round-5 GPU call 14: (1) 2 chi = 512 exchange in two stages (16 then 4 workgroups per job; a
# round's second stage beside the next round's first) in the library as built: gram_big parity,
# then config 5 interleaved against one stage (AQC_GB_STAGES=1, same library);
# (2) the capacity-64 environment chains with resident operands (k_env64, libaqchip_env3.so):
# parity, step phases, local-cost latency.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c14_gb_tests.log 2>&1
rc=$?
echo "gb tests rc=$rc" > gpurun_out/r5c14.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -eq 0 ]; then
  for r in 1 2; do
    for t in 2 1; do
      AQC_GB_STAGES=$t timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c14_c5_s${t}_$r.json 2> gpurun_out/r5c14_c5_s${t}_$r.err || exit $?
    done
  done
fi
AQC_LIB=$L/libaqchip_env3.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py::test_z_all_batch_split_environments_vs_oracle \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c14_env3_tests.log 2>&1
r=$?
echo "env3 tests rc=$r" >> gpurun_out/r5c14.rc
if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
AQC_LIB=$L/libaqchip_env3.so timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c14_env3_probe.json 2>&1 || exit $?
for t in env3 cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c14_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit $rc
