#!/bin/bash
# Round-5 GPU call 22: k_env64 with a chain's four workgroups on one XCD (grid (chains rounded up to
# 8, 4): linear ids chain + 8m w, libaqchip_xcd.so) -- parity, step phases, local-cost latency against
# the library as built.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_xcd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_mps.py::test_z_all_batch_split_environments_vs_oracle \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c22_xcd_tests.log 2>&1
rc=$?
echo "xcd tests rc=$rc" > gpurun_out/r5c22.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for t in xcd cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 tools/env_probe.py 7 > gpurun_out/r5c22_probe_$t.json 2>&1 || exit $?
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c22_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit 0
