#!/bin/bash
# Round-5 GPU call 37: the pair-RDM chains (k_rdm_chain) with a state's chains on one XCD
# (libaqchip_rdmx.so): entanglement parity, then the ISL all-pair timing against the library as built.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_rdmx.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_binding.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c37_rdmx_tests.log 2>&1
rc=$?
echo "rdmx tests rc=$rc" > gpurun_out/r5c37.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for t in cur rdmx cur rdmx; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 tools/isl_timing.py >> gpurun_out/r5c37_isl_$t.txt 2>&1 || exit $?
done
exit 0
