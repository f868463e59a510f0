#!/bin/bash
# Round-5 GPU call 41: the pair-RDM closing traces with P stored transposed (three of the four
# operands and E read along rows; k_rdm_ztrace both along rows) and DPP wave sums instead of the
# 256-wide LDS tree (libaqchip.so as built) against the previous commit (libaqchip_head.so):
# entanglement / z_all parity, then the ISL all-pair timing.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ent.py tests/test_gpu_binding.py tests/test_gpu_mps.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c41_tests.log 2>&1 || exit $?
for t in head cur head cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 tools/isl_timing.py >> gpurun_out/r5c41_isl_$t.txt 2>&1 || exit $?
done
exit 0
