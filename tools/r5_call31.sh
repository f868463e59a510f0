#!/bin/bash
# Round-5 GPU call 31: k_theta with 32 x 32 tiles and 2 x 2 positions per thread (half the LDS
# operand reads per FMA; libaqchip_th32.so): the whole -m gpu suite on it, then config 5 interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_th32.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5c31_th32_tests.log 2>&1
rc=$?
echo "th32 tests rc=$rc" > gpurun_out/r5c31.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur th32; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c31_c5_${t}_$r.json 2> gpurun_out/r5c31_c5_${t}_$r.err || exit $?
  done
done
exit 0
