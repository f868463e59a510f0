#!/bin/bash
# Round-5 GPU call 32: k_gb_eig with 16 lanes per eigenvalue, 7 rounds of 17-section (libaqchip_eig16.so)
# -- parity, then config 5 interleaved.
#
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_eig16.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py tests/test_gpu_mps.py tests/test_gpu_svd.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c32_eig16_tests.log 2>&1
rc=$?
echo "eig16 tests rc=$rc" > gpurun_out/r5c32.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur eig16; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c32_c5_${t}_$r.json 2> gpurun_out/r5c32_c5_${t}_$r.err || exit $?
  done
done
exit 0
