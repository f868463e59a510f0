#!/bin/bash
# Round-5 GPU call 18: 3M complex products in block_cgemm for the matrix-core-bound callers --
# k_gb_gram (libaqchip_m3g.so) and also the standalone split GEMM (libaqchip_m3gs.so): parity, then
# config 5 interleaved against the library as built; th3 adds theta as one 3M GEMM on the matrix cores
# (k_theta_mm + k_theta_gate) for capacities >= 128.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_th3.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py tests/test_gpu_mps.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c18_th3_tests.log 2>&1
rc=$?
echo "th3 tests rc=$rc" > gpurun_out/r5c18.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur m3g m3gs th3; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c18_c5_${t}_$r.json 2> gpurun_out/r5c18_c5_${t}_$r.err || exit $?
  done
done
exit 0
