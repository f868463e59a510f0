#!/bin/bash
# Round-5 GPU call 11: S3 phase B without a cross-wave exchange -- p^H v from row terms the column
# pass leaves in the LDS (x4): SVD / headline / threshold parity, phase probes, interleaved bench A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_x4.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py \
  tests/test_gpu_threshold.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c11_tests.log 2>&1
rc=$?
echo "x4 tests rc=$rc" > gpurun_out/r5c11.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for t in cur x4; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/r5c11_probe_$t.txt 2>&1 || exit $?
done
AB_REPS=2 timeout -k 10 300 bash tools/ab_repeat.sh cur x4 || exit $?
exit 0
