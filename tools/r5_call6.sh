#!/bin/bash
# Round-5 GPU call 6: S3 phase B on two waves handing p^H v over through the LDS (x = z - s v formed
# once per row; skip groups of two registers: the library as built) -- SVD / headline / threshold
# parity, phase probes, interleaved bench A/B against round 4's S3 (g4) and the same phase B with
# groups of four (x3g4); then one compile layer of the paper setting (tools/layer_profile.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py tests/test_gpu_threshold.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r5c6_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c6_tests.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for t in cur x3g4; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/r5c6_probe_$t.txt 2>&1 || exit $?
done
AB_REPS=2 timeout -k 10 400 bash tools/ab_repeat.sh cur g4 x3g4 || exit $?
timeout -k 10 500 python3 -u tools/layer_profile.py > gpurun_out/r5_layer.json 2> gpurun_out/r5_layer.err || exit $?
exit 0
