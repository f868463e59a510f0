#!/bin/bash
# Round-5 GPU call 25: the gradient sweep's grouped chains (k_sweep_chain8) with a state's groups on one XCD
# (libaqchip_swx.so): gradient parity, then interleaved bench repeats and config 4 against the
# library as built.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_swx.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_sweep_modes.py tests/test_gpu_headline.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c25_swx_tests.log 2>&1
rc=$?
echo "swx tests rc=$rc" > gpurun_out/r5c25.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur swx; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 4 > gpurun_out/r5c25_c4_${t}_$r.json 2> gpurun_out/r5c25_c4_${t}_$r.err || exit $?
  done
done
AB_REPS=2 timeout -k 10 400 bash tools/ab_repeat.sh cur swx || exit $?
exit 0
