#!/bin/bash
# Round-5 GPU call 7: the four-workgroup environment chains (k_env_split, libaqchip_envsplit.so):
# <Z> / pair-RDM parity against the oracle, then the MPS local-cost batch latency through the
# reference's CostMinimiser (tests/test_gpu_binding.py prints the per-gate times); structured SV gates.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_envsplit.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mps.py tests/test_gpu_ent.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c7_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c7_tests.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for t in envsplit cur; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c7_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
# config 2: structured SV gates (rotations 4 FMAs per amplitude, CX as register exchanges, no
# folding into a dense 4x4: libaqchip_svkind.so) -- SV parity, then an interleaved A/B
AQC_LIB=$L/libaqchip_svkind.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sv.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c7_sv_tests.log 2>&1
r=$?; echo "sv tests rc=$r" >> gpurun_out/r5c7_tests.rc
if [ $r -ne 0 ]; then exit $r; fi
for r in 1 2; do
  for t in cur svkind; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/r5c7_c2_${t}_$r.json 2> gpurun_out/r5c7_c2_${t}_$r.err || exit $?
  done
done
# S3 phase B's hand-off wait without s_sleep (nosleep) against the library as built
for t in cur nosleep; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/r5c7_probe_$t.txt 2>&1 || exit $?
done
AB_REPS=2 timeout -k 10 300 bash tools/ab_repeat.sh cur nosleep || exit $?
# one compile layer on a target with decaying Schmidt spectra (the near-product one is in r5_layer.json)
timeout -k 10 400 python3 -u tools/layer_profile.py --target graded > gpurun_out/r5_layer_graded.json 2> gpurun_out/r5_layer_graded.err || exit $?
exit 0
