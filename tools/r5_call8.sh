#!/bin/bash
# Round-5 GPU call 8: the library as built (S3 x3, the 2 chi = 128 certificate, the four-workgroup
# environment chains) through the MPS / SVD / threshold / unbounded / compiler / binding suites, with
# unbounded runs growing their capacity on demand (Python); then experiment builds: the SV tile pass
# with the next gate's matrix read during the current gate (svpf), the environment chains with
# 64-deep k tiles (envkt64); then the compile-layer profile on both targets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py tests/test_gpu_threshold.py \
  tests/test_gpu_mps.py tests/test_gpu_ent.py tests/test_gpu_bigchi.py tests/test_gpu_grad.py tests/test_gpu_compiler.py \
  tests/test_gpu_binding.py -q --timeout 300 --timeout-method thread > gpurun_out/r5c8_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > gpurun_out/r5c8_tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AQC_LIB=$L/libaqchip_svpf.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sv.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c8_sv_tests.log 2>&1
r=$?; echo "sv tests rc=$r" >> gpurun_out/r5c8_tests.rc
if [ $r -ne 0 ]; then exit $r; fi
for r in 1 2; do
  for t in cur svpf; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/r5c8_c2_${t}_$r.json 2> gpurun_out/r5c8_c2_${t}_$r.err || exit $?
  done
done
AQC_LIB=$L/libaqchip_envkt64.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_mps.py -x -q -k "z_all" \
  --timeout 200 --timeout-method thread > gpurun_out/r5c8_kt64_tests.log 2>&1
r=$?; echo "kt64 tests rc=$r" >> gpurun_out/r5c8_tests.rc
if [ $r -ne 0 ]; then exit $r; fi
AQC_LIB=$L/libaqchip_envkt64.so timeout -k 10 200 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
  -q -s --timeout 180 --timeout-method thread > gpurun_out/r5c8_local_envkt64.log 2>&1
r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
timeout -k 10 200 python3 -u tools/layer_profile.py --target graded > gpurun_out/r5_layer_graded_adaptive.json 2> gpurun_out/r5_layer_graded_adaptive.err || exit $?
timeout -k 10 300 python3 -u tools/layer_profile.py --layers 4 > gpurun_out/r5_layer_nearproduct_adaptive.json 2> gpurun_out/r5_layer_nearproduct_adaptive.err || exit $?
exit 0
