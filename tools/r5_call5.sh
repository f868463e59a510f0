#!/bin/bash
# Round-5 GPU call 5: S3 variants -- the dead-column skip per register (AQC_S3_GROUP 1, the current
# library, vs 4 = round 4's groups) and x = z - s v formed once in phase B (xpre: phase B unrolled over
# its two rows; xpre2: the same with skip groups of two registers -- no register moves per column): SVD / headline parity of cur and xpre, phase probes, interleaved bench A/B;
# config 2 with one tile workgroup per CU forced (svpad).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5c5_tests_cur.log 2>&1
rc=$?
echo "cur tests rc=$rc" > gpurun_out/r5c5_tests.rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AQC_LIB=$L/libaqchip_xpre.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r5c5_tests_xpre.log 2>&1
rc2=$?
echo "xpre tests rc=$rc2" >> gpurun_out/r5c5_tests.rc
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
for t in cur xpre xpre2; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/r5c5_probe_$t.txt 2>&1 || exit $?
done
AB_REPS=2 timeout -k 10 500 bash tools/ab_repeat.sh cur g4 xpre xpre2 || exit $?
# config 2: k_sv_tile_reg with 64 KB of extra dynamic LDS (one workgroup per CU forced) vs as built
for r in 1 2; do
  for t in cur svpad; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/r5c5_c2_${t}_$r.json 2> gpurun_out/r5c5_c2_${t}_$r.err || exit $?
  done
done
# the MPS local-cost batch (z_all_batch's environment chains with k-tile prefetch and coalesced
# tile loads, envpf) against the library as built: the binding test prints the per-gate latencies
for t in cur envpf; do
  if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_binding.py::test_reference_rotoselect_batched_mps_local_and_softened" \
    -q -s --timeout 240 --timeout-method thread > gpurun_out/r5c5_local_$t.log 2>&1
  r=$?; if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
exit $rc
