#!/bin/bash
# Round-5 GPU call 17: k_gb_back with 3M complex products (libaqchip_gbb.so): gram_big parity, then
# config 5 interleaved against the library as built; the bench's rocprofv3 kernel summary.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
AQC_LIB=$L/libaqchip_gbb.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r5c17_gbb_tests.log 2>&1
rc=$?
echo "gbb tests rc=$rc" > gpurun_out/r5c17.rc
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for t in cur gbb; do
    if [ "$t" = cur ]; then lib=$L/libaqchip.so; else lib=$L/libaqchip_$t.so; fi
    AQC_LIB=$lib timeout -k 10 200 python3 tools/configs_bench.py --configs 5 --reps 4 > gpurun_out/r5c17_c5_${t}_$r.json 2> gpurun_out/r5c17_c5_${t}_$r.err || exit $?
  done
done
# the bench's kernel summary (the call-16 attempt deleted the database before summarising it)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r5_prof_bench.json 2> gpurun_out/r5_prof_bench.err || exit $?
db=$(find gpurun_out/r5prof -name "*.db" | head -1)
python3 tools/rocpd_stats.py "$db" > gpurun_out/r5_bench_kernel_stats.csv || exit $?
rm -rf gpurun_out/r5prof
exit 0
