#!/bin/bash
# round 6: Gram body inlined into its callers (no call frame) vs the default build: bench A/B
# (interleaved) and WRITE_SIZE of k_chain per launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-parity"
for t in cur inl cur inl; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -k 10 200 python3 bench.py $B >> gpurun_out/r6c30_bench_$t.json 2>> gpurun_out/r6c30_bench_$t.err || exit $?
done
for t in cur inl; do
  if [ "$t" = cur ]; then lib=$PWD/adaptaqc_amd/libaqchip.so; else lib=$PWD/adaptaqc_amd/libaqchip_$t.so; fi
  AQC_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6c30_w_$t -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r6c30_w_$t.log 2>&1 || exit $?
  AQC_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6c30_f_$t -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r6c30_f_$t.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py gpurun_out/r6c30_f_$t gpurun_out/r6c30_w_$t k_chain > gpurun_out/r6c30_traffic_$t.json
  rm -rf gpurun_out/r6c30_w_$t gpurun_out/r6c30_f_$t
done
