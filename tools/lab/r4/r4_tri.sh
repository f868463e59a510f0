#!/bin/bash
# Round-4 call: the lower-triangle S3 on 1024 threads (svd path 2) -- SVD-level tests, then the
# headline workload through k_chain, then phase probes and bench lines for path 1 and 2; plus the
# SV slot A/B.  Any failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/tri_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/tri_steps.txt
  return $rc
}
step tri_diag 120 python3 tools/tri_diag.py || exit $?
step tri_svd 300 python3 -u -m pytest tests/test_gpu_svd.py -x -v --timeout 120 --timeout-method thread -k "gram" || exit $?
step tri_headline 400 python3 -u -m pytest tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread || exit $?
step tri_probe 300 env AQC_SVD_PATH=2 python3 tools/chain256_probe.py 25 32,256 || exit $?
step full_probe 300 python3 tools/chain256_probe.py 25 32,256 || exit $?
step bench_tri 400 env AQC_SVD_PATH=2 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency || exit $?
step bench_full 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-parity || exit $?
step sv_tests 400 python3 -u -m pytest tests/test_gpu_sv.py tests/test_gpu_binding.py -x -q --timeout 200 --timeout-method thread || exit $?
step cfg2_s4 300 python3 tools/configs_bench.py --configs 2 || exit $?
step cfg2_s3 300 env AQC_SV_SLOTS=3 python3 tools/configs_bench.py --configs 2 || exit $?
step bench_t16 400 env AQC_LIB=$PWD/adaptaqc_amd/libaqchip_theta16.so python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-parity || exit $?
step bench_t8 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-parity || exit $?
