#!/bin/bash
# Round-4 call: the single-workgroup tail of the multi-workgroup tridiagonalisation (k_gb_tail) --
# the gram_big tests (tail and exchange-to-end), config 5 with the tail and without it (A/B), and
# the kernel statistics of config 5 with the tail.  Any failure ends it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/tail_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/tail_steps.txt
  return $rc
}
step tail_tests 400 python3 -u -m pytest tests/test_gpu_gram_big.py -x -v --timeout 120 --timeout-method thread || exit $?
step cfg5_tail 300 python3 tools/configs_bench.py --configs 5 || exit $?
AQC_GB_TAIL=0 step cfg5_notail 300 python3 tools/configs_bench.py --configs 5 || exit $?
step cfg5_tail_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tailprof -o run -- python3 tools/configs_bench.py --configs 5 || exit $?
python3 tools/rocpd_stats.py gpurun_out/tailprof/run_results.db > gpurun_out/cfg5_tail_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/tailprof
