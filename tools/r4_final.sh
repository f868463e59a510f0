#!/bin/bash
# Round-4 final measurement (GPU box), after the defaults are decided: the whole GPU suite, a bench
# line, rocprofv3 kernel stats of a short bench run, the PMC passes, and the untraced BASELINE
# configs.  Each step has its own limit; a failure ends the call.  Outputs under gpurun_out/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/final_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/final_steps.txt
  return $rc
}
if [ -z "$SKIP_SUITE" ]; then
  step fsuite 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
fi
step fktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fktrace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency || exit $?
python3 tools/rocpd_stats.py gpurun_out/fktrace/run_results.db > gpurun_out/final_kernel_stats.csv
rm -rf gpurun_out/fktrace
timeout -k 10 900 bash tools/pmc_bench.sh
rc=$?; echo "pmc rc=$rc" >> gpurun_out/final_steps.txt; [ $rc -eq 0 ] || exit $rc
step fconfigs 400 python3 tools/configs_bench.py --configs 2,4,5 || exit $?
step fbench 600 python3 bench.py || exit $?
