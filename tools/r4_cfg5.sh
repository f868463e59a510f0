#!/bin/bash
# Round-4 call: the whole GPU suite, then config 5 at two tridiagonalisation workgroups per CU
# (default) under rocprofv3 --kernel-trace --stats (the run that ended rc = 139 at
# teardown), then config 5 at one per CU (A/B), then the Rotoselect profile.  Any failure ends it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/cfg5_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/cfg5_steps.txt
  return $rc
}
if [ -z "$SKIP_SUITE" ]; then
  step suite 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
fi
step cfg5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg5prof -o run -- python3 tools/configs_bench.py --configs 5 || exit $?
python3 tools/rocpd_stats.py gpurun_out/cfg5prof/run_results.db > gpurun_out/cfg5_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/cfg5prof
AQC_GB_PER_CU=1 step cfg5_percu1 300 python3 tools/configs_bench.py --configs 5 || exit $?
step cfg5_percu2 300 python3 tools/configs_bench.py --configs 5 || exit $?
step roto 300 python3 tools/roto_profile.py || exit $?
