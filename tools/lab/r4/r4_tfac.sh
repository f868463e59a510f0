#!/bin/bash
# Round-4 call: config 5 with the compact-WY factors on a third stream (default) and in line
# (AQC_GB_TFAC_SIDE=0), alternating, after the gram_big tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/tfac_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/tfac_steps.txt
  return $rc
}
step tfac_tests 400 python3 -u -m pytest tests/test_gpu_gram_big.py tests/test_gpu_bigchi.py -x -q --timeout 120 --timeout-method thread || exit $?
for i in 1 2; do
  step c5_side_$i 200 python3 tools/configs_bench.py --configs 5 || exit $?
  AQC_GB_TFAC_SIDE=0 step c5_inline_$i 200 python3 tools/configs_bench.py --configs 5 || exit $?
done
