#!/bin/bash
# Round-4 call: grouped sweep chains of 16 first qubits (default) against 8 (AQC_SWEEP_GROUP=8):
# the gradient / sweep tests in both, config 4 and the bench step, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/g16_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/g16_steps.txt
  return $rc
}
step g16_tests 300 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_sweep_modes.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread || exit $?
AQC_SWEEP_GROUP=8 step g8_tests 300 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_sweep_modes.py -x -q --timeout 120 --timeout-method thread || exit $?
for i in 1 2; do
  step c4_g16_$i 200 python3 tools/configs_bench.py --configs 4 || exit $?
  AQC_SWEEP_GROUP=8 step c4_g8_$i 200 python3 tools/configs_bench.py --configs 4 || exit $?
done
step b_g16 300 python3 bench.py --no-cpu-baseline --no-latency --no-parity || exit $?
AQC_SWEEP_GROUP=8 step b_g8 300 python3 bench.py --no-cpu-baseline --no-latency --no-parity || exit $?
