#!/bin/bash
# Round-4 staged GPU call: the 256-thread SVD alone, then the chain's headline parity, then (STAGE>=3)
# the whole GPU suite, then (STAGE>=4) a bench line.  Stops at the first failure of any kind.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/steps.txt
  return $rc
}
: > gpurun_out/steps.txt
run svd256 240 python3 -u -m pytest tests/test_gpu_svd.py -x -v --timeout 120 --timeout-method thread -k "gram" || exit $?
[ "${STAGE:-2}" -ge 2 ] || exit 0
run headline 400 python3 -u -m pytest tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread || exit $?
[ "${STAGE:-2}" -ge 3 ] || exit 0
run suite 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
[ "${STAGE:-2}" -ge 4 ] || exit 0
run bench 400 python3 bench.py --steps 20 --warmup 5 || exit $?
cp gpurun_out/bench.log gpurun_out/bench.json
# (STAGE>=5) the same bench on the 1024-thread chain for comparison
[ "${STAGE:-2}" -ge 5 ] || exit 0
AQC_CHAIN=1024 run bench1024 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-parity || exit $?
