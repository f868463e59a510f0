#!/bin/bash
# Round-4 profiling, part B (GPU box; profiles/r4_exec_k_chain.json and r4_traffic.json from part A
# committed first): the full bench line, the other BASELINE configs under rocprofv3 kernel-trace
# stats, and the scaling projections (state-sharded weak scaling at N = 2, 4, 8; the strong-scaling
# batch of sweeps at N = 8).  Each step has its own limit; a failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/profb_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/profb_steps.txt
  return $rc
}
step bench 400 python3 bench.py --steps 20 --warmup 5 || exit $?
step configs 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kcfg -o run -- python3 tools/configs_bench.py --configs 2,4,5 || exit $?
python3 tools/rocpd_stats.py gpurun_out/kcfg/run_results.db > gpurun_out/configs_kernel_stats.csv
rm -rf gpurun_out/kcfg
for N in 2 4 8; do
  step weak$N 300 python3 bench.py --steps 10 --warmup 3 --simulate-world $N --no-cpu-baseline --no-parity --no-latency || exit $?
done
step strong1024 300 python3 bench.py --strong --global-states 1024 --simulate-world 8 --steps 5 --warmup 2 || exit $?
step strong256 300 python3 bench.py --strong --global-states 256 --simulate-world 8 --steps 5 --warmup 2 || exit $?
