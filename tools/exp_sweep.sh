#!/bin/bash
# Sweep-kernel experiment: parity tests, then config-4 timings per chain mode and batch size with
# per-kernel stats (gpurun_out/sweep_*.{json,csv}).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sweep_modes.py tests/test_gpu_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1
for B in 1 32; do
  for M in 1 2; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sw_${B}_${M} -o run -- python3 tools/configs_bench.py --configs 4 --states4 $B --reps 5 --chain-mode $M > gpurun_out/sweep_${B}_${M}.json 2> gpurun_out/sweep_${B}_${M}.err
    python3 tools/rocpd_stats.py gpurun_out/sw_${B}_${M}/run_results.db > gpurun_out/sweep_${B}_${M}_stats.csv
    rm -rf gpurun_out/sw_${B}_${M}
  done
done
