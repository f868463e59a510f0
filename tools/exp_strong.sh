#!/bin/bash
# Config-4 strong-scaling projection (bench.py --strong --simulate-world 8) at two global batch
# sizes, the sweep parity tests, and a short headline bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sweep_modes.py tests/test_gpu_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1
for G in ${GS:-256 1024}; do
  timeout -k 10 400 python3 bench.py --strong --simulate-world 8 --global-states $G --steps 3 --warmup 1 > gpurun_out/strong_$G.json 2> gpurun_out/strong_$G.err
done
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/e_bench.json 2> gpurun_out/e_bench.err
