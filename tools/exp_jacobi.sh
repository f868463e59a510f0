#!/bin/bash
# Jacobi threshold experiment: degenerate-spectrum probe, SVD / MPS GPU tests, bench, config 5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 tools/probe_degenerate.py > gpurun_out/deg.txt 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_mps.py tests/test_gpu_bigchi.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/jtests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/e_bench.json 2> gpurun_out/e_bench.err
timeout -k 10 300 python3 tools/configs_bench.py --configs 5 > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
