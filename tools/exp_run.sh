#!/bin/bash
# Experiment driver for one gpurun call: GPU tests, a short bench with the parity check, and the
# k_chain FETCH/WRITE passes (gpurun_out/traffic.json).  AQC_LIB selects an experiment library.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
fi
B="--steps 3 --warmup 1 --no-cpu-baseline --no-latency"
timeout -k 10 300 python3 bench.py $B > gpurun_out/e_bench.json 2> gpurun_out/e_bench.err
timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/svdg.txt 2>&1
Q="--steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-latency"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 bench.py $Q > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 bench.py $Q > gpurun_out/pmc_write.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write k_chain > gpurun_out/traffic.json
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
