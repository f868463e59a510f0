#!/bin/bash
# One GPU call of diagnostics: the sweep-only host timing, the S3 diagnostic probe (libaqchip_diag.so
# built with -DAQC_S3_DIAG=1), and a kernel trace of a short bench run with its per-step GPU idle
# gaps.  Every step has its own time limit; the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/sweep_host_timing.py 10 > gpurun_out/sweep_host.txt 2>&1
AQC_LIB=$PWD/adaptaqc_amd/libaqchip_diag.so timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/probe_diag.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gaps -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/gaps_bench.json 2> gpurun_out/gaps.err
python3 tools/step_gaps.py gpurun_out/gaps/run_results.db > gpurun_out/step_gaps.txt 2>&1
rm -rf gpurun_out/gaps
