#!/bin/bash
# Round-4 profiling, part A (GPU box): rocprofv3 kernel-trace stats of a short bench run, then the
# PMC passes (tools/pmc_bench.sh: separate passes, the guide's counter limits).  Outputs under
# gpurun_out/; copy exec_k_chain.json / traffic.json / kernel_stats.csv / pmc_summary.txt into
# profiles/ as r4_* before part B (the full bench line reads them).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/profa_steps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/ktrace_bench.json 2> gpurun_out/ktrace.err
rc=$?; echo "ktrace rc=$rc" >> gpurun_out/profa_steps.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_stats.py gpurun_out/ktrace/run_results.db > gpurun_out/kernel_stats.csv
rm -rf gpurun_out/ktrace
timeout -k 10 900 bash tools/pmc_bench.sh
rc=$?; echo "pmc rc=$rc" >> gpurun_out/profa_steps.txt; exit $rc
