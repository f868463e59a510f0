#!/bin/bash
# Kernel-trace statistics of the single-state candidate sweep (tools/single_sweep_timing.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seg -o run -- python3 tools/single_sweep_timing.py 10 > gpurun_out/prof_seg.txt 2>&1
python3 tools/rocpd_stats.py gpurun_out/prof_seg/run_results.db > gpurun_out/prof_seg_stats.csv 2>&1 || find gpurun_out/prof_seg -name "*.csv" | head > gpurun_out/prof_seg_files.txt
rm -rf gpurun_out/prof_seg
