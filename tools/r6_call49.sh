#!/bin/bash
# round 6: what runs on the box after the GPU suite (two bench lines run right after it were slow)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6c49_tests.log 2>&1 || exit $?
ps -eo pid,ppid,pcpu,rss,etime,comm,args --sort=-pcpu | head -40 > gpurun_out/r6c49_ps_after_suite.txt
uptime >> gpurun_out/r6c49_ps_after_suite.txt
timeout -k 10 400 python3 bench.py --no-latency > gpurun_out/r6c49_bench.json 2> gpurun_out/r6c49_bench.err || exit $?
ps -eo pid,ppid,pcpu,rss,etime,comm,args --sort=-pcpu | head -20 > gpurun_out/r6c49_ps_after_bench.txt
