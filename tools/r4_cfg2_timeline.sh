#!/bin/bash
# Round-4 call: config 2's device timeline (kernels + copies) -> idle gaps by kind.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl -o run -- python3 tools/configs_bench.py --configs 2 --reps 1 > gpurun_out/tl.log 2>&1 || exit $?
find gpurun_out/tl -name "*.csv" >> gpurun_out/tl.log
P=$(find gpurun_out/tl -name "*_kernel_trace.csv" | head -n 1)
python3 tools/timeline_gaps.py "${P%_kernel_trace.csv}" > gpurun_out/cfg2_gaps.json
rm -f gpurun_out/tl/*/*agent_info.csv gpurun_out/tl/*agent_info.csv
