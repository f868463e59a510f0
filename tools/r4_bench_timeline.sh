#!/bin/bash
# Round-4 call: the bench step's device timeline (kernels + copies) -> idle gaps by kind.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/btl -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-parity > gpurun_out/btl.log 2>&1 || exit $?
python3 tools/timeline_gaps.py gpurun_out/btl/run --match k_chain > gpurun_out/bench_gaps.json
rm -f gpurun_out/btl/run_agent_info.csv
