#!/bin/bash
# Round-5 GPU call 28: the bench step's device idle time (kernel trace -> tools/step_gaps.py) now
# that the sweep takes 0.63 ms per step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5gap -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r5c28_bench.json 2> gpurun_out/r5c28_bench.err || exit $?
db=$(find gpurun_out/r5gap -name "*.db" | head -1)
python3 tools/step_gaps.py "$db" > gpurun_out/r5c28_gaps.txt 2>&1 || exit $?
rm -rf gpurun_out/r5gap
AQC_HOST_TIMING=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-latency > gpurun_out/r5c28_hosttiming.json 2> gpurun_out/r5c28_hosttiming.err || exit $?
exit 0
