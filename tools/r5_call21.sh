#!/bin/bash
# Round-5 GPU call 21: BASELINE configs 2 / 4 / 5 without the kernel trace (under rocprofv3
# --kernel-trace config 5's two-stage rounds lose their cross-stream overlap: 0.37 against 0.29 ms
# per gate; the traced run is kept for the kernel summary only), twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r5c21_configs_$r.json 2> gpurun_out/r5c21_configs_$r.err || exit $?
done
exit 0
