#!/bin/bash
# Round-5 GPU call 33 (final library): smoke(), configs 2 / 4 / 5 without the trace, the default
# bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c33_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/configs_bench.py --configs 2,4,5 > gpurun_out/r5c33_configs.json 2> gpurun_out/r5c33_configs.err || exit $?
timeout -k 10 500 python3 bench.py > gpurun_out/r5c33_bench.json 2> gpurun_out/r5c33_bench.err || exit $?
exit 0
