# GPU tests + one bench line (+ config 2/4/5 when CONFIGS is set).  Outputs under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
if [ -n "$CONFIGS" ]; then
timeout -k 10 400 python3 tools/configs_bench.py --configs $CONFIGS > gpurun_out/configs.json 2> gpurun_out/configs.err
fi
