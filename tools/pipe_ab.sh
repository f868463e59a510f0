set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_headline.py tests/test_gpu_mps.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/bench_pipe.json 2> gpurun_out/bench_pipe.err
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-pipeline > gpurun_out/bench_nopipe.json 2> gpurun_out/bench_nopipe.err
