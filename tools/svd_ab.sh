# Gram SVD change check on the GPU box: SVD / headline / MPS tests, Gram phase ticks, bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svd.py tests/test_gpu_headline.py tests/test_gpu_mps.py tests/test_gpu_bigchi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1
timeout -k 10 200 python3 tools/svd32_probe.py 5 > gpurun_out/svd32.txt 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/bench_svd.json 2> gpurun_out/bench_svd.err
