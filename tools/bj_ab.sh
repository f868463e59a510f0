# Block Jacobi A/B on the GPU box: big-chi tests, config 5 with block-pair visits (default) and
# with the per-rotation kernels (AQC_BJ=rot).  Outputs under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bigchi.py tests/test_gpu_svd.py -x -v --timeout 120 --timeout-method thread > gpurun_out/bj_tests.log 2>&1
timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/bj_pair.json 2>gpurun_out/bj_pair.err
AQC_BJ=rot timeout -k 10 200 python3 tools/configs_bench.py --configs 5 > gpurun_out/bj_rot.json 2>gpurun_out/bj_rot.err
