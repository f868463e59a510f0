#!/bin/bash
# round 6: bench with and without the CPU-baseline leg before it (the full line was 3.4 ms a step
# slower than the kernel-trace run), per-step times; overlap kernel on dynamic LDS
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_zsum.py > gpurun_out/r6c23_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --no-latency > gpurun_out/r6c23_bench_nocpu.json 2> gpurun_out/r6c23_bench_nocpu.err || exit $?
timeout -k 10 400 python3 bench.py --no-parity --no-latency > gpurun_out/r6c23_bench_cpu.json 2> gpurun_out/r6c23_bench_cpu.err || exit $?
AQC_HOST_TIMING=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --no-latency > gpurun_out/r6c23_bench_ht.json 2> gpurun_out/r6c23_bench_ht.err || exit $?
