#!/bin/bash
# round 6: lean gram_big (counters zeroed in k_gb_gram, final status written to pinned host memory
# by k_gb_cert_end) and polled stream drains at the read-backs -- A/B on the 11-layer compile,
# interleaved; gram_big and async-flag tests; the bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gram_big.py tests/test_gpu_async_flags.py tests/test_gpu_staging_ring.py > gpurun_out/r6c56_tests.log 2>&1 || exit $?
for rep in 1 2; do
  for v in lean_spin base; do
    if [ $v = base ]; then export AQC_GB_LEAN=0 AQC_SPIN_SYNC=0; else unset AQC_GB_LEAN AQC_SPIN_SYNC; fi
    timeout -k 10 300 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c56_layers_${v}_${rep}.json 2> gpurun_out/r6c56_layers_${v}_${rep}.err || exit $?
  done
done
unset AQC_GB_LEAN AQC_SPIN_SYNC
export AQC_GB_LEAN=0
timeout -k 10 300 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c56_layers_spin_only.json 2> gpurun_out/r6c56_layers_spin_only.err || exit $?
unset AQC_GB_LEAN
export AQC_SPIN_SYNC=0
timeout -k 10 300 python3 -u tools/layer_profile.py --target graded --cpu-pairs 0 > gpurun_out/r6c56_layers_lean_only.json 2> gpurun_out/r6c56_layers_lean_only.err || exit $?
unset AQC_SPIN_SYNC
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r6c56_bench.json 2> gpurun_out/r6c56_bench.err || exit $?
