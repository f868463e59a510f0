#!/bin/bash
# round 6: the staging-ring growth test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_staging_ring.py > gpurun_out/r6c55_tests.log 2>&1 || exit $?
