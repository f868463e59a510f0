#!/bin/bash
# Round-5 GPU call 34: PMC passes over config 5 on the final library (executed FP64 rate and wait
# share of k_gb_tridiag, traffic).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 bash tools/pmc_configs.sh 5 k_gb_tridiag || exit $?
exit 0
