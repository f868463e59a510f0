#!/bin/bash
# Round-5 GPU call 20 (final profile of the round's library): the bench's kernel summary, the PMC
# passes (executed FP64 work and HBM traffic of k_chain), the default bench line, and configs 2 / 4 /
# 5 under the kernel trace -- tools/profile_round.sh with ROUND=r5 (tests ran in call 16).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROUND=r5 SKIP_TESTS=1 timeout -k 10 1000 bash tools/profile_round.sh
