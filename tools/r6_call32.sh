#!/bin/bash
# round 6: torch device visibility diagnostic (torch.cuda init failed after libaqchip tests in call 31)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "import torch; print('torch alone', torch.cuda.is_available(), torch.cuda.device_count())" > gpurun_out/r6c32_diag.txt 2>&1
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, '.')
from adaptaqc_amd import _lib
from adaptaqc_amd.device import DeviceMPS
d = DeviceMPS(4, 4, 1e-16, 4)
import torch; print('after libaqchip', torch.cuda.is_available(), torch.cuda.device_count())" >> gpurun_out/r6c32_diag.txt 2>&1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grad.py > gpurun_out/r6c32_grad.log 2>&1
echo "grad alone rc=$?" >> gpurun_out/r6c32_diag.txt
env | grep -i "visible\|hip_\|rocr\|cuda" >> gpurun_out/r6c32_diag.txt
