"""libaqchip before torch in one process: both must share one HIP runtime (adaptaqc_amd/_lib.py
loads torch first).  Loaded the other way round, torch found no GPU after the library's first call
(GPU call 32 of round 6: torch.cuda.is_available() False)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

_CHILD = """
import sys
sys.path.insert(0, {root!r})
from adaptaqc_amd.device import DeviceMPS
d = DeviceMPS(4, 4, 1e-16, 4)
d.apply([(__import__('numpy').eye(4), (0, 1))])
import torch
assert torch.cuda.is_available(), "torch lost the GPU after libaqchip's first call"
x = torch.ones(3, device="cuda")
print(float(x.sum()))
"""


def test_library_first_then_torch():
    r = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("3.0")
