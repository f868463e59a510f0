"""Single 128x128 two-site update (CX at the middle of a random chi=64 MPS), repeated."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd import gates as G  # noqa: E402
from adaptaqc_amd.device import DeviceMPS  # noqa: E402

q = bench.random_vidal_mps(50, 64, 1000)
base = DeviceMPS(50, 64, 1e-16, 64)
base.load_aer(q)
w = DeviceMPS(50, 64, 1e-16, 64)
ops = _lib.ops_array([(G.TWO_QUBIT["cx"], (24, 25))])
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    w.copy_from(base)
    w.apply(ops)
print("done", w.overlap_zero())
