"""Probe the two-site SVD kernel: sweeps and time per 128x128 update vs Jacobi tolerance."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd import gates as G  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, apply_batch  # noqa: E402

q = bench.random_vidal_mps(50, 64, 1000)
l = _lib.lib()
for tolf in (1.0, 4.0, 16.0, 64.0):
    _lib.check(l.aqc_mps_set_jacobi_tol(tolf))
    base = DeviceMPS(50, 64, 1e-16, 64)
    base.load_aer(q)
    w = DeviceMPS(50, 64, 1e-16, 64)
    for reps in range(2):
        w.copy_from(base)
        ops = _lib.ops_array([(G.TWO_QUBIT["cx"], (24, 25))])
        _lib.timing_reset(); _lib.timing_enable(True)
        t = time.perf_counter()
        w.apply(ops)
        dt = time.perf_counter() - t
        _lib.timing_enable(False)
        sw = ctypes.c_int()
        _lib.check(l.aqc_mps_jacobi_stats(w.h, ctypes.byref(sw)))
    ov = w.overlap_zero()
    print(f"tol x{tolf:5.1f}: sweeps={sw.value:3d} wall={dt*1e3:8.2f} ms svd={_lib.timing_query('mps_svd')['ms']:8.2f} ms "
          f"theta={_lib.timing_query('mps_theta')['ms']:.3f} split={_lib.timing_query('mps_split')['ms']:.3f} ov={ov}", flush=True)
# batch of 256 concurrent updates
_lib.check(l.aqc_mps_set_jacobi_tol(1.0))
base = DeviceMPS(50, 64, 1e-16, 64); base.load_aer(q)
ws = [DeviceMPS(50, 64, 1e-16, 64) for _ in range(256)]
for x in ws: x.copy_from(base)
ops = [_lib.ops_array([(G.TWO_QUBIT["cx"], (24, 25))]) for _ in ws]
_lib.timing_reset(); _lib.timing_enable(True)
t = time.perf_counter(); apply_batch(ws, ops); dt = time.perf_counter() - t
_lib.timing_enable(False)
print(f"batch 256: wall {dt*1e3:.2f} ms, svd {_lib.timing_query('mps_svd')['ms']:.2f} ms")
