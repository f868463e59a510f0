"""A/B the Jacobi kernel variants in one process (interleaved rounds), batch of N updates."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd import gates as G  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, apply_batch  # noqa: E402

l = _lib.lib()
q = bench.random_vidal_mps(50, 64, 1000)
base = DeviceMPS(50, 64, 1e-16, 64)
base.load_aer(q)
for nb in (1, 256, 1024):
    ws = [DeviceMPS(50, 64, 1e-16, 64) for _ in range(nb)]
    ops = [_lib.ops_array([(G.TWO_QUBIT["cx"], (24, 25))]) for _ in ws]
    res = {0: [], 2: [], 3: []}
    for rnd in range(3):
        for v in (0, 2, 3):
            _lib.check(l.aqc_mps_set_jacobi_variant(v))
            for x in ws:
                x.copy_from(base)
            _lib.timing_reset(); _lib.timing_enable(True)
            apply_batch(ws, ops)
            _lib.timing_enable(False)
            res[v].append(_lib.timing_query("mps_svd")["ms"])
            sw = ctypes.c_int()
            _lib.check(l.aqc_mps_jacobi_stats(ws[0].h, ctypes.byref(sw)))
            if rnd == 2:
                print(f"   variant {v}: ov={ws[0].overlap_zero()} sweeps={sw.value} dims={ws[0].dims()[24:27]}",
                      flush=True)
    print(f"batch {nb:5d}: " + "  ".join(f"v{v} {min(res[v]):8.2f} ms ({min(res[v]) * 256 / nb:7.2f} CU-ms/SVD)"
                                         for v in res), flush=True)
