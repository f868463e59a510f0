"""ISL all-pair sweep timing at config-3 size (50 q, chi = 64, 1225 pairs) (lab tool)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, entanglement_measures  # noqa: E402
from adaptaqc_amd.utils.constants import coupling_map_fully_entangled  # noqa: E402

pairs = np.asarray(coupling_map_fully_entangled(50), dtype=np.int32).reshape(-1)
for ns in (1, 8, 32):
    states = []
    for s in range(ns):
        d = DeviceMPS(50, 64, 1e-16, 64)
        d.load_aer(bench.random_vidal_mps(50, 64, 1000 + s % 4))
        states.append(d)
    arr = (ctypes.c_void_p * ns)(*[s.h.value for s in states])
    out = np.zeros(ns * len(pairs) // 2 * 16, dtype=np.complex128)
    L = _lib.lib()
    for rep in range(3):
        _lib.timing_reset()
        _lib.timing_enable(True)
        t0 = time.perf_counter()
        _lib.check(L.aqc_mps_pair_rdms_batch(arr, ns, _lib.ptr(pairs), len(pairs) // 2, _lib.ptr(out), 0))
        c = entanglement_measures(out.reshape(-1, 4, 4), "concurrence")
        t1 = time.perf_counter()
        _lib.timing_enable(False)
    env = _lib.timing_query("rdm_env")
    ch = _lib.timing_query("rdm_chain")
    print(f"states {ns:3d}: {1e3 * (t1 - t0):8.2f} ms wall for {ns} x 1225 pairs "
          f"(env {env['ms']:.2f} ms, chain {ch['ms']:.2f} ms = {ch['flops'] / (ch['ms'] * 1e-3) / 1e12:.2f} TFLOP/s); "
          f"mean C {c.mean():.4f}", flush=True)
