"""Per-state max Jacobi sweeps on the bench overlap workload (lab tool; run on an MI355X)."""
import collections
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, apply_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
tolf = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
variant = int(sys.argv[3]) if len(sys.argv) > 3 else 2
L = _lib.lib()
_lib.check(L.aqc_mps_set_jacobi_tol(ctypes.c_double(tolf)))
_lib.check(L.aqc_mps_set_jacobi_variant(variant))
distinct = [bench.random_vidal_mps(50, 64, 1000 + k) for k in range(8)]
states = []
for s in range(B):
    d = DeviceMPS(50, 64, 1e-16, 64)
    d.load_aer(distinct[s % 8])
    states.append(d)
rng = np.random.default_rng(7)
work, ops, dist = [], [], []
for s in range(B):
    for dd in bench.DISTANCES:
        w = DeviceMPS(50, 64, 1e-16, 64)
        w.copy_from(states[s])
        work.append(w)
        ops.append(_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + dd, rng.uniform(-np.pi, np.pi, 4))))
        dist.append(dd)
for w in work:
    ms = ctypes.c_int()
    _lib.check(L.aqc_mps_jacobi_stats(w.h, ctypes.byref(ms)))
t0 = time.perf_counter()
apply_batch(work, ops)
hist = collections.defaultdict(collections.Counter)
for w, dd in zip(work, dist):
    ms = ctypes.c_int()
    _lib.check(L.aqc_mps_jacobi_stats(w.h, ctypes.byref(ms)))
    hist[dd][ms.value] += 1
print(f"variant {variant} tol factor {tolf}: apply_batch {1e3 * (time.perf_counter() - t0):.1f} ms (incl. stats)")
for dd in sorted(hist):
    print(f"  d={dd}: max-sweeps histogram {dict(sorted(hist[dd].items()))}")
