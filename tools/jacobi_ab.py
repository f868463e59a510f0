"""A/B of the two-site SVD kernel configurations on the bench's overlap workload (lab tool; MI355X).

    python tools/jacobi_ab.py [states] [variant:tiny[:fused[:tol_factor]] ...]   e.g. 256 2:1e-6 2:1e-6:0 2:1e-6:1:32

Per config: the bench's overlap evaluations (thinly-dressed layers at distances 1, 2, 5, 25 on
`states` random 50-qubit chi = 64 states: Aer routing, SVD truncation at chi = 64, sort back) run
twice; the second run's wall time, its mps_svd / mps_chain kernel time (HIP events on the MPS
stream) and the largest sweep count of a sample of states are reported, and each config's overlaps <0|psi> are compared with the first's (relative).
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, apply_batch, copy_batch, overlap_zero_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
def _cfg(c):
    f = c.split(":")
    return (int(f[0]), float(f[1]), int(f[2]) if len(f) > 2 else 1, float(f[3]) if len(f) > 3 else 1.0)


configs = [_cfg(c) for c in sys.argv[2:]] or [(2, 1e-6, 1, 1.0), (2, 1e-6, 0, 1.0)]
L = _lib.lib()
distinct = [bench.random_vidal_mps(50, bench.CHI, 1000 + k) for k in range(8)]
states = []
for s in range(B):
    d = DeviceMPS(50, bench.CHI, 1e-16, bench.CHI)
    d.load_aer(distinct[s % len(distinct)])
    states.append(d)
work = [DeviceMPS(50, bench.CHI, 1e-16, bench.CHI) for _ in range(B * len(bench.DISTANCES))]
src = [states[k // len(bench.DISTANCES)] for k in range(len(work))]
rng = np.random.default_rng(7)
ops = [_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + d, rng.uniform(-np.pi, np.pi, 4)))
       for _ in range(B) for d in bench.DISTANCES]
ref = None
try:
    for variant, tiny, fused, tolf in configs:
        _lib.check(L.aqc_mps_set_jacobi_tol(ctypes.c_double(tolf)))
        _lib.check(L.aqc_mps_set_jacobi_variant(variant))
        _lib.check(L.aqc_mps_set_jacobi_stop(ctypes.c_double(tiny)))
        _lib.check(L.aqc_mps_set_fused_chain(fused))
        for rep in range(2):
            if rep == 1 and fused and variant == 2:
                _lib.check(L.aqc_mps_chain_ticks(_lib.ptr(np.zeros(5))))
            copy_batch(work, src)
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            apply_batch(work, ops, sort=True)
            wall = time.perf_counter() - t0
            ov = overlap_zero_batch(work)
            wall2 = time.perf_counter() - t0
            _lib.timing_enable(False)
        svd = _lib.timing_query("mps_chain" if fused and variant == 2 else "mps_svd")
        sw = ctypes.c_int()
        msw = 0
        for w in work[:: max(1, len(work) // 64)]:
            _lib.check(L.aqc_mps_jacobi_stats(w.h, ctypes.byref(sw)))
            msw = max(msw, sw.value)
        if fused and variant == 2:
            tks = np.zeros(5)
            _lib.check(L.aqc_mps_chain_ticks(_lib.ptr(tks)))
            nu = tks[:4].sum()
            print("   chain phase shares: " + ", ".join(f"{nm} {100 * v / max(nu, 1):.1f}%" for nm, v in
                                                    zip(("theta", "jacobi", "rank", "split"), tks[:4])), flush=True)
        if ref is None:
            ref = ov
        print(f"variant {variant} tiny {tiny:.0e} fused {fused} tol x{tolf:g}: apply {wall * 1e3:8.2f} ms wall "
              f"({wall2 * 1e3:8.2f} with the overlaps), "
              f"{'chain' if fused and variant == 2 else 'svd'} {svd['ms']:8.2f} ms over {svd['launches']} launches "
              f"({svd['ms'] / max(svd['launches'], 1):.3f} ms/launch), max sweeps {msw}, "
              f"max |<0|psi> - ref| / |ref| {np.max(np.abs(ov - ref) / np.abs(ref)):.2e}", flush=True)
finally:
    _lib.check(L.aqc_mps_set_jacobi_variant(2))
    _lib.check(L.aqc_mps_set_jacobi_stop(ctypes.c_double(0.0)))
    _lib.check(L.aqc_mps_set_fused_chain(1))
    _lib.check(L.aqc_mps_set_jacobi_tol(ctypes.c_double(1.0)))
