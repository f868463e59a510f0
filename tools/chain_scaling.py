"""How does the fused chain's per-update time depend on how many CUs run it at once?

For ns states (one workgroup each) with the same d = 25 layer (97 two-site updates per state),
report the launch time, the shader-clock ticks per workgroup (s_memtime, thread 0) and their ratio
(the effective shader clock if every workgroup runs concurrently: ns <= 256).  Flat ticks with a
growing launch time -> the clock drops under load; growing ticks -> a shared resource is contended.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, apply_batch, copy_batch  # noqa: E402

n, chi = bench.N_QUBITS, bench.CHI
kind = sys.argv[1] if len(sys.argv) > 1 else "near-product"
dist = int(sys.argv[2]) if len(sys.argv) > 2 else 25
src_q = bench.bench_states(n, chi, 4, kind)
srcs = []
for q in src_q:
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(q)
    srcs.append(d)
L = _lib.lib()
rng = np.random.default_rng(5)
res = []
for ns in (32, 64, 128, 192, 256, 512):
    work = [DeviceMPS(n, chi, 1e-16, chi) for _ in range(ns)]
    ops = [_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + dist, rng.uniform(-np.pi, np.pi, 4)))
           for _ in range(ns)]
    pick = [srcs[k % len(srcs)] for k in range(ns)]
    copy_batch(work, pick)
    apply_batch(work, ops, sort=True)  # warm-up
    t = (ctypes.c_double * 5)()
    _lib.check(L.aqc_mps_chain_ticks(t))
    reps = 3
    _lib.timing_reset()
    _lib.timing_enable(True)
    for _ in range(reps):
        copy_batch(work, pick)
        apply_batch(work, ops, sort=True)
    _lib.timing_enable(False)
    tq = _lib.timing_query("mps_chain")
    _lib.check(L.aqc_mps_chain_ticks(t))
    ticks = np.array(list(t)) / (reps * ns)  # per workgroup
    launch_ms = tq["ms"] / max(tq["launches"], 1)
    upd = 2 * (dist - 1) + 1  # route, gate, sort back
    row = {"states": ns, "launch_ms": launch_ms, "ticks_per_wg": float(ticks.sum()),
           "ticks_split": [float(x) for x in ticks], "updates_per_state": upd,
           "us_per_update_wall": 1e3 * launch_ms / upd * (1 if ns <= 256 else 256 / ns),
           "eff_clock_ghz": float(ticks.sum()) / (launch_ms * 1e-3) / 1e9 * (1 if ns <= 256 else ns / 256)}
    res.append(row)
    print(json.dumps(row), flush=True)
