"""Phase costs of the fused chain (k_chain256 or, with AQC_CHAIN=1024, k_chain) on the bench's d = 25
lists: per workgroup shader-clock ticks of theta / SVD / rank / split per two-site update, and the
Gram SVD's phases per decomposition (S1+S3, S4, S5, S6, output), for ns states at once -- ns = 32
(one state per CU: the lone latency) up to 512 (two per CU) -- with the launch time per update."""
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
dist = int(sys.argv[1]) if len(sys.argv) > 1 else 25
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32, 256, 512, 1024]
src_q = bench.bench_states(n, chi, 4, "near-product")
srcs = []
for q in src_q:
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(q)
    srcs.append(d)
L = _lib.lib()
svd_path = int(os.environ.get("AQC_SVD_PATH", "1"))  # 2: the lower-triangle S3 in the 1024-thread body
_lib.check(L.aqc_mps_set_svd_path(svd_path, 64))
rng = np.random.default_rng(5)
for ns in sizes:
    work = [DeviceMPS(n, chi, 1e-16, chi) for _ in range(ns)]
    ops = [_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + dist, rng.uniform(-np.pi, np.pi, 4)))
           for _ in range(ns)]
    pick = [srcs[k % len(srcs)] for k in range(ns)]
    copy_batch(work, pick)
    apply_batch(work, ops, sort=True)  # warm-up
    t = (ctypes.c_double * 5)()
    g = np.zeros(12)
    _lib.check(L.aqc_mps_chain_ticks(t))
    _lib.check(L.aqc_svd_gram_ticks(_lib.ptr(g)))
    reps = 3
    _lib.timing_reset()
    _lib.timing_enable(True)
    for _ in range(reps):
        copy_batch(work, pick)
        apply_batch(work, ops, sort=True)
    _lib.timing_enable(False)
    tq = _lib.timing_query("mps_chain")
    _lib.check(L.aqc_mps_chain_ticks(t))
    g = np.zeros(12)
    _lib.check(L.aqc_svd_gram_ticks(_lib.ptr(g)))
    upd = (2 * (dist - 1) + 1) * reps * ns
    launch_ms = tq["ms"] / max(tq["launches"], 1)
    row = {"chain": os.environ.get("AQC_CHAIN", "1024"), "svd_path": svd_path, "states": ns, "launch_ms": launch_ms,
           "us_per_update_wall": 1e3 * launch_ms * reps / upd,
           "ticks_per_update": {k: round(float(v) / upd) for k, v in zip(("theta", "svd", "rank", "split", "one_site"), t)},
           "gram_ticks_per_svd": {k: round(float(g[i]) / upd) for k, i in
                                  (("S1", 0), ("S1S3|S3", 1), ("S4", 2), ("S5", 3), ("S6", 4), ("out", 5),
                                   ("256:S3pass+A|1024:S3steps", 6), ("256:S3rows+B|1024:S5inv", 7),
                                   ("1024:S3phaseA", 8), ("256:S1", 9), ("256:repack", 10))}}
    print(json.dumps(row), flush=True)
