"""Gram-path (2 chi <= 128) phase ticks per decomposition in two workloads: a 7-layer
paper-setting compile (tools/layer_profile.py's graded target, lock-step k_svd_gram) and the bench's
chain (k_chain).  S5 minus its inverse-iteration part is the Gram-Schmidt in clusters + Rayleigh
quotients.

    python3 tools/gram_phase_compile.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

NAMES = ["S1", "S2+S3", "S4", "S5", "S6", "output", "S3_columns", "S5_inverse_iteration", "S3_phaseA",
         "S3_cols_32_63", "S3_cols_64_95", "S3_cols_96_on"]


def read(L):
    t = np.zeros(12)
    s = np.zeros(6)
    L.aqc_svd_gram_ticks(t.ctypes.data)
    L.aqc_svd_gram_stats(s.ctypes.data)
    return t, s


def per_call(t, s):
    calls = max(s[1], 1.0)
    out = {n: float(t[k] / calls) for k, n in enumerate(NAMES)}
    out["S5_gs_and_rayleigh"] = out["S5"] - out["S5_inverse_iteration"]
    out["calls"] = float(s[0])
    out["taken"] = float(s[1])
    return out


def main():
    import torch  # noqa: F401  (one HIP runtime: torch first)

    import layer_profile as lp
    from adaptaqc_amd import _lib

    L = _lib.lib()

    class A:
        target, threshold, max_chi, seed, layers = "graded", 1e-8, 0, 21, 7

    read(L)
    lp.gpu_layers(A)
    t, s = read(L)
    res = {"compile_7_layers": per_call(t, s)}
    import bench  # noqa: F401
    from adaptaqc_amd.device import DeviceMPS, OpsBatch, apply_batch, copy_batch

    distinct = bench.bench_states(50, 64, 4, "near-product")
    src = []
    for a in distinct:
        d = DeviceMPS(50, 64, 1e-16, 64)
        d.load_aer(a)
        src.append(d)
    work = [DeviceMPS(50, 64, 1e-16, 64) for _ in range(256)]
    rng = np.random.default_rng(7)
    ops = [_lib.ops_array(bench.thin_layer_ops(12, 12 + 25, rng.uniform(-np.pi, np.pi, 4))) for _ in work]
    batch = OpsBatch(ops)
    copy_batch(work, [src[k % 4] for k in range(len(work))])
    read(L)
    apply_batch(work, batch, sort=True)
    t, s = read(L)
    res["bench_chain_d25"] = per_call(t, s)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
