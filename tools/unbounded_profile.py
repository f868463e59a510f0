"""Gram-path coverage and time per two-site update under the reference's DEFAULT MPS settings
(mps_sim_with_args, aer_mps_backend.py:27-42: max_chi=None; python_default_backends.py:19) and the
reference example's threshold 1e-8 (examples/advanced_mps_example.py:46): the bench's thin layers
(distances 1, 2, 5, 25, Aer swap routing, sort back) on 50-qubit chi = 64 states, capacity
512 (the unbounded limit at n = 50; the bond dimensions grow as the layers need), one batch per
configuration.  Per configuration: the Gram-path counters of both SVD paths (2 chi = 128:
aqc_svd_gram_stats; 2 chi > 128: aqc_svd_gram_big_stats), the kernel-family times (HIP events), the
wall time of the batch, the bond dimensions reached, and the time per two-site update.  For
comparison the same layers at max_chi = 64 (capacity 64: the fused chain, and capacity 512: the
lock-step path).

    python3 tools/unbounded_profile.py [--states 8] > gpurun_out/r5_unbounded.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

FAMILIES = ("mps_theta", "mps_svd", "mps_split", "mps_chain", "mps_copy")


def run(kind, thr, max_chi, cap, nstates, states_cache):
    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceMPS, apply_batch

    n, chi = bench.N_QUBITS, bench.CHI
    key = kind
    if key not in states_cache:
        states_cache[key] = bench.bench_states(n, chi, nstates, kind)
    aers = states_cache[key]
    rng = np.random.default_rng(5)
    work, ops = [], []
    for s, aer in enumerate(aers):
        for d in bench.DISTANCES:
            w = DeviceMPS(n, cap, thr, max_chi)
            w.load_aer(aer)
            work.append(w)
            ops.append(_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + d, rng.uniform(-np.pi, np.pi, 4))))
    _lib.gram_stats()
    _lib.gram_big_stats()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    apply_batch(work, ops, sort=True)
    wall = (time.perf_counter() - t0) * 1e3
    _lib.timing_enable(False)
    fam = {f: _lib.timing_query(f) for f in FAMILIES}
    g, gb = _lib.gram_stats(), _lib.gram_big_stats()
    dims = np.array([w.dims() for w in work])
    for w in work:
        w.close()
    updates = g["calls"] + gb["calls"]  # every two-site update at 2 chi >= 128 tries one of the paths
    out = {"kind": kind, "threshold": thr, "max_chi": max_chi, "chi_cap": cap, "evaluations": len(work),
           "wall_ms": wall, "gram128": g, "gram_big": gb,
           "gram128_taken_frac": g["taken"] / g["calls"] if g["calls"] else None,
           "gram_big_taken_frac": gb["taken"] / gb["calls"] if gb["calls"] else None,
           "updates_2chi_ge_128": updates, "ms_per_update": wall / updates if updates else None,
           "max_bond": int(dims.max()), "mean_max_bond": float(dims.max(axis=1).mean()),
           "families_ms": {f: round(v["ms"], 3) for f, v in fam.items() if v["launches"]}}
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", type=int, default=8)
    args = ap.parse_args()
    from adaptaqc_amd.mps_operations import _full_cap

    # the whole unbounded limit from the start (chi_cap_for now starts unbounded runs small and the
    # product paths grow the capacity on overflow; this lab tool applies one batch directly)
    cap = _full_cap(bench.N_QUBITS)
    cache = {}
    rows = []
    for kind in ("near-product", "random"):
        for thr in (1e-16, 1e-8):
            rows.append(run(kind, thr, None, cap, args.states, cache))
        rows.append(run(kind, 1e-16, 64, cap, args.states, cache))   # K = 64, lock-step at capacity 512
        rows.append(run(kind, 1e-16, 64, 64, args.states, cache))    # K = 64, the fused chain
    print(json.dumps({"summary": [{k: r[k] for k in ("kind", "threshold", "max_chi", "chi_cap", "gram128_taken_frac",
                                                  "gram_big_taken_frac", "ms_per_update", "max_bond")}
                                  for r in rows]}), flush=True)


if __name__ == "__main__":
    main()
