"""Latency of ONE candidate sweep (one state, every pair of the 50-qubit full coupling map), the
reference's per-layer call (gradients.py:81-122 via adapt_compiler.py:839-856): the chain form
(aqc_sweep_set_chain_mode 1) against the segmented form (mode 3, sweep_seg.h), at chi = 64 and 128.

    python3 tools/single_sweep_timing.py [reps]

One JSON line per (chi, mode): median / min wall time of a whole call (host result, so the
device work is complete), and the arg-max pair (identical across modes).
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch
    from adaptaqc_amd.utils.constants import coupling_map_fully_entangled

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 50
    cmap = coupling_map_fully_entangled(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    L = _lib.lib()
    for chi in (64, 128):
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.load_aer(bench.near_product_mps(n, chi, 4000 + chi))
        for mode in (1, 3):
            _lib.check(L.aqc_sweep_set_chain_mode(ctypes.c_int(mode)))
            for _ in range(3):
                out = pair_grads_batch([d], svec, cmap, u0, gm, deg)
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                out = pair_grads_batch([d], svec, cmap, u0, gm, deg)
                ts.append(time.perf_counter() - t0)
            print(json.dumps({"chi": chi, "mode": {1: "chain", 3: "segmented"}[mode], "pairs": len(cmap),
                              "median_ms": 1e3 * float(np.median(ts)), "min_ms": 1e3 * float(np.min(ts)),
                              "argmax": int(np.argmax(out[0])), "max_grad": float(np.max(out[0]))}), flush=True)
    _lib.check(L.aqc_sweep_set_chain_mode(ctypes.c_int(0)))


if __name__ == "__main__":
    main()
