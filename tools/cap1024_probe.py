"""Capacity-1024 probe: the 21-qubit depth-24 brickwork at threshold 1e-8, max_chi None (the
test_gpu_bigchi.py case), replayed on the device with per-stage timing and the SVD path counters;
prints a line per stage so a long run shows progress."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from adaptaqc_amd import _lib
    from adaptaqc_amd import mps_operations as mo
    from adaptaqc_amd.backends import mps_sim_with_args
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops_array
    from adaptaqc_amd.device import DeviceMPS

    n, depth = int(sys.argv[1]) if len(sys.argv) > 1 else 21, int(sys.argv[2]) if len(sys.argv) > 2 else 24
    rng = np.random.default_rng(5)
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            qc.ry(float(rng.uniform(-np.pi, np.pi)), q)
            qc.rz(float(rng.uniform(-np.pi, np.pi)), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    ops = device_ops_array(qc, 0)
    for cap in (128, 256, 512, 1024):
        d = DeviceMPS(n, cap, 1e-8, None)
        d.load_aer(mo.zero_aer_mps(n))
        _lib.gram_stats(), _lib.gram_big_stats()
        t0 = time.perf_counter()
        try:
            d.apply(ops)
            d.sort()
            ok = True
        except Exception as e:  # capacity overflow below 1024
            ok = str(e)[:80]
        dt = time.perf_counter() - t0
        print(f"cap {cap}: {dt:.3f} s, ok={ok}, gram128={_lib.gram_stats()}, gram_big={_lib.gram_big_stats()}",
              flush=True)
        if ok is True:
            print("dims", d.dims().tolist(), flush=True)
            break


if __name__ == "__main__":
    main()
