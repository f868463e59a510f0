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


if __name__ == "__main__" and (len(sys.argv) < 2 or sys.argv[1].isdigit()):
    main()


def steps():
    """The capacity-1024 test's steps one by one with timing (test_gpu_bigchi.py)."""
    import ctypes

    from adaptaqc_amd import _lib
    from adaptaqc_amd.backends import mps_sim_with_args
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops
    from adaptaqc_amd.device import DeviceMPS
    from adaptaqc_amd.mps_operations import device_mps_from_circuit

    def t(msg, t0):
        print(f"{msg}: {time.perf_counter() - t0:.3f} s", flush=True)
        return time.perf_counter()

    n, depth = 21, 24
    rng = np.random.default_rng(5)
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            qc.ry(float(rng.uniform(-np.pi, np.pi)), q)
            qc.rz(float(rng.uniform(-np.pi, np.pi)), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    t0 = time.perf_counter()
    d = device_mps_from_circuit(qc, mps_sim_with_args(mps_truncation_threshold=1e-8))
    t0 = t(f"replay cap {d.chi_cap}", t0)
    print(d.dims().tolist(), flush=True)
    t0 = t("dims", t0)
    ov = d.overlap_zero()
    t0 = t(f"overlap_zero {ov}", t0)
    c = DeviceMPS(n, d.chi_cap, 1e-16, None)
    t0 = t("create", t0)
    c.copy_from(d)
    t0 = t("copy", t0)
    qc1 = QuantumCircuit(n)
    for q in range(n):
        qc1.ry(0.3, q)
    c.apply(device_ops(qc1))
    t0 = t("apply 1q", t0)
    print(c.overlap_zero(), flush=True)
    t0 = t("overlap_zero of copy", t0)
    lib = _lib.load()
    z = d.z_all()
    t0 = t(f"z_all {z[:3]}", t0)
    cnt = ctypes.c_longlong(0)
    _lib.check(lib.aqc_env_fallbacks(ctypes.byref(cnt)))
    print("env fallbacks", cnt.value, flush=True)
    gam, lam = d.to_aer()
    t0 = t("to_aer", t0)
    pre = d.preprocessed()
    t0 = t("preprocessed", t0)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "steps":
    steps()


def zall(n, chi, cap, single):
    """z_all of one random n-qubit bond-chi state at capacity cap (single: one workgroup per chain)."""
    import bench
    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceMPS

    lib = _lib.load()
    d = DeviceMPS(n, cap, 1e-16, None)
    d.load_aer(bench.random_vidal_mps(n, chi, 3))
    _lib.check(lib.aqc_env_set_single(1 if single else 0))
    t0 = time.perf_counter()
    z = d.z_all()
    print(f"z_all n={n} chi={chi} cap={cap} single={single}: {time.perf_counter() - t0:.3f} s {z[:2]}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "zall":
    zall(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1")
