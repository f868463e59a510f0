"""Single-workgroup timing of the register Jacobi's phases (run under rocprofv3 --kernel-trace).

    rocprofv3 --kernel-trace -d gpurun_out/svdph -o run -- python3 tools/svd_phase_timing.py [reps] [variant ...]
    python3 tools/svd_phase_timing.py --report gpurun_out/svdph/run_results.db [reps] [variant ...]

A swap-routed two-site theta of the bench's random chi = 64 state (sites 24, 25) is decomposed
`reps` times with the QR phase only (aqc_svd_debug stop_after_qr = 1), then `reps` times in full;
the report splits the k_jacobi_reg dispatches in launch order, per variant (default 2).
"""
import ctypes
import os
import sqlite3
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def swap_theta(seed=1000, site=24):
    import bench

    gam, lam = bench.random_vidal_mps(50, 64, seed)
    G0 = np.stack(gam[site])
    G1 = np.stack(gam[site + 1])
    ll, lm, lr = lam[site - 1], lam[site], lam[site + 1]
    # theta[s1, l, s2, r] = ll[l] G0[s1, l, m] lm[m] G1[s2, m, r] lr[r]
    th = np.einsum("l,alm,m,bmr,r->albr", ll, G0, lm, G1, lr)
    th = th.transpose(2, 1, 0, 3)  # SWAP: (s2, l, s1, r)
    chl, chr_ = G0.shape[1], G1.shape[2]
    return th.reshape(2 * chl, 2 * chr_)


def run(reps, variants):
    from adaptaqc_amd import _lib

    T = swap_theta()
    m, n = T.shape
    th = np.asfortranarray(T.astype(np.complex128)).ravel(order="F").view(np.float64).copy()
    w = np.zeros(2 * m * n)
    sig = np.zeros(max(m, n))
    perm = np.zeros(max(m, n), dtype=np.int32)
    sw = ctypes.c_int()
    L = _lib.lib()
    for v in variants:
        for qr_only in (1, 0):
            for _ in range(reps):
                _lib.check(L.aqc_svd_debug(_lib.ptr(th), m, n, v, qr_only, _lib.ptr(w), _lib.ptr(sig),
                                           _lib.ptr(perm), ctypes.byref(sw)))
            print(f"variant {v} stop_after_qr={qr_only}: sweeps={sw.value}", flush=True)
    print("sigma[:4]", sig[:4], "min", sig[:min(m, n)].min())


def report(db, reps, variants):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels order by start").fetchall()
    d = [du for nm, du in rows if "k_jacobi_reg" in nm or "k_jacobi_b2" in nm]
    for k, v in enumerate(variants):
        qr, full = d[2 * k * reps:(2 * k + 1) * reps], d[(2 * k + 1) * reps:(2 * k + 2) * reps]
        print(f"variant {v}: QR phase: {np.mean(qr) / 1e3:.1f} us; full: {np.mean(full) / 1e3:.1f} us "
              f"(sweeps phase {np.mean(full) / 1e3 - np.mean(qr) / 1e3:.1f} us)")


def ticks(variants):
    """QR-step phase split from the kernel's shader-clock ticks (aqc_svd_debug mode 2)."""
    from adaptaqc_amd import _lib

    T = swap_theta()
    m, n = T.shape
    th = np.asfortranarray(T.astype(np.complex128)).ravel(order="F").view(np.float64).copy()
    w = np.zeros(2 * m * n)
    sig = np.zeros(max(m, n))
    perm = np.zeros(max(m, n), dtype=np.int32)
    sw = ctypes.c_int()
    L = _lib.lib()
    names = ("downdate + pivot key", "pivot barrier", "reflector + barrier", "update")
    for v in variants:
        for _ in range(3):
            _lib.check(L.aqc_svd_debug(_lib.ptr(th), m, n, v, 2, _lib.ptr(w), _lib.ptr(sig), _lib.ptr(perm),
                                       ctypes.byref(sw)))
        steps = min(m, n)
        tot = sig[:4].sum()
        print(f"variant {v}: {tot / steps:.0f} ticks per QR step: " +
              ", ".join(f"{nm} {sig[i] / steps:.0f}" for i, nm in enumerate(names)), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--ticks"]:
        ticks([int(v) for v in sys.argv[2:]] or [2])
    elif sys.argv[1:2] == ["--report"]:
        report(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 5, [int(v) for v in sys.argv[4:]] or [2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 5, [int(v) for v in sys.argv[2:]] or [2])
