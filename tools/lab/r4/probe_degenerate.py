"""Register-Jacobi accuracy on spectra with degenerate clusters and on graded columns (aqc_svd_debug
variants 2 / 7) against numpy, per Jacobi noise-floor factor (aqc_mps_set_jacobi_noise): max |sigma -
ref| over the top 64 (relative to sigma_1), sweeps, and for the graded cases the worst singular-vector
error where sigma > 1e-8 sigma_1 (the test_gpu_svd contract).

    python3 tools/probe_degenerate.py [noise factors...]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_svd import _run, _spectrum_theta, _theta  # noqa: E402

rng = np.random.default_rng(0)
SPECTRA = [
    ("8x1 + 120x1e-6", np.concatenate([np.ones(8), 1e-6 * np.ones(120)])),
    ("8x1 + 120x1e-5", np.concatenate([np.ones(8), 1e-5 * np.ones(120)])),
    ("8x1 + 120x1e-3", np.concatenate([np.ones(8), 1e-3 * np.ones(120)])),
    ("8x1 + 120x1e-6(1+0.1r)", np.concatenate([np.ones(8), 1e-6 * (1 + 0.1 * rng.random(120))])),
    ("64x1 + 64x1e-6", np.concatenate([np.ones(64), 1e-6 * np.ones(64)])),
    ("2x1 + 126 graded", np.concatenate([np.ones(2), 0.5 * 0.9 ** np.arange(126)])),
    ("0.93^i", 0.93 ** np.arange(128)),
]
GRADED = [(32, 32), (64, 64), (128, 64), (128, 128)]


def vec_err(th, w, sig):
    m, n = th.shape
    u, s, vh = np.linalg.svd(th, full_matrices=False)
    k = int(np.sum(s > 1e-8 * s[0]))
    order = np.argsort(-sig, kind="stable")
    w, sig = w[:, order], sig[order]
    ref = vh[:k].conj().T if m >= n else u[:, :k]
    cols = w[:, :k] / sig[:k]
    return float(np.max(np.abs(np.abs(cols.conj().T @ ref) - np.eye(k))))


def main():
    from adaptaqc_amd import _lib

    L = _lib.lib()
    factors = [float(x) for x in sys.argv[1:]] or [16.0]
    for f in factors:
        _lib.check(L.aqc_mps_set_jacobi_noise(ctypes.c_double(f)))
        print(f"--- noise factor {f}")
        for name, s in SPECTRA:
            th = _spectrum_theta(128, 128, s, 5)
            ref = np.linalg.svd(th, compute_uv=False)
            for v in (2, 7):
                w, sig, _, sw = _run(th, v)
                err = np.max(np.abs(np.sort(sig)[::-1][:64] - ref[:64])) / ref[0]
                print(f"{name:26s} v{v}: sweeps {sw:2d} max|dsig| {err:.2e}", flush=True)
        for m, n in GRADED:
            th = _theta(m, n, m * 31 + n)
            w, sig, _, sw = _run(th, 2)
            print(f"graded {m}x{n} v2: sweeps {sw:2d} vector err {vec_err(th, w, sig):.2e}", flush=True)
    _lib.check(L.aqc_mps_set_jacobi_noise(ctypes.c_double(16.0)))


if __name__ == "__main__":
    main()
