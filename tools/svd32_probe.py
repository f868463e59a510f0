"""The Gram path (aqc_svd_debug variant 7) and the register Jacobi (variant 2) on the bench's
swap-routed two-site thetas: singular values and kept subspace against numpy, the Gram path's
phase ticks.  (Until round 2 it also ran the FP32 Jacobi, variant 6, now removed: tools/lab.)

    python3 tools/svd32_probe.py [reps]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def swap_theta(aer, site=24):
    gam, lam = aer
    G0 = np.stack(gam[site])
    G1 = np.stack(gam[site + 1])
    ll, lm, lr = lam[site - 1], lam[site], lam[site + 1]
    th = np.einsum("l,alm,m,bmr,r->albr", ll, G0, lm, G1, lr)
    th = th.transpose(2, 1, 0, 3)  # SWAP: (s2, l, s1, r)
    return th.reshape(2 * G0.shape[1], 2 * G1.shape[2])


def main():
    from adaptaqc_amd import _lib

    if os.environ.get("AQC_LIB"):  # experiment builds
        _lib.load(os.environ["AQC_LIB"])
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    L = _lib.lib()
    for kind in ("near-product", "random"):
        aer = bench.bench_states(50, 64, 1, kind)[0]
        T = swap_theta(aer)
        m, n = T.shape
        ref = np.linalg.svd(T, compute_uv=False)
        th = np.asfortranarray(T.astype(np.complex128)).ravel(order="F").view(np.float64).copy()
        w = np.zeros(2 * m * n)
        sig = np.zeros(max(m, n))
        sw = ctypes.c_int()
        for v, tiny in [(2, None), (7, None)]:
            for _ in range(reps):
                _lib.check(L.aqc_svd_debug(_lib.ptr(th), m, n, v, 0, _lib.ptr(w), _lib.ptr(sig), None,
                                           ctypes.byref(sw)))
            got = np.sort(sig[:min(m, n)])[::-1]
            kk = 64 if v == 7 else min(m, n)  # the Gram path returns the top 64
            err = np.max(np.abs(got[:kk] - ref[:kk])) / ref[0]
            # the columns: right singular vectors x sigma (variant 2 / 6 contract); check V^H V
            W = w.view(np.complex128).reshape(min(m, n), -1)[: (64 if v == 7 else min(m, n))]
            nn = np.linalg.norm(W, axis=1)
            V = W / nn[:, None]
            orth = np.max(np.abs(V.conj() @ V.T - np.eye(len(V))))
            if v in (2, 7):  # kept subspace (top 64) against numpy
                _, _, vh = np.linalg.svd(T)
                Vt = vh[:64].conj().T
                idx = np.argsort(-sig[:min(m, n)])[:64]
                Vk = (w.view(np.complex128).reshape(min(m, n), -1)[idx] / np.sort(sig[:min(m, n)])[::-1][:64, None]).T
                sub = np.linalg.norm(Vk @ Vk.conj().T - Vt @ Vt.conj().T, 2)
                print(f"   kept-subspace distance {sub:.2e}")
            if v == 7:
                tk = np.zeros(12)
                _lib.check(L.aqc_svd_gram_ticks(_lib.ptr(tk)))
                print("   gram phase ticks per call (S1 gram, S3 tridiag [C part], S4 eig, S5 vec, S6 back, out, S3 column steps, S5 inverse iteration part, S3 phase A, [diag] zlarfg done, wave-13 column pass):",
                      (tk[:11] / reps).astype(int).tolist())
            print(f"{kind:12s} variant {v} tiny {tiny}: sweeps {sw.value:2d}  max|sigma - ref|/sigma_1 {err:.2e}  "
                  f"max|V^H V - I| {orth:.2e}", flush=True)


if __name__ == "__main__":
    main()
