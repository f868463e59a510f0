"""numpy prototype of the in-kernel QRP-preconditioned one-sided Jacobi (lab tool).

Mirrors k_jacobi_reg's QR phase step by step (zlarfg-style reflectors, H^H applied to the
trailing columns, pivot = largest trailing norm with ties to the lowest column id) and the
output convention: Jacobi runs on X = R^H, whose orthogonalised columns are the *other* side's
singular vectors times sigma, with rows mapped back through the pivot permutation.
"""
import numpy as np


def qrp_inplace(W):
    """W (L x C, L >= C) -> (R columns in place, perm) exactly as the kernel does it."""
    W = W.astype(np.complex128).copy()
    L, C = W.shape
    piv = np.zeros(C, bool)
    perm = np.zeros(C, int)
    for k in range(C):
        tn = np.where(piv, -1.0, np.sum(np.abs(W[k:, :]) ** 2, axis=0))
        p = int(np.argmax(tn))  # first maximum = lowest id
        x = W[:, p]
        alpha = x[k]
        sig2 = np.sum(np.abs(x[k + 1:]) ** 2)
        v = np.zeros(L, complex)
        if sig2 == 0.0 and alpha.imag == 0.0:
            tau, beta = 0.0, alpha.real
        else:
            beta = -np.copysign(np.sqrt(abs(alpha) ** 2 + sig2), alpha.real)
            tau = (beta - alpha) / beta
            v[k + 1:] = x[k + 1:] / (alpha - beta)
        v[k] = 1.0
        newcol = x.copy()
        newcol[k] = beta
        newcol[k + 1:] = 0.0
        W[:, p] = newcol
        piv[p] = True
        perm[k] = p
        rest = ~piv
        wv = v.conj() @ W[:, rest]                    # v^H c
        W[:, rest] -= np.conj(tau) * np.outer(v, wv)  # c -= conj(tau) v (v^H c)
    R = W[:C, perm]  # R columns in pivot order (upper triangular)
    return R, perm


def jacobi(X, tol_f=1.0):
    X = X.copy()
    L, C = X.shape
    tol = tol_f * L * 2.220446049250313e-16
    for sw in range(60):
        rot = 0
        for a in range(C - 1):
            for b in range(a + 1, C):
                x, y = X[:, a], X[:, b]
                al, be, ga = np.vdot(x, x).real, np.vdot(y, y).real, np.vdot(x, y)
                g = abs(ga)
                if g > tol * np.sqrt(al * be) and al > 0 and be > 0:
                    z = (be - al) / (2 * g)
                    t = (1.0 if z >= 0 else -1.0) / (abs(z) + np.sqrt(1 + z * z))
                    c = 1 / np.sqrt(1 + t * t)
                    s = c * t
                    e = ga / g
                    X[:, a], X[:, b] = c * x - s * np.conj(e) * y, s * e * x + c * y
                    rot += 1
        if rot == 0:
            return X, sw + 1
    return X, 60


def check(theta):
    M, N = theta.shape
    tr = M < N
    W = theta.conj().T if tr else theta
    R, perm = qrp_inplace(W)
    assert np.allclose(np.tril(R, -1), 0)
    np.testing.assert_allclose(np.abs(np.linalg.qr(W[:, perm])[1]), np.abs(R), atol=1e-12)
    X = R.conj().T
    Xf, sweeps = jacobi(X)
    C = X.shape[1]
    out = np.zeros_like(Xf)
    out[perm, :] = Xf                       # row i of X -> original column perm[i]
    sig = np.linalg.norm(out, axis=0)
    order = np.argsort(-sig, kind="stable")
    sig, out = sig[order], out[:, order]
    u, s, vh = np.linalg.svd(theta, full_matrices=False)
    np.testing.assert_allclose(sig, s, atol=1e-13)
    k = int(np.sum(s > 1e-10))
    if not tr:
        # out columns = V sigma (V = right singular vectors of theta): conj(out)/sig = rows of Vh
        V = out[:, :k] / sig[:k]
        U = theta @ V / sig[:k]                       # other side by GEMM
    else:
        U = out[:, :k] / sig[:k]                      # out columns = U sigma
        V = (U.conj().T @ theta).conj().T / sig[:k]
    np.testing.assert_allclose((U * sig[:k]) @ V.conj().T, theta, atol=1e-12 * max(1, np.abs(theta).max()))
    return sweeps


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    for (m, n) in [(8, 8), (12, 6), (6, 12), (16, 16), (32, 24)]:
        A = rng.standard_normal((m, n)) + 1j * rng.standard_normal((m, n))
        A = A * (0.7 ** np.arange(n))[None, :]
        print((m, n), "sweeps", check(A))
    # rank-deficient
    A = (rng.standard_normal((16, 3)) + 1j * rng.standard_normal((16, 3))) @ (rng.standard_normal((3, 12)) + 0j)
    print("rank3", "sweeps", check(A))
    print("ok")
