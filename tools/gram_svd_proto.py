"""Numpy prototype of the Gram / tridiagonal two-site SVD (the device kernel svd_gram.h follows it
step by step): G = X^H X, Householder tridiagonalisation (zhetd2, lower), multisection for the
top-K eigenvalues of the real tridiagonal T, inverse iteration (tridiagonal LU with partial
pivoting) + Gram-Schmidt inside clusters, Rayleigh-quotient sigma, back-transformation V = Q Z.
Checks sigma and the kept subspace against numpy's SVD on the bench's swap thetas."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def zhetd2_lower(G):
    G = G.copy()
    n = G.shape[0]
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    vs, taus = [], []
    for k in range(n - 1):
        x = G[k + 1:, k].copy()
        alpha = x[0]
        xnorm2 = np.sum(np.abs(x[1:]) ** 2)
        if xnorm2 == 0 and alpha.imag == 0:
            tau = 0.0
            beta = alpha.real
            v = np.zeros_like(x)
            v[0] = 1
        else:
            beta = -np.copysign(np.sqrt(abs(alpha) ** 2 + xnorm2), alpha.real)
            tau = complex((beta - alpha.real) / beta, -alpha.imag / beta)
            v = x / (alpha - beta)
            v[0] = 1
        e[k] = beta
        d[k] = G[k, k].real
        A22 = G[k + 1:, k + 1:]
        if tau != 0:
            w = tau * (A22 @ v)
            a2 = -0.5 * tau * np.vdot(w, v)
            w = w + a2 * v
            A22 -= np.outer(v, w.conj()) + np.outer(w, v.conj())
        vs.append(v)
        taus.append(tau)
    d[n - 1] = G[n - 1, n - 1].real
    return d, e, vs, taus


def sturm_count(d, e, x, pivmin):
    c = 0
    q = d[0] - x
    if abs(q) < pivmin:
        q = -pivmin
    c += q < 0
    for j in range(1, len(d)):
        q = (d[j] - x) - e[j - 1] ** 2 / q
        if abs(q) < pivmin:
            q = -pivmin
        c += q < 0
    return c


def multisection(d, e, K, ways=16, rounds=8):
    n = len(d)
    r = np.abs(np.concatenate([[0], e])) + np.abs(np.concatenate([e, [0]]))
    lo0, hi0 = np.min(d - r), np.max(d + r)
    span = max(hi0 - lo0, 1e-300)
    pivmin = 1e-300 + np.finfo(float).tiny
    lams = []
    for i in range(K):
        a = n - 1 - i  # ascending index
        lo, hi = lo0 - 1e-12 * span, hi0 + 1e-12 * span
        for _ in range(rounds):
            pts = lo + (hi - lo) * np.arange(1, ways + 1) / (ways + 1)
            cnt = np.array([sturm_count(d, e, x, pivmin) for x in pts])
            # largest point with count <= a -> new lo ; smallest with count >= a+1 -> new hi
            below = np.nonzero(cnt <= a)[0]
            above = np.nonzero(cnt >= a + 1)[0]
            nlo = pts[below[-1]] if len(below) else lo
            nhi = pts[above[0]] if len(above) else hi
            lo, hi = nlo, nhi
        lams.append(0.5 * (lo + hi))
    return np.array(lams)


def tri_solve(d, e, lam, b):
    """(T - lam I) z = b by Gaussian elimination with partial pivoting (dgtsv-like)."""
    n = len(d)
    dl = e.copy()
    dd = d - lam
    du = e.copy()
    du2 = np.zeros(n)
    b = b.copy()
    eps = 1e-300
    # forward elimination with row interchanges
    dd = dd.astype(float)
    for i in range(n - 1):
        if abs(dd[i]) >= abs(dl[i]):
            if dd[i] == 0:
                dd[i] = eps
            m = dl[i] / dd[i]
            dd[i + 1] -= m * du[i]
            b[i + 1] -= m * b[i]
            if i < n - 2:
                du2[i] = 0
        else:
            m = dd[i] / dl[i]
            dd[i] = dl[i]
            tmp = dd[i + 1]
            dd[i + 1] = du[i] - m * tmp
            if i < n - 2:
                du2[i] = du[i + 1]
                du[i + 1] = -m * du[i + 1]
            du[i] = tmp
            b[i], b[i + 1] = b[i + 1], b[i] - m * b[i + 1]
    if dd[n - 1] == 0:
        dd[n - 1] = eps
    z = np.zeros(n)
    z[n - 1] = b[n - 1] / dd[n - 1]
    if n > 1:
        z[n - 2] = (b[n - 2] - du[n - 2] * z[n - 1]) / dd[n - 2]
    for i in range(n - 3, -1, -1):
        z[i] = (b[i] - du[i] * z[i + 1] - du2[i] * z[i + 2]) / dd[i]
    return z


def gram_svd(X, K):
    L, C = X.shape
    G = X.conj().T @ X
    d, e, vs, taus = zhetd2_lower(G)
    lam = multisection(d, e, K)
    tnorm = np.max(np.abs(d)) + 2 * np.max(np.abs(e)) if len(e) else np.max(np.abs(d))
    Z = np.zeros((C, K))
    for i in range(K):
        rng = np.random.default_rng(i)
        z = rng.uniform(-1, 1, C)
        for _ in range(3):
            z = tri_solve(d, e, lam[i], z)
            z /= np.linalg.norm(z)
        Z[:, i] = z
    # Gram-Schmidt within clusters
    ortol = 1e-3 * tnorm
    start = 0
    for i in range(1, K):
        if lam[i - 1] - lam[i] >= ortol:
            start = i
            continue
        for jj in range(start, i):
            Z[:, i] -= (Z[:, jj] @ Z[:, i]) * Z[:, jj]
        Z[:, i] /= np.linalg.norm(Z[:, i])
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    sig2 = np.einsum("ij,ij->j", Z, T @ Z)
    # back-transformation V = H_0 ... H_{n-2} Z
    V = Z.astype(complex)
    for k in range(C - 2, -1, -1):
        v, tau = vs[k], taus[k]
        s = v.conj() @ V[k + 1:, :]
        V[k + 1:, :] -= tau * np.outer(v, s)
    return V, np.sqrt(np.maximum(sig2, 0)), lam


def main():
    import bench
    from tools.svd32_probe import swap_theta

    for kind in ("random", "near-product"):
        aer = bench.bench_states(50, 64, 1, kind)[0]
        T = swap_theta(aer)
        u, s, vh = np.linalg.svd(T)
        V, sig, lam = gram_svd(T, 64)
        print(kind, "sigma err", np.max(np.abs(sig - s[:64])) / s[0], "lam_K/lam_0", s[63] ** 2 / s[0] ** 2)
        Vt = vh[:64].conj().T
        # kept-subspace distance
        P = V @ V.conj().T - Vt @ Vt.conj().T
        print("  subspace err", np.linalg.norm(P, 2), " V^H V - I", np.max(np.abs(V.conj().T @ V - np.eye(64))))


if __name__ == "__main__":
    main()


def ldl_solve(d, e, lam, b, tnorm):
    """(T - lam I) z = b by the unpivoted LDL^T factorisation (D only stored; tiny pivots replaced
    by eps * ||T||), as the device kernel does."""
    n = len(d)
    D = np.zeros(n)
    y = b.copy()
    piv = 2.2e-16 * tnorm
    for j in range(n):
        Dj = d[j] - lam - (e[j - 1] ** 2 / D[j - 1] if j > 0 else 0.0)
        if abs(Dj) < piv:
            Dj = piv if Dj >= 0 else -piv
        D[j] = Dj
        if j > 0:
            y[j] -= (e[j - 1] / D[j - 1]) * y[j - 1]
    z = np.zeros(n)
    z[n - 1] = y[n - 1] / D[n - 1]
    for j in range(n - 2, -1, -1):
        z[j] = (y[j] - e[j] * z[j + 1]) / D[j]
    return z


def gram_svd_ldl(X, K, iters=3):
    L, C = X.shape
    G = X.conj().T @ X
    d, e, vs, taus = zhetd2_lower(G)
    lam = multisection(d, e, K)
    tnorm = np.max(np.abs(d)) + 2 * np.max(np.abs(e))
    Z = np.zeros((C, K))
    for i in range(K):
        z = np.cos(np.arange(C) * (1.0 + 0.37 * i))  # deterministic, not aligned with anything
        for _ in range(iters):
            z = ldl_solve(d, e, lam[i], z, tnorm)
            z /= np.linalg.norm(z)
        Z[:, i] = z
    ortol = 1e-3 * tnorm
    start = 0
    for i in range(1, K):
        if lam[i - 1] - lam[i] >= ortol:
            start = i
            continue
        for jj in range(start, i):
            Z[:, i] -= (Z[:, jj] @ Z[:, i]) * Z[:, jj]
        Z[:, i] /= np.linalg.norm(Z[:, i])
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    sig2 = np.einsum("ij,ij->j", Z, T @ Z)
    V = Z.astype(complex)
    for k in range(C - 2, -1, -1):
        v, tau = vs[k], taus[k]
        s = v.conj() @ V[k + 1:, :]
        V[k + 1:, :] -= tau * np.outer(v, s)
    return V, np.sqrt(np.maximum(sig2, 0)), lam


def main_ldl():
    import bench
    from tools.svd32_probe import swap_theta

    for kind in ("random", "near-product"):
        for seed in range(3):
            aer = bench.bench_states(50, 64, 1 + seed, kind)[seed]
            for site in (10, 24, 37):
                T = swap_theta(aer, site)
                u, s, vh = np.linalg.svd(T)
                for iters in (2, 3):
                    V, sig, lam = gram_svd_ldl(T, 64, iters)
                    Vt = vh[:64].conj().T
                    P = V @ V.conj().T - Vt @ Vt.conj().T
                    print(kind, seed, site, iters, "sig err %.1e" % (np.max(np.abs(sig - s[:64])) / s[0]),
                          "subspace %.1e" % np.linalg.norm(P, 2),
                          "orth %.1e" % np.max(np.abs(V.conj().T @ V - np.eye(64))),
                          "minrelgap %.1e" % np.min(-np.diff(s[:65] ** 2) / s[0] ** 2))
