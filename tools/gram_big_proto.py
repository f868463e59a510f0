"""Numpy model of the multi-workgroup Gram SVD (gram_big.hip) for 2 chi = C in {256, 512, 1024}.

Follows the device algorithm step for step so index and sign conventions can be checked on the
CPU: G = X^H X; zhetd2 (lower) with G's rows dealt cyclically to P workgroups, one exchange per
column carrying p (each row from its owner) and the OLD row k+1 (from its owner), from which every
workgroup forms the NEW row k+1 itself; bisection for the top K eigenvalues of T; inverse
iteration; V = Q Z by the reflectors one at a time (last first); W = V sigma.

    python tools/gram_big_proto.py [C] [K]
"""
import sys

import numpy as np


def zlarfg(alpha, xnorm):
    # LAPACK zlarfg: H^H (alpha, x) = (beta, 0), H = I - tau v v^H, v = (1, x / (alpha - beta))
    if xnorm == 0.0 and alpha.imag == 0.0:
        return 0.0 + 0.0j, alpha.real, 0.0 + 0.0j
    beta = -np.copysign(np.sqrt(abs(alpha) ** 2 + xnorm ** 2), alpha.real)
    tau = complex((beta - alpha.real) / beta, -alpha.imag / beta)
    return tau, beta, 1.0 / (alpha - beta)


def tridiag_distributed(G, P):
    C = G.shape[0]
    A = G.copy()  # each "workgroup" g holds rows r % P == g; all updates below touch only own rows
    d = np.zeros(C)
    e = np.zeros(C - 1)
    taus = np.zeros(C - 1, complex)
    Y = np.zeros((C, C), complex)  # reflector k in row k, entries c >= k + 1
    rho = A[0].copy()  # row 0 read by everyone from G
    for k in range(C - 1):
        d[k] = rho[k].real
        x = np.conj(rho)  # column k below the diagonal = conj(row k)
        alpha = x[k + 1]
        xnorm = np.sqrt(np.sum(np.abs(x[k + 2:]) ** 2))
        tau, beta, sc = zlarfg(alpha, xnorm)
        v = np.zeros(C, complex)
        v[k + 1] = 1.0
        v[k + 2:] = x[k + 2:] * sc
        e[k] = beta
        taus[k] = tau
        Y[k] = v
        # p_r = tau (A v)_r for own rows r >= k + 1 (0 for r <= k)
        p = np.zeros(C, complex)
        for g in range(P):
            rows = np.arange(g, C, P)
            rows = rows[rows >= k + 1]
            p[rows] = tau * (A[rows] @ v)
        old = A[k + 1].copy()  # published by owner(k + 1) before its update
        a2 = -0.5 * tau * np.vdot(p, v)
        w = p + a2 * v
        rho = old - v[k + 1] * np.conj(w) - w[k + 1] * np.conj(v)
        A -= np.outer(v, np.conj(w)) + np.outer(w, np.conj(v))
        assert np.allclose(rho[k + 1:], A[k + 1, k + 1:])
    d[C - 1] = rho[C - 1].real
    return d, e, taus, Y


def sturm(d, e2, x):
    # eigenvalues of T below x
    cnt = 0
    q = d[0] - x
    cnt += q < 0
    for i in range(1, len(d)):
        q = d[i] - x - e2[i - 1] / (q if q != 0 else 1e-300)
        cnt += q < 0
    return cnt


def top_eigs(d, e, K):
    C = len(d)
    e2 = e * e
    ae = np.abs(e)
    lo = np.min(d - np.r_[0, ae] - np.r_[ae, 0])
    hi = np.max(d + np.r_[0, ae] + np.r_[ae, 0])
    lam = np.zeros(K)
    for i in range(K):
        a = C - 1 - i  # ascending index
        l, h = lo, hi
        for _ in range(60):
            m = 0.5 * (l + h)
            if sturm(d, e2, m) >= a + 1:
                h = m
            else:
                l = m
        lam[i] = 0.5 * (l + h)
    return lam


def inverse_iteration(d, e, lam, tn):
    C = len(d)
    K = len(lam)
    Z = np.zeros((C, K))
    rng = np.random.default_rng(0)
    for i in range(K):
        Tm = np.diag(d - lam[i]) + np.diag(e, 1) + np.diag(e, -1)
        z = rng.uniform(-1, 1, C)
        for _ in range(3):
            try:
                z = np.linalg.solve(Tm + 1e-300 * np.eye(C), z)
            except np.linalg.LinAlgError:
                z = np.linalg.lstsq(Tm, z, rcond=None)[0]
            z /= np.linalg.norm(z)
        Z[:, i] = z
    # Gram-Schmidt inside clusters
    start = 0
    for i in range(1, K):
        if lam[i - 1] - lam[i] >= 1e-7 * tn:
            start = i
            continue
        for jj in range(start, i):
            Z[:, i] -= (Z[:, i] @ Z[:, jj]) * Z[:, jj]
        Z[:, i] /= np.linalg.norm(Z[:, i])
    return Z


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    K = int(sys.argv[2]) if len(sys.argv) > 2 else C // 2
    P = C * C // 16384
    rng = np.random.default_rng(1)
    X = rng.normal(size=(C, C)) + 1j * rng.normal(size=(C, C))
    X *= np.exp(-np.arange(C) / C * 3)[None, :]
    G = X.conj().T @ X
    d, e, taus, Y = tridiag_distributed(G, P)
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    lam = top_eigs(d, e, K)
    ref = np.sort(np.linalg.eigvalsh(G))[::-1][:K]
    print("eig rel err", np.max(np.abs(lam - ref)) / ref[0])
    tn = np.max(np.abs(d) + np.r_[0, np.abs(e)] + np.r_[np.abs(e), 0])
    Z = inverse_iteration(d, e, lam, tn).astype(complex)
    sig2 = np.einsum("ri,rs,si->i", Z.real, T, Z.real)
    # V = H_0 H_1 ... H_{C-2} Z, H_k = I - tau_k v_k v_k^H, applied last first
    V = Z.copy()
    for k in range(C - 2, -1, -1):
        v = Y[k]
        V -= taus[k] * np.outer(v, v.conj() @ V)
    res = np.linalg.norm(G @ V - V * sig2[None, :]) / np.linalg.norm(G)
    orth = np.linalg.norm(V.conj().T @ V - np.eye(K))
    print("C", C, "K", K, "P", P, "residual", res, "orth", orth)
    W = V * np.sqrt(sig2)[None, :]
    # the truncated product X V V^H vs the SVD's
    U, s, Vh = np.linalg.svd(X)
    best = (U[:, :K] * s[:K]) @ Vh[:K]
    print("truncation diff", np.linalg.norm(X @ V @ V.conj().T - best) / np.linalg.norm(best))
    print("sigma rel err", np.max(np.abs(np.sqrt(sig2) - s[:K]) / s[0]))
    del W


if __name__ == "__main__":
    main()
