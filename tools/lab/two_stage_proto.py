"""Two-stage Hermitian tridiagonalisation, numpy prototype (the index map of gram_big.hip's
two-stage path).

Stage 1 (dense -> band, bandwidth b): panel p (columns c0 = b p .. c0 + b - 1) is QR-factored below
the band -- rows r0 = c0 + b .. C - 1 -- by b Householder reflectors (zgeqr2: H_i = I - tau_i v_i v_i^H,
v_i[i] = 1, zero above), Q_p = H_0 ... H_{b-1} = I - V T V^H (zlarft); the panel becomes [R; 0] and
the trailing block A22 = A[r0:, r0:] becomes Q_p^H A22 Q_p = A22 - V W^H - W V^H with
X = A22 V T, W = X - V (T^H (V^H X)) / 2.

Stage 2 (band -> tridiagonal, one column per sweep): sweep j annihilates column j below its
subdiagonal with a reflector on rows j + 1 .. j + b, then chases the fill: step s cleans the first
column of the previous window (rows below window + b) with a reflector on the next b rows.

Checks: T's eigenvalues equal G's, Q = Q1 Q2 unitary with G = Q T Q^H, and the nonzero extents the
kernels assume (printed).
"""
import sys

import numpy as np


def house(x):
    """zlarfg: H = I - tau v v^H, v[0] = 1, H^H x = beta e1 with beta real."""
    alpha = x[0]
    xn2 = float(np.vdot(x[1:], x[1:]).real) if len(x) > 1 else 0.0
    v = np.zeros_like(x)
    v[0] = 1.0
    if xn2 == 0.0 and alpha.imag == 0.0:
        return v, 0.0 + 0j, alpha.real
    nrm = np.sqrt(abs(alpha) ** 2 + xn2)
    beta = -nrm if alpha.real >= 0 else nrm
    tau = complex((beta - alpha.real) / beta, -alpha.imag / beta)
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def stage1(G, b):
    A = G.copy()
    C = A.shape[0]
    panels = []
    for c0 in range(0, C - b, b):
        r0 = c0 + b
        m = C - r0
        P = A[r0:, c0:c0 + b].copy()
        nb = min(b, m)
        V = np.zeros((m, b), complex)
        taus = np.zeros(b, complex)
        for i in range(nb):
            v, tau, beta = house(P[i:, i].copy())
            V[i:, i] = v
            taus[i] = tau
            # H^H P (zgeqr2 applies H^H = I - conj(tau) v v^H from the left)
            P[i:, i:] -= np.conj(tau) * np.outer(v, v.conj() @ P[i:, i:])
        # zlarft (forward, columnwise): Q = H_0 ... H_{nb-1} = I - V T V^H
        T = np.zeros((b, b), complex)
        for i in range(nb):
            T[i, i] = taus[i]
            if i:
                T[:i, i] = -taus[i] * T[:i, :i] @ (V[:, :i].conj().T @ V[:, i])
        Q = np.eye(m) - V @ T @ V.conj().T
        assert np.allclose(Q.conj().T @ A[r0:, c0:c0 + b], np.triu(P), atol=1e-10)
        A[r0:, c0:c0 + b] = np.triu(P)
        A[c0:c0 + b, r0:] = np.triu(P).conj().T
        A22 = A[r0:, r0:]
        X = A22 @ V @ T
        W = X - 0.5 * V @ (T.conj().T @ (V.conj().T @ X))
        A[r0:, r0:] = A22 - V @ W.conj().T - W @ V.conj().T
        panels.append((r0, V, T))
    return A, panels


def stage2(B, b, log=None):
    """Band (Hermitian, full storage here) -> tridiagonal; returns T's d, e (complex) and the
    reflectors (row start, v, tau) in application order."""
    A = B.copy()
    C = A.shape[0]
    refl = []
    for j in range(C - 2):
        col, rs = j, j + 1
        while True:
            re = min(rs + b - 1, C - 1)
            if re - rs < 1:
                break
            x = A[rs:re + 1, col].copy()
            v, tau, beta = house(x)
            # extents the kernels assume: nonzeros of the window rows / columns
            if log is not None:
                rows = np.nonzero(np.abs(A[rs:re + 1, :]) > 0)[1]
                cols = np.nonzero(np.abs(A[:, rs:re + 1]) > 0)[0]
                log.append((j, rs, col, rows.min() - rs, rows.max() - rs, cols.min() - rs, cols.max() - rs))
            Hh = np.eye(re - rs + 1) - np.conj(tau) * np.outer(v, v.conj())  # H^H
            A[rs:re + 1, :] = Hh @ A[rs:re + 1, :]
            A[:, rs:re + 1] = A[:, rs:re + 1] @ Hh.conj().T
            A[rs + 1:re + 1, col] = 0
            A[col, rs + 1:re + 1] = 0
            refl.append((rs, v, tau))
            col, rs = rs, re + 1
            if rs >= C:
                break
    return A, refl


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rng = np.random.default_rng(1)
    X = rng.standard_normal((C, C)) + 1j * rng.standard_normal((C, C))
    G = X.conj().T @ X
    A1, panels = stage1(G, b)
    band = np.abs(np.subtract.outer(np.arange(C), np.arange(C))) > b
    print("stage 1: max |entry| outside the band", np.abs(A1[band]).max())
    A1[band] = 0
    log = []
    T, refl = stage2(A1, b, log)
    tri = np.abs(np.subtract.outer(np.arange(C), np.arange(C))) > 1
    print("stage 2: max |entry| outside tridiagonal", np.abs(T[tri]).max(), "reflectors", len(refl))
    ev = np.linalg.eigvalsh(G)
    et = np.linalg.eigvalsh(T)
    print("eigenvalues: max rel diff", np.abs(ev - et).max() / ev.max())
    # Q = Q1 Q2: G = Q T Q^H
    Q = np.eye(C, dtype=complex)
    for r0, V, Tf in panels:
        Qp = np.eye(C, dtype=complex)
        Qp[r0:, r0:] -= V @ Tf @ V.conj().T
        Q = Q @ Qp
    for rs, v, tau in refl:
        H = np.eye(C, dtype=complex)
        H[rs:rs + len(v), rs:rs + len(v)] -= tau * np.outer(v, v.conj())
        Q = Q @ H
    print("G = Q T Q^H:", np.abs(Q @ T @ Q.conj().T - G).max() / np.abs(G).max(),
          "unitary:", np.abs(Q.conj().T @ Q - np.eye(C)).max())
    lg = np.array(log)
    print("window-row extent rel. rs: [%d, %d]; window-column extent: [%d, %d]"
          % (lg[:, 3].min(), lg[:, 4].max(), lg[:, 5].min(), lg[:, 6].max()))
    print("col - rs:", sorted(set((lg[:, 2] - lg[:, 1]).tolist())))
    # eigenvectors: G z = lam z  <=>  T (Q^H z) = lam (Q^H z)
    w, Z = np.linalg.eigh(T)
    V = Q @ Z
    print("eigvec residual", np.abs(G @ V - V * w).max() / np.abs(G).max())


if __name__ == "__main__":
    main()
