"""Oracle (test infrastructure only): the chi = 1 variational compression behind
``starting_circuit="tenpy_product_state"`` (approximate_compiler.py:222-242,
utils/utilityfunctions.py:291-385).

The reference compresses the target MPS with tenpy's variational method (physics-tenpy ~=1.0.2,
setup.py; not installed here) at ``trunc_params = {"chi_max": 1}``, ``min_sweeps = 10``,
``max_sweeps = 50``, then turns the chi = 1 MPS into one single-qubit unitary per qubit.  Restated
from the published algorithm: with every other site fixed the overlap of a product state with psi
is a bilinear form in two neighbouring site vectors, <s|psi> = sum_ab conj(s_i[a]) conj(s_{i+1}[b])
F[a][b] with F = l_i A_i[a] A_{i+1}[b] r_{i+2}, maximised by the top singular pair of the 2 x 2 F;
sweeps alternate left-to-right and right-to-left.  Parity against tenpy itself is unpinned (tenpy
is absent; its initial guess is psi itself, here the chi = 1 truncation of the canonical form);
the tests pin the device kernel to this restatement and check local optimality.
"""
import numpy as np


def initial_guess(gammas):
    """chi = 1 truncation of the canonical (Vidal) form: Gamma_i[s][0][0], normalised."""
    out = []
    for g in gammas:
        v = np.array([g[0][0, 0], g[1][0, 0]], dtype=complex)
        nn = np.linalg.norm(v)
        out.append(v / nn if nn > 0 else np.array([1.0, 0.0], dtype=complex))
    return out


def top_pair(F):
    u, s, vh = np.linalg.svd(F)
    return u[:, 0], vh[0], s[0]  # s_i = u_1, s_{i+1} = conj(v_1) = vh[0], sigma_1


def _m(a, s):
    return np.conj(s[0]) * a[0] + np.conj(s[1]) * a[1]


def product_fit(psi, svec, min_sweeps=10, max_sweeps=50, tol=1e-12):
    """psi: preprocessed MPS (list of (2, l, r)); svec: list of 2-vectors (initial guess).
    Returns (svec, fidelity |<s|psi>|^2, sweeps)."""
    n = len(psi)
    s = [np.array(x, dtype=complex) for x in svec]
    if n == 1:
        v = psi[0][:, 0, 0]
        return [v / np.linalg.norm(v)], float(np.linalg.norm(v) ** 2), 0
    prev, fid, sweep = -1.0, 0.0, 0
    for sweep in range(max_sweeps):
        r = [None] * (n + 1)
        r[n] = np.ones(1, dtype=complex)
        for k in range(n - 1, -1, -1):
            r[k] = _m(psi[k], s[k]) @ r[k + 1]
        lv = np.ones(1, dtype=complex)
        for i in range(n - 1):
            u = np.stack([lv @ psi[i][a] for a in range(2)])
            w = np.stack([psi[i + 1][b] @ r[i + 2] for b in range(2)])
            s[i], s[i + 1], sg = top_pair(u @ w.T)
            fid = sg * sg
            lv = np.conj(s[i][0]) * u[0] + np.conj(s[i][1]) * u[1]
        l = [None] * (n + 1)
        l[0] = np.ones(1, dtype=complex)
        for k in range(n):
            l[k + 1] = l[k] @ _m(psi[k], s[k])
        rv = np.ones(1, dtype=complex)
        for i in range(n - 2, -1, -1):
            u = np.stack([l[i] @ psi[i][a] for a in range(2)])
            w = np.stack([psi[i + 1][b] @ rv for b in range(2)])
            s[i], s[i + 1], sg = top_pair(u @ w.T)
            fid = sg * sg
            rv = np.conj(s[i + 1][0]) * w[0] + np.conj(s[i + 1][1]) * w[1]
        if sweep + 1 >= min_sweeps and prev >= 0.0 and abs(fid - prev) <= tol * fid:
            sweep += 1
            break
        prev = fid
    else:
        sweep = max_sweeps
    return s, float(fid), sweep


def overlap(psi, svec):
    """<s|psi> for a product state s."""
    v = np.ones(1, dtype=complex)
    for a, s in zip(psi, svec):
        v = v @ _m(a, s)
    return complex(v[0])
