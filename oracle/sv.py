"""Statevector restatement of ``AerSVBackend`` (reference adaptaqc/backends/aer_sv_backend.py).

Aer's ``statevector_simulator`` (qiskit-aer ~=0.16.0, C++ ``QubitVector``) applies each
gate matrix to the little-endian state.  The reference re-simulates the whole
``compiler.full_circuit`` from |0...0> on every cost evaluation (aer_sv_backend.py:37-47);
this restatement does the same so it doubles as the CPU baseline.
"""
import numpy as np

from . import gates as G


def ccx_matrix():
    m = np.eye(8, dtype=complex)
    # controls = qubits 0,1 (bits b0,b1); target = qubit 2 (b2): swap |011> <-> |111>
    m[[3, 7]] = m[[7, 3]]
    return m


def apply_matrix(psi, n, qubits, m):
    """Apply a k-qubit matrix (little-endian over ``qubits``) to state ``psi`` of n qubits."""
    k = len(qubits)
    t = psi.reshape([2] * n)  # axis j <-> qubit n-1-j
    axes = [n - 1 - q for q in reversed(qubits)]  # matrix row index = sum b_i 2^i, b_{k-1} most significant
    mt = m.reshape([2] * (2 * k))
    t = np.tensordot(mt, t, axes=(list(range(k, 2 * k)), axes))
    t = np.moveaxis(t, list(range(k)), axes)
    return np.ascontiguousarray(t).reshape(-1)


def gate_matrix(name, params):
    if name == "ccx":
        return ccx_matrix()
    return G.matrix(name, params)


def simulate(n, ops, psi=None):
    """Run a list of ``(name, qubits, params)`` ops on |0..0> (or ``psi``)."""
    if psi is None:
        psi = np.zeros(2 ** n, dtype=complex)
        psi[0] = 1.0
    for name, qubits, params in ops:
        if name in ("barrier", "measure"):
            continue
        psi = apply_matrix(psi, n, tuple(qubits), gate_matrix(name, params))
    return psi


def global_cost(psi):
    """``1 - |sv[0]|^2`` (aer_sv_backend.py:23-30)."""
    return 1.0 - abs(psi[0]) ** 2


def z_expectations(psi, n):
    """<Z_i> = p0 - p1 from ``sv.probabilities([i])`` for i < n (aer_sv_backend.py:49-59)."""
    p = (np.abs(psi) ** 2).reshape([2] * n)
    out = []
    for q in range(n):
        ax = n - 1 - q
        pq = p.sum(axis=tuple(a for a in range(n) if a != ax))
        out.append(float(pq[0] - pq[1]))
    return out


def local_cost(psi, n):
    """``0.5 * (1 - mean(e_vals))`` (aer_sv_backend.py:32-35)."""
    return 0.5 * (1.0 - np.mean(z_expectations(psi, n)))
