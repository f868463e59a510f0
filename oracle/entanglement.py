"""CPU restatement of the ISL entanglement path (test infrastructure only -- never imported by the
product).

Follows adaptaqc/utils/entanglement_measures.py:
  * partial_trace (SV)      :326-340 (qiskit.quantum_info.partial_trace: remaining qubits in
                            ascending order, little-endian -> index = 2*bit(max) + bit(min))
  * concurrence             :278-296 (eig of rho * rho_tilde, clip, sort, C = l1-l2-l3-l4)
  * eof                     :263-275
  * negativity / log-neg.   :299-306 (partial_transpose :343-356, trace_norm :359-369)
and the MPS two-qubit reduced density matrix of aqc_research.mps_operations.partial_trace
(un-vendored; its semantics are pinned by the reference's SV == MPS test,
test_entanglement_measures.py:93-112): a plain contraction of the preprocessed MPS
(A_i = Gamma_i lambda_{i+1}) with every site but a, b traced -- no canonical form assumed.
"""
import itertools

import numpy as np
import scipy.linalg as sla

SIGMA_Y = np.array([[0, -1j], [1j, 0]])
SY_SY = np.kron(SIGMA_Y, SIGMA_Y)

METHODS = ("concurrence", "eof", "negativity", "log_negativity")


def partial_trace_sv(psi, a, b):
    """4x4 RDM of qubits a, b; row index = 2*bit(max(a,b)) + bit(min(a,b))."""
    n = int(round(np.log2(len(psi))))
    lo, hi = min(a, b), max(a, b)
    t = np.asarray(psi).reshape([2] * n)  # axis k <-> qubit n-1-k (little-endian)
    keep = [n - 1 - hi, n - 1 - lo]
    rest = [k for k in range(n) if k not in keep]
    m = np.transpose(t, keep + rest).reshape(4, -1)
    return m @ m.conj().T


def mps_rdm(pre, a, b):
    """4x4 RDM of qubits a < b from a preprocessed MPS [(2, chi_l, chi_r)] by direct contraction."""
    a, b = min(a, b), max(a, b)
    n = len(pre)
    L = np.ones((1, 1), complex)  # L[bra][ket]
    for i in range(a):
        L = sum(pre[i][s].conj().T @ L @ pre[i][s] for s in range(2))
    R = np.ones((1, 1), complex)  # R[ket][bra]
    for i in range(n - 1, b, -1):
        R = sum(pre[i][s] @ R @ pre[i][s].conj().T for s in range(2))
    # E[sb_bra][s_ket] = A_a^{s_bra dag} L A_a^{s_ket}
    E = [[pre[a][sb].conj().T @ L @ pre[a][s] for s in range(2)] for sb in range(2)]
    for i in range(a + 1, b):
        E = [[sum(pre[i][t].conj().T @ E[sb][s] @ pre[i][t] for t in range(2)) for s in range(2)] for sb in range(2)]
    rho = np.zeros((4, 4), complex)
    for sa, sab, sbk, sbb in itertools.product(range(2), repeat=4):
        # rho[(ket sa, ket sbk), (bra sab, bra sbb)] = Tr(A_b^{sbb dag} E[sab][sa] A_b^{sbk} R)
        val = np.trace(pre[b][sbb].conj().T @ E[sab][sa] @ pre[b][sbk] @ R)
        rho[2 * sbk + sa, 2 * sbb + sab] = val
    return rho


def concurrence(rho):
    rho_t = SY_SY @ rho.conjugate() @ SY_SY
    ev = sla.eig(rho @ rho_t, left=False, right=False)
    if not np.allclose(np.imag(ev), 0):
        return 0.0
    lam = sorted(np.sqrt(np.real(ev).clip(min=0)), reverse=True)
    return float(max(0.0, lam[0] - lam[1] - lam[2] - lam[3]))


def eof(rho):
    c = concurrence(rho)
    if c == 0:
        return 0.0
    x = 0.5 * (1 + np.sqrt(1 - c ** 2))
    return float(-x * np.log2(x) - (1 - x) * np.log2(1 - x))


def partial_transpose(rho, wrt=1):
    tp = rho.copy()
    for ja, ka, jb, kb in itertools.product(range(2), repeat=4):
        if wrt == 1:
            tp[ka * 2 + jb][ja * 2 + kb] = rho[ja * 2 + jb][ka * 2 + kb]
        else:
            tp[ja * 2 + kb][ka * 2 + jb] = rho[ja * 2 + jb][ka * 2 + kb]
    return tp


def trace_norm(m):
    return float(np.real(np.trace(sla.sqrtm(m @ m.conj().T))))


def negativity(rho):
    return (trace_norm(partial_transpose(rho)) - 1) / 2


def log_negativity(rho):
    return float(np.log2(trace_norm(partial_transpose(rho))))


def measure(method, rho):
    return {"concurrence": concurrence, "eof": eof, "negativity": negativity,
            "log_negativity": log_negativity}[method](rho)
