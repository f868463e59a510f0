"""Restatement of adaptaqc/utils/gradients.py (reference lines 23-224).

``general_grad_of_pairs_ref`` keeps the reference's structure exactly (and is the CPU
baseline): one MPS build + one whole-psi dot per (pair, generator), gradients.py:81-122.
``general_grad_of_pairs_env`` is a cross-check that evaluates the same quantities through
left/right environments of a product starting state; the tests pin it to the
reference-structured version before it is used on large inputs.

Ops are ``(name, qubits, params)`` tuples; a generator / layer is a 2-qubit op list.
"""
import numpy as np

from . import gates as G
from . import mps as M

ROT = ("rx", "ry", "rz")


def remove_unnecessary_2q_gates(ops):
    """circuit_operations_optimisation.py:167-204: cancel adjacent identical CX/CY/CZ pairs."""
    ops = list(ops)
    to_remove, dealt = [], []
    for gi in range(len(ops) - 1, -1, -1):
        name, qargs, _ = ops[gi]
        if name not in ("cx", "cy", "cz") or gi in to_remove or gi in dealt:
            continue
        # find_previous_gate_on_qubit (circuit_operations_circuit_division.py:19-42)
        req = set(qargs)
        pi = gi - 1
        while pi >= 0 and not (req & set(ops[pi][1])):
            pi -= 1
        if pi < 0 or ops[pi][0] != name:
            continue
        if pi in to_remove or pi in dealt:
            continue
        if tuple(ops[pi][1]) == tuple(qargs):
            to_remove += [gi, pi]
    for i in sorted(to_remove, reverse=True):
        del ops[i]
    return ops


def get_generator(ansatz, index, op):
    """gradients.py:173-224."""
    if op not in ROT:
        raise ValueError("op must be one of rx, ry or rz")
    gen = []
    for i, (name, qubits, _) in enumerate(ansatz):
        if name not in ("rx", "ry", "rz", "cx"):
            raise ValueError("Circuit must only contain rx, ry, rz and cx gates")
        if i == index:
            gen.append(({"rx": "x", "ry": "y", "rz": "z"}[op], (qubits[0],), ()))
        if name == "cx":
            gen.append(("cx", tuple(qubits), ()))
    return remove_unnecessary_2q_gates(gen)


def inverse_ops(ops):
    out = []
    for name, q, p in reversed(ops):
        if name in ("rx", "ry", "rz", "p", "u1"):
            out.append((name, q, (-p[0],)))
        elif name in ("x", "y", "z", "h", "cx", "cy", "cz", "swap", "id"):
            out.append((name, q, p))
        elif name == "unitary":
            out.append((name, q, (np.conj(np.asarray(p[0])).T,)))
        else:
            raise ValueError(name)
    return out


def _key(ops):
    return tuple((n, tuple(q), tuple(np.round(p, 15)) if p else ()) for n, q, p in ops)


def get_generators_and_degeneracies(ansatz, rotoselect=False, inverse=False):
    """gradients.py:127-170 with utilityfunctions.get_distinct_items_and_degeneracies (:401-426)."""
    gens = []
    for i, (name, _, _) in enumerate(ansatz):
        if name in ROT:
            for op in (ROT if rotoselect else (name,)):
                g = get_generator(ansatz, i, op)
                gens.append(inverse_ops(g) if inverse else g)
    distinct, deg = [], []
    for g in gens:
        k = _key(g)
        for j, d in enumerate(distinct):
            if _key(d) == k:
                deg[j] += 1
                break
        else:
            distinct.append(g)
            deg.append(1)
    return distinct, deg


def ops_matrix(ops):
    """4x4 unitary (little-endian over (q0, q1)) of a 2-qubit op list."""
    u = np.eye(4, dtype=complex)
    from .sv import apply_matrix

    cols = []
    for c in range(4):
        v = np.zeros(4, dtype=complex)
        v[c] = 1
        for name, q, p in ops:
            v = apply_matrix(v, 2, tuple(q), G.matrix(name, p))
        cols.append(v)
    u = np.stack(cols, axis=1)
    return u


def _compose(start_ops, ops, c, t):
    mapping = {0: c, 1: t}
    return list(start_ops) + [(n, tuple(mapping[x] for x in q), p) for n, q, p in ops]


def general_grad_of_pairs_ref(psi_mps, n, inverse_zero_ansatz, generators, degeneracies,
                              coupling_map, starting_ops=(), thr=1e-16, max_chi=None):
    """gradients.py:23-124, reference structure (per pair, per generator MPS + dot).

    ``psi_mps``: preprocessed MPS of |psi> (the reference builds it at :60-62).
    """
    resolves_to_id = np.allclose(ops_matrix(inverse_zero_ansatz), np.eye(4))
    if resolves_to_id:
        s_mps = M.run_circuit(n, list(starting_ops), thr, max_chi).preprocessed()
        zero_overlap = M.mps_dot(psi_mps, s_mps)
    out = []
    for c, t in coupling_map:
        if not resolves_to_id:
            u0s = M.run_circuit(n, _compose(starting_ops, inverse_zero_ansatz, c, t), thr, max_chi)
            zero_overlap = M.mps_dot(psi_mps, u0s.preprocessed())
        g = 0.0
        for gen, deg in zip(generators, degeneracies):
            st = M.run_circuit(n, _compose(starting_ops, gen, c, t), thr, max_chi)
            ov = M.mps_dot(st.preprocessed(), psi_mps)
            gg = -1.0 * np.imag(ov * zero_overlap)
            g += gg * gg * deg
        out.append(float(np.sqrt(g)))
    return out


def product_state_vectors(n, starting_ops):
    """Per-qubit 2-vectors of a starting circuit made only of 1-qubit gates."""
    s = [np.array([1.0, 0.0], dtype=complex) for _ in range(n)]
    for name, q, p in starting_ops:
        if len(q) != 1:
            raise ValueError("product starting state required")
        s[q[0]] = G.matrix(name, p) @ s[q[0]]
    return s


def pair_tensors_env(psi_mps, svec):
    """T[a,b][sa,sb] = <s_{not ab}, sa sb | psi> for all a<b via left/right environments."""
    n = len(psi_mps)
    m = [np.einsum("s,sij->ij", np.conj(svec[i]), psi_mps[i]) for i in range(n)]
    left = [np.ones((1,), dtype=complex)]
    for i in range(n - 1):
        left.append(left[-1] @ m[i])
    right = [None] * (n + 1)
    right[n] = np.ones((1,), dtype=complex)
    for i in range(n - 1, -1, -1):
        right[i] = m[i] @ right[i + 1]
    w = [np.stack([psi_mps[b][s] @ right[b + 1] for s in range(2)]) for b in range(n)]
    T = {}
    for a in range(n - 1):
        v = np.stack([left[a] @ psi_mps[a][s] for s in range(2)])  # (2, chi_a)
        for b in range(a + 1, n):
            T[(a, b)] = v @ w[b].T  # (2 sa, 2 sb)
            v = v @ m[b]
    return T


def bra_vectors(svec, a, b, ops_mats):
    """row vectors (s_a (x) s_b)^dagger O for each 4x4 O (basis index 2*sb + sa)."""
    s4 = np.kron(svec[b], svec[a])  # index 2*sb + sa
    return [np.conj(s4) @ o for o in ops_mats]


def general_grad_of_pairs_env(psi_mps, n, inverse_zero_ansatz, generators, degeneracies,
                              coupling_map, starting_ops=()):
    svec = product_state_vectors(n, starting_ops)
    T = pair_tensors_env(psi_mps, svec)
    u0 = ops_matrix(inverse_zero_ansatz).conj().T  # U0 = (U0^dagger)^dagger
    gmats = [ops_matrix(g).conj().T for g in generators]  # generators are given as G_k^dagger
    out = []
    for c, t in coupling_map:
        a, b = min(c, t), max(c, t)
        tab = T[(a, b)]
        # operator qubit 0 -> c, qubit 1 -> t ; T index [s_a, s_b]
        vec = np.zeros(4, dtype=complex)  # little-endian over (c, t): index 2*st + sc
        for sa in range(2):
            for sb in range(2):
                sc, st = (sa, sb) if c == a else (sb, sa)
                vec[2 * st + sc] = tab[sa, sb]
        s4 = np.kron(svec[t], svec[c])
        z = np.conj(np.conj(s4) @ u0 @ vec)  # <psi|U0^dagger|s>
        g = 0.0
        for gm, deg in zip(gmats, degeneracies):
            ov = np.conj(s4) @ gm @ vec  # <s|G_k|psi>
            gg = -np.imag(ov * z)
            g += gg * gg * deg
        out.append(float(np.sqrt(g)))
    return out
