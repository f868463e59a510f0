"""Gate matrices in Qiskit conventions (qiskit ~=1.3.1 is not a dependency of this package).

A k-qubit matrix acts on the little-endian basis of its own qubit arguments: for qubits
(q0, q1) the row/column index is 2*b1 + b0 with b0 the bit of q0.
"""
import numpy as np

_R2 = 1.0 / np.sqrt(2.0)

PAULI = {
    "x": np.array([[0, 1], [1, 0]], dtype=complex),
    "y": np.array([[0, -1j], [1j, 0]], dtype=complex),
    "z": np.array([[1, 0], [0, -1]], dtype=complex),
}

CONST_1Q = {
    "id": np.eye(2, dtype=complex),
    **PAULI,
    "h": np.array([[_R2, _R2], [_R2, -_R2]], dtype=complex),
    "s": np.diag([1, 1j]).astype(complex),
    "sdg": np.diag([1, -1j]).astype(complex),
    "t": np.diag([1, np.exp(0.25j * np.pi)]).astype(complex),
    "tdg": np.diag([1, np.exp(-0.25j * np.pi)]).astype(complex),
    "sx": 0.5 * np.array([[1 + 1j, 1 - 1j], [1 - 1j, 1 + 1j]], dtype=complex),
    "sxdg": 0.5 * np.array([[1 - 1j, 1 + 1j], [1 + 1j, 1 - 1j]], dtype=complex),
}

ROTATIONS = ("rx", "ry", "rz")


def u3(theta, phi, lam):
    c, s = np.cos(theta / 2), np.sin(theta / 2)
    return np.array(
        [[c, -np.exp(1j * lam) * s], [np.exp(1j * phi) * s, np.exp(1j * (phi + lam)) * c]], dtype=complex
    )


def one_qubit(name, params=()):
    if name in CONST_1Q:
        return CONST_1Q[name]
    if name == "rx":
        c, s = np.cos(params[0] / 2), np.sin(params[0] / 2)
        return np.array([[c, -1j * s], [-1j * s, c]], dtype=complex)
    if name == "ry":
        c, s = np.cos(params[0] / 2), np.sin(params[0] / 2)
        return np.array([[c, -s], [s, c]], dtype=complex)
    if name == "rz":
        return np.diag([np.exp(-0.5j * params[0]), np.exp(0.5j * params[0])])
    if name in ("p", "u1"):
        return np.diag([1.0, np.exp(1j * params[0])]).astype(complex)
    if name in ("u", "u3"):
        return u3(*params)
    if name == "u2":
        return u3(np.pi / 2, params[0], params[1])
    raise ValueError(f"unsupported 1-qubit gate {name!r}")


def _controlled(u):
    m = np.eye(4, dtype=complex)
    m[np.ix_([1, 3], [1, 3])] = u
    return m


TWO_QUBIT = {
    "cx": _controlled(PAULI["x"]),
    "cy": _controlled(PAULI["y"]),
    "cz": _controlled(PAULI["z"]),
    "swap": np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=complex),
}


def two_qubit(name, params=()):
    if name in TWO_QUBIT:
        return TWO_QUBIT[name]
    if name == "crx":
        return _controlled(one_qubit("rx", params))
    if name == "cry":
        return _controlled(one_qubit("ry", params))
    if name == "crz":
        return _controlled(one_qubit("rz", params))
    if name in ("cp", "cu1"):
        return _controlled(one_qubit("p", params))
    if name == "rzz":
        t = params[0]
        return np.diag([np.exp(-0.5j * t), np.exp(0.5j * t), np.exp(0.5j * t), np.exp(-0.5j * t)])
    raise ValueError(f"unsupported 2-qubit gate {name!r}")


def kron_le(*mats):
    """Little-endian tensor product: kron_le(U_q0, U_q1) acts with U_q0 on bit 0."""
    out = np.eye(1, dtype=complex)
    for m in mats:
        out = np.kron(m, out)
    return out
