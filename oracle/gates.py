"""Gate matrices in Qiskit conventions (restated; qiskit ~=1.3.1 is absent).

Multi-qubit matrices act on the little-endian basis of their own qubit arguments:
for a gate applied to qubits (q0, q1) the matrix row/column index is 2*b1 + b0,
where b0 is the bit of q0 (Qiskit ``Operator`` convention).  ``cx(c, t)`` therefore
has the control on the least significant bit.
"""
import numpy as np

_S2 = 1.0 / np.sqrt(2.0)


def rx(t):
    c, s = np.cos(t / 2), np.sin(t / 2)
    return np.array([[c, -1j * s], [-1j * s, c]], dtype=complex)


def ry(t):
    c, s = np.cos(t / 2), np.sin(t / 2)
    return np.array([[c, -s], [s, c]], dtype=complex)


def rz(t):
    return np.array([[np.exp(-0.5j * t), 0], [0, np.exp(0.5j * t)]], dtype=complex)


def u3(theta, phi, lam):
    c, s = np.cos(theta / 2), np.sin(theta / 2)
    return np.array(
        [[c, -np.exp(1j * lam) * s], [np.exp(1j * phi) * s, np.exp(1j * (phi + lam)) * c]],
        dtype=complex,
    )


FIXED_1Q = {
    "id": np.eye(2, dtype=complex),
    "x": np.array([[0, 1], [1, 0]], dtype=complex),
    "y": np.array([[0, -1j], [1j, 0]], dtype=complex),
    "z": np.array([[1, 0], [0, -1]], dtype=complex),
    "h": np.array([[_S2, _S2], [_S2, -_S2]], dtype=complex),
    "s": np.array([[1, 0], [0, 1j]], dtype=complex),
    "sdg": np.array([[1, 0], [0, -1j]], dtype=complex),
    "t": np.array([[1, 0], [0, np.exp(0.25j * np.pi)]], dtype=complex),
    "tdg": np.array([[1, 0], [0, np.exp(-0.25j * np.pi)]], dtype=complex),
    "sx": 0.5 * np.array([[1 + 1j, 1 - 1j], [1 - 1j, 1 + 1j]], dtype=complex),
}


def controlled(u):
    """Controlled-u with control = first qubit argument (LSB)."""
    m = np.eye(4, dtype=complex)
    # indices with b0 (control) = 1 : 1 (b1=0) and 3 (b1=1)
    m[np.ix_([1, 3], [1, 3])] = u
    return m


SWAP = np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=complex)
CX = controlled(FIXED_1Q["x"])
CY = controlled(FIXED_1Q["y"])
CZ = controlled(FIXED_1Q["z"])


def matrix(name, params=()):
    """Return the unitary of a named gate (1- or 2-qubit)."""
    if name in FIXED_1Q:
        return FIXED_1Q[name]
    if name == "rx":
        return rx(params[0])
    if name == "ry":
        return ry(params[0])
    if name == "rz":
        return rz(params[0])
    if name in ("p", "u1"):
        return np.array([[1, 0], [0, np.exp(1j * params[0])]], dtype=complex)
    if name in ("u", "u3"):
        return u3(*params)
    if name == "u2":
        return u3(np.pi / 2, params[0], params[1])
    if name == "cx":
        return CX
    if name == "cy":
        return CY
    if name == "cz":
        return CZ
    if name == "swap":
        return SWAP
    if name == "unitary":
        return np.asarray(params[0], dtype=complex)
    raise ValueError(f"unsupported gate {name}")
