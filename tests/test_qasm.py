"""qasm2_dumps unrolls gates outside qelib1 (the reference unrolls its target to basis
gates first, approximate_compiler.py:195, so compile(save_circuit_history=True) never meets one)."""
import numpy as np
import pytest

from adaptaqc_amd import gates as G
from adaptaqc_amd.circuit import QuantumCircuit, qasm2_dumps, u3_params, unroll_two_qubit


def _haar(d, rng):
    z = (rng.standard_normal((d, d)) + 1j * rng.standard_normal((d, d))) / np.sqrt(2)
    q, r = np.linalg.qr(z)
    return q * (np.diag(r) / abs(np.diag(r)))


def _piece(name, params):
    if name == "cu3":
        m = np.eye(4, dtype=complex)
        m[np.ix_([1, 3], [1, 3])] = G.u3(*params)
        return m
    return G.one_qubit(name, params) if name in ("u3", "u1", "ry", "rz") else G.two_qubit(name, params)


def _product(pieces):
    swap = G.TWO_QUBIT["swap"]
    out = np.eye(4, dtype=complex)
    for name, params, qs in pieces:
        m = _piece(name, params)
        if len(qs) == 1:
            m = G.kron_le(m, np.eye(2)) if qs[0] == 0 else G.kron_le(np.eye(2), m)
        elif qs == (1, 0):
            m = swap @ m @ swap
        out = m @ out
    return out


def _equal_up_to_phase(a, b):
    k = np.argmax(abs(b))
    ph = a.flat[k] / b.flat[k]
    assert abs(abs(ph) - 1) < 1e-10
    np.testing.assert_allclose(a, ph * b, atol=1e-10)


@pytest.mark.parametrize("seed", range(6))
def test_u3_params_reconstruct(seed):
    rng = np.random.default_rng(seed)
    for v in (_haar(2, rng), np.diag(np.exp(1j * rng.uniform(-3, 3, 2))), G.PAULI["x"] * np.exp(0.3j), G.PAULI["y"]):
        t, p, l, a = u3_params(v)
        np.testing.assert_allclose(np.exp(1j * a) * G.u3(t, p, l), v, atol=1e-12)


@pytest.mark.parametrize("seed", range(8))
def test_two_qubit_unroll_reconstructs(seed):
    rng = np.random.default_rng(100 + seed)
    cases = [_haar(4, rng), G.TWO_QUBIT["swap"], G.two_qubit("rzz", (0.7,)), np.eye(4, dtype=complex),
             G.kron_le(_haar(2, rng), _haar(2, rng))]
    for u in cases:
        _equal_up_to_phase(_product(unroll_two_qubit(u)), u)


def test_qasm2_dumps_unrolls_non_standard_gates():
    rng = np.random.default_rng(7)
    u = _haar(4, rng)
    qc = QuantumCircuit(3).rx(0.5, 0).cx(0, 1)
    qc.unitary(u, [2, 0])
    qc.unitary(_haar(2, rng), [1])
    text = qasm2_dumps(qc)
    body = text.splitlines()[3:]
    assert body[:2] == ["rx(0.5) q[0];", "cx q[0],q[1];"]
    names = {ln.split("(")[0].split(" ")[0] for ln in body}
    assert names <= {"rx", "cx", "u3", "u1", "cu3", "ry", "cry"}
    # the two-qubit unitary's pieces on (q2, q0) rebuild it
    pieces = unroll_two_qubit(u)
    assert len(body) == 2 + len(pieces) + 1
    assert body[2].endswith("q[2];") and "cu3" in body[4] and body[4].endswith("q[0],q[2];")
