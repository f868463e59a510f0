"""Host-side circuit -> aqc_op_t conversion (no GPU): the vectorised ``_lib.ops_array`` and the
per-circuit memo of ``circuit.device_ops_array`` against the plain per-op conversion, through the
edits ADAPT-AQC makes between evaluations (an angle rewritten in place, a layer appended, gates
removed or replaced) -- the rows must equal a fresh conversion byte for byte every time."""
import gc

import numpy as np

from adaptaqc_amd import _lib
from adaptaqc_amd import circuit as C
from adaptaqc_amd.circuit import CircuitInstruction, Operation, QuantumCircuit, device_ops, device_ops_array


def _old_ops_array(ops):
    arr = np.zeros(len(ops), dtype=_lib.OP_DTYPE)
    for i, (m, qubits) in enumerate(ops):
        m = np.asarray(m, dtype=np.complex128).reshape(-1)
        arr[i]["nq"] = len(qubits)
        arr[i]["q0"] = qubits[0]
        arr[i]["q1"] = qubits[1] if len(qubits) == 2 else 0
        arr[i]["m"][: 2 * m.size : 2] = m.real
        arr[i]["m"][1 : 2 * m.size : 2] = m.imag
    return arr


def _brickwork(n, depth, seed):
    rng = np.random.default_rng(seed)
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            getattr(qc, ("rx", "ry", "rz")[rng.integers(3)])(rng.uniform(-np.pi, np.pi), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    return qc


def _fresh(qc, start=0):
    return _lib.ops_array(device_ops(qc, start)).tobytes()


def test_ops_array_matches_per_op_fill():
    qc = _brickwork(8, 4, 1)
    qc.ccx(0, 1, 2)
    ops = device_ops(qc)
    assert _lib.ops_array(ops).tobytes() == _old_ops_array(ops).tobytes()
    assert _lib.ops_array([]).shape == (0,)


def test_device_ops_array_memo_follows_edits():
    qc = _brickwork(10, 6, 2)
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    assert device_ops_array(qc).tobytes() == _fresh(qc)  # memo hit
    qc.data[5].operation.params[0] += 0.25  # Rotosolve: one angle in place
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    qc.rz(0.1, 3)  # a layer appended
    qc.cx(3, 4)
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    del qc.data[7]  # a gate removed: every later row shifts
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    qc.data[2] = CircuitInstruction(Operation("ry", 1, [0.7]), (9,))  # replaced on another qubit
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    qc.data[4] = CircuitInstruction(Operation(qc.data[4].operation.name, 1, list(qc.data[4].operation.params)),
                                    (qc.data[4].qubits[0] ^ 1,))  # same gate, other qubit
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    assert device_ops_array(qc, 11).tobytes() == _fresh(qc, 11)  # another start: rebuilt
    assert device_ops_array(qc).tobytes() == _fresh(qc)


def test_device_ops_array_skips_and_decomposes():
    qc = QuantumCircuit(4)
    qc.h(0)
    qc.barrier()
    qc.ccx(0, 1, 2)
    u = np.linalg.qr(np.random.default_rng(3).standard_normal((4, 4)) + 0j)[0]
    qc.append(Operation("unitary", 2, [u]), (1, 3))
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    qc.data[-1].operation.params[0] = u.conj().T  # a matrix parameter: never reused stale
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    empty = QuantumCircuit(2)
    assert device_ops_array(empty).shape == (0,) and device_ops_array(empty).dtype == _lib.OP_DTYPE


def test_device_ops_array_memo_released_with_circuit():
    qc = _brickwork(6, 2, 4)
    device_ops_array(qc)
    key = id(qc)
    assert key in C._OPS_MEMO
    del qc
    gc.collect()
    assert key not in C._OPS_MEMO


class _CustomGate:
    """A qiskit-shaped custom gate: a non-standard name, no parameters, its matrix from
    to_matrix() (two instances with the same name can hold different matrices)."""

    def __init__(self, name, mat):
        self.name = name
        self.num_qubits = 1
        self.params = []
        self._m = np.asarray(mat, dtype=complex)

    def to_matrix(self):
        return self._m


class _SubclassedRz(Operation):
    pass


def test_memo_reconverts_custom_gates_and_other_types():
    qc = _brickwork(4, 2, 3)
    qc.data.append(CircuitInstruction(_CustomGate("mygate", [[0, 1], [1, 0]]), (1,)))
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    # the same name at the same index with another matrix: must not reuse the memoised rows
    qc.data[-1] = CircuitInstruction(_CustomGate("mygate", [[1, 0], [0, -1]]), (1,))
    assert device_ops_array(qc).tobytes() == _fresh(qc)
    assert C._params_snapshot(qc.data[-1].operation) is None
    # a standard gate swapped for an object of another type with equal name and parameters
    op = qc.data[0].operation
    qc.data[0] = CircuitInstruction(_SubclassedRz(op.name, 1, list(op.params)), qc.data[0].qubits)
    assert device_ops_array(qc).tobytes() == _fresh(qc)


def test_device_ops_rows_slices_the_memo():
    """circuit.device_ops_rows (the cached MPS evaluator's suffix): the rows of any instruction range
    equal a direct conversion of that range, also after an angle is rewritten in place, a gate
    replaced and instructions inserted (every op, a ccx's several rows included)."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops_rows
    from adaptaqc_amd.utils.cached_rotations import _ops

    rng = np.random.default_rng(0)
    qc = QuantumCircuit(6)
    for layer in range(5):
        for q in range(6):
            qc.rz(float(rng.uniform()), q)
            qc.ry(float(rng.uniform()), q)
        for q in range(layer % 2, 5, 2):
            qc.cx(q, q + 1)
    qc.ccx(0, 2, 4)

    def same(lo, hi):
        assert device_ops_rows(qc, lo, hi).tobytes() == _lib.ops_array(_ops(qc, lo, hi)).tobytes()

    for lo, hi in [(0, len(qc.data)), (3, 17), (20, len(qc.data)), (len(qc.data) - 2, len(qc.data)), (9, 9)]:
        same(lo, hi)
    qc.data[5].operation.params = [0.77]
    same(2, 30)
    other = QuantumCircuit(6)
    other.rx(0.4, 3)
    qc.data[7] = other.data[0]
    same(0, len(qc.data))
    qc.cx(1, 2)
    same(10, len(qc.data))
