# (C) Copyright IBM 2025.
#
# This code is licensed under the Apache License, Version 2.0. You may
# obtain a copy of this license in the LICENSE.txt file in the root directory
# of this source tree or at http://www.apache.org/licenses/LICENSE-2.0.
#
# Any modifications or derivative works of this code must retain this
# copyright notice, and modified files need to carry a notice indicating
# that they have been altered from the originals.
#
# Modified for adaptaqc_amd: this file restates the reference file named in its docstring
# (qiskit-community/adapt-aqc) on top of the MI355X engine (libaqchip); it has been altered
# from the original.

"""Circuit surgery helpers used by the compilers (reference utils/circuit_operations/*).

Host-only list manipulation on ``adaptaqc_amd.circuit.QuantumCircuit``; no simulation here
except ``calculate_overlap_between_circuits`` which runs on the device statevector engine.
"""
import numpy as np

from ..circuit import CircuitInstruction, Operation, QuantumCircuit

SUPPORTED_1Q_GATES = ["rx", "ry", "rz"]
SUPPORTED_2Q_GATES = ["cx", "cz"]
MINIMUM_ROTATION_ANGLE = 1e-3


def create_1q_gate(gate_name, angle):
    if gate_name not in SUPPORTED_1Q_GATES:
        raise ValueError(f"Unsupported gate {gate_name}")
    return Operation(gate_name, 1, [angle], label=gate_name)


def is_supported_1q_gate(gate):
    if not isinstance(gate, Operation):
        return False
    name = gate.label if gate.label is not None else gate.name
    if "@" in name:
        return False
    return name.split("#")[0] in SUPPORTED_1Q_GATES


def add_gate(circuit, gate, gate_index=None, qubit_indexes=None):
    if gate_index is None:
        gate_index = len(circuit.data)
    circuit.data.insert(gate_index, CircuitInstruction(gate, qubit_indexes or []))


def replace_1q_gate(circuit, gate_index, gate_name, angle):
    """circuit_operations_basic.py:70-110."""
    if gate_name is None:
        return
    qargs = circuit.data[gate_index].qubits
    circuit.data[gate_index] = CircuitInstruction(create_1q_gate(gate_name, angle), qargs)


def add_dressed_cnot(circuit, control, target, thinly_dressed=False, gate_index=None, v1=True, v2=True, v3=True,
                     v4=True):
    """circuit_operations_basic.py:135-189: rz (ry rz) on each qubit, cx, again."""
    if gate_index is None:
        gate_index = len(circuit.data)

    def rot(q, loc):
        add_gate(circuit, create_1q_gate("rz", 0), loc, [q])
        loc += 1
        if not thinly_dressed:
            add_gate(circuit, create_1q_gate("ry", 0), loc, [q])
            add_gate(circuit, create_1q_gate("rz", 0), loc + 1, [q])
            loc += 2
        return loc

    if v1:
        gate_index = rot(control, gate_index)
    if v2:
        gate_index = rot(target, gate_index)
    add_gate(circuit, Operation("cx", 2), gate_index, [control, target])
    gate_index += 1
    if v3:
        gate_index = rot(control, gate_index)
    if v4:
        rot(target, gate_index)


def add_to_circuit(original, to_add, location=None, qubit_subset=None):
    """Insert ``to_add``'s gates at ``location`` (qubit i of to_add -> qubit_subset[i])."""
    if location is None:
        location = len(original.data)
    # a dict maps only the qubits the gates use (the general-initial-state circuit has 2n qubits,
    # its variational gates act on the first n)
    mapping = (lambda q: q) if qubit_subset is None else (lambda q: qubit_subset[q])
    for k, ins in enumerate(to_add.data):
        op = ins.operation.copy()
        if op.label is None and op.name in SUPPORTED_1Q_GATES:
            op.label = op.name
        original.data.insert(location + k, CircuitInstruction(op, [mapping(q) for q in ins.qubits]))


def extract_inner_circuit(circuit, gate_range):
    inner = QuantumCircuit(circuit.num_qubits)
    inner.data = [circuit.data[i] for i in range(*gate_range)]
    return inner


def remove_inner_circuit(circuit, gate_range):
    del circuit.data[gate_range[0]:gate_range[1]]


def replace_inner_circuit(circuit, replacement, gate_range):
    remove_inner_circuit(circuit, gate_range)
    if replacement is not None and len(replacement.data) > 0:
        add_to_circuit(circuit, replacement, gate_range[0])


def circuit_by_inverting_circuit(circuit):
    """circuit_operations_full_circuit.py:364-382 (labels kept, rotation angles negated)."""
    out = QuantumCircuit(circuit.num_qubits)
    for ins in reversed(circuit.data):
        op = ins.operation
        if op.label in SUPPORTED_1Q_GATES:
            inv = op.copy()
            inv.params[0] *= -1
        else:
            inv = op.inverse()
            inv.label = op.label
        out.data.append(CircuitInstruction(inv, ins.qubits))
    return out


def find_num_gates(circuit, gate_range=None):
    """(num_2q_gates, num_1q_gates) over ``gate_range``."""
    if circuit is None:
        return 0, 0
    if gate_range is None:
        gate_range = (0, len(circuit.data))
    n2 = n1 = 0
    for i in range(*gate_range):
        ins = circuit.data[i]
        if ins.operation.name in ("set_matrix_product_state", "barrier", "measure"):
            continue
        if len(ins.qubits) >= 2:
            n2 += 1
        elif len(ins.qubits) == 1:
            n1 += 1
    return n2, n1


def find_angles_in_circuit(circuit, gate_range=None):
    if gate_range is None:
        gate_range = (0, len(circuit.data))
    return [circuit.data[i].operation.params[0] for i in range(*gate_range)
            if is_supported_1q_gate(circuit.data[i].operation)]


def update_angles_in_circuit(circuit, angles, gate_range=None):
    if gate_range is None:
        gate_range = (0, len(circuit.data))
    k = 0
    for i in range(*gate_range):
        op = circuit.data[i].operation
        if is_supported_1q_gate(op):
            op.params[0] = float(angles[k])
            k += 1


def zyz_angles(u):
    """(theta, phi, lam) with u = e^{i g} Rz(phi) Ry(theta) Rz(lam) (OneQubitEulerDecomposer)."""
    u = np.asarray(u, dtype=complex)
    det = np.linalg.det(u)
    v = u / np.sqrt(det)
    theta = 2 * np.arctan2(abs(v[1, 0]), abs(v[0, 0]))
    phiplam = 2 * np.angle(v[1, 1])
    phimlam = 2 * np.angle(v[1, 0])
    return theta, (phiplam + phimlam) / 2, (phiplam - phimlam) / 2


def _prev_on_qubit(circuit, gi):
    req = set(circuit.data[gi].qubits)
    i = gi - 1
    while i >= 0:
        if req & set(circuit.data[i].qubits):
            return circuit.data[i].operation, i
        i -= 1
    return None, None


def remove_unnecessary_1q_gates_from_circuit(circuit, remove_zero_gates=True, remove_small_gates=False,
                                             gate_range=None, min_rotation_angle=MINIMUM_ROTATION_ANGLE):
    """circuit_operations_optimisation.py:73-164."""
    if gate_range is None:
        gate_range = (0, len(circuit.data))
    to_remove, dealt = [], []
    for gi in range(gate_range[1] - 1, gate_range[0] - 1, -1):
        gate = circuit.data[gi].operation
        if gi in to_remove or gi in dealt or not is_supported_1q_gate(gate):
            continue
        if (remove_zero_gates and gate.params[0] == 0) or (
                remove_small_gates and abs(gate.params[0]) < min_rotation_angle):
            to_remove.append(gi)
            continue
        matrix = gate.to_matrix()
        idxs = [gi]
        pg, pi = _prev_on_qubit(circuit, gi)
        while pg is not None and is_supported_1q_gate(pg) and pi >= gate_range[0]:
            if (remove_zero_gates and pg.params[0] == 0) or (
                    remove_small_gates and abs(pg.params[0]) < min_rotation_angle):
                to_remove.append(pi)
            else:
                idxs.append(pi)
                matrix = matrix @ pg.to_matrix()
            pg, pi = _prev_on_qubit(circuit, pi)
        if len(idxs) > 3:
            theta, phi, lam = zyz_angles(matrix)
            replace_1q_gate(circuit, idxs[0], "rz", phi)
            replace_1q_gate(circuit, idxs[1], "ry", theta)
            replace_1q_gate(circuit, idxs[2], "rz", lam)
            dealt += [idxs[1], idxs[2]]
            to_remove += idxs[3:]
        else:
            dealt += idxs
    for i in sorted(set(to_remove), reverse=True):
        del circuit.data[i]


def remove_unnecessary_2q_gates_from_circuit(circuit, gate_range=None):
    """circuit_operations_optimisation.py:167-204."""
    if gate_range is None:
        gate_range = (0, len(circuit.data))
    to_remove, dealt = [], []
    for gi in range(gate_range[1] - 1, gate_range[0] - 1, -1):
        ins = circuit.data[gi]
        if ins.operation.name not in ("cx", "cy", "cz") or gi in to_remove or gi in dealt:
            continue
        pg, pi = _prev_on_qubit(circuit, gi)
        if pg is None or pg.name != ins.operation.name or pi < gate_range[0]:
            continue
        if pi in to_remove or pi in dealt:
            continue
        if circuit.data[pi].qubits == ins.qubits:
            to_remove += [gi, pi]
    for i in sorted(to_remove, reverse=True):
        del circuit.data[i]


def remove_unnecessary_gates_from_circuit(circuit, remove_zero_gates=True, remove_small_gates=False,
                                          gate_range=None):
    """circuit_operations_optimisation.py:30-70: alternate 1q merging and 2q cancellation."""
    gate_range = [0, len(circuit.data)] if gate_range is None else list(gate_range)
    last = len(circuit.data)
    i = 0
    while True:
        if i == 0:
            remove_unnecessary_1q_gates_from_circuit(circuit, remove_zero_gates, remove_small_gates, gate_range)
            i = 1
        else:
            remove_unnecessary_2q_gates_from_circuit(circuit, gate_range)
            i = 0
        new = len(circuit.data)
        if new != last:
            gate_range[1] -= last - new
            last = new
        elif i == 0:
            return


def calculate_overlap_between_circuits(circuit1, circuit2):
    """|<0|U1^dag U2|0>|^2 = |<psi1|psi2>|^2, evaluated on the device statevector engine."""
    from ..circuit import device_ops
    from ..device import DeviceSV

    d = DeviceSV(circuit1.num_qubits)
    d.apply(device_ops(circuit2) + device_ops(circuit1.inverse()))
    return float(abs(d.amp0()) ** 2)
