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

"""Two-qubit layer templates (reference adaptaqc/utils/ansatzes.py:14-100)."""
from ..circuit import QuantumCircuit


def _build(spec):
    qc = QuantumCircuit(2)
    for name, q in spec:
        if name == "cx":
            qc.cx(*q)
        else:
            getattr(qc, name)(0.0, q)
    return qc


def u4():
    return _build([("rz", 0), ("ry", 0), ("rz", 0), ("rz", 1), ("ry", 1), ("rz", 1), ("cx", (1, 0)),
                   ("rz", 0), ("ry", 1), ("cx", (0, 1)), ("ry", 1), ("cx", (1, 0)), ("rz", 0), ("ry", 0),
                   ("rz", 0), ("rz", 1), ("ry", 1), ("rz", 1)])


def thinly_dressed_cnot():
    return _build([("rx", 0), ("rx", 1), ("cx", (0, 1)), ("rx", 0), ("rx", 1)])


def fully_dressed_cnot():
    return _build([("rz", 0), ("ry", 0), ("rz", 0), ("rz", 1), ("ry", 1), ("rz", 1), ("cx", (0, 1)),
                   ("rz", 0), ("ry", 0), ("rz", 0), ("rz", 1), ("ry", 1), ("rz", 1)])


def identity_resolvable():
    return _build([("rx", 0), ("rx", 1), ("cx", (0, 1)), ("rx", 0), ("rx", 1), ("cx", (0, 1)), ("rx", 0),
                   ("rx", 1)])


def heisenberg():
    return _build([("rz", 1), ("cx", (1, 0)), ("rz", 0), ("ry", 1), ("cx", (0, 1)), ("ry", 1), ("cx", (1, 0)),
                   ("rz", 0)])
