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

"""Coupling maps and constants (reference adaptaqc/utils/constants.py:17-110)."""
from typing import List, Tuple

import numpy as np

QiskitMPS = Tuple[List[Tuple[np.ndarray, np.ndarray]], List[np.ndarray]]

ALG_ROTOSOLVE = "rotosolve"
ALG_ROTOSELECT = "rotoselect"
FIXED_GATE_LABEL = "fixed_gate"
CMAP_FULL = "CMAP_FULL"
CMAP_LINEAR = "CMAP_LINEAR"
CMAP_LADDER = "CMAP_LADDER"
DEFAULT_SUFFICIENT_COST = 1e-2


def generate_coupling_map(num_qubits, map_kind, both_dir=False, loop=False):
    if map_kind == CMAP_FULL:
        return coupling_map_fully_entangled(num_qubits, both_dir)
    if map_kind == CMAP_LINEAR:
        return coupling_map_linear(num_qubits, both_dir, loop)
    if map_kind == CMAP_LADDER:
        return coupling_map_ladder(num_qubits, both_dir, loop)
    raise ValueError(f"Invalid coupling map type {map_kind}")


def _with_reverse(c_map, both_dir):
    return c_map + [(t, s) for (s, t) in c_map] if both_dir else c_map


def coupling_map_fully_entangled(num_qubits, both_dir=False):
    """All pairs, ordered by distance then by first qubit."""
    return _with_reverse([(j, j + d) for d in range(1, num_qubits) for j in range(num_qubits - d)], both_dir)


def coupling_map_linear(num_qubits, both_dir=False, loop=False):
    c_map = [(j, j + 1) for j in range(num_qubits - 1)]
    if loop:
        c_map.append((num_qubits - 1, 0))
    return _with_reverse(c_map, both_dir)


def coupling_map_ladder(num_qubits, both_dir=False, loop=False):
    c_map = [(j, j + 1) for j in range(0, num_qubits - 1, 2)]
    if loop and num_qubits % 2 == 1:
        c_map.append((num_qubits - 1, 0))
    c_map += [(j, j + 1) for j in range(1, num_qubits - 1, 2)]
    if loop and num_qubits % 2 == 0:
        c_map.append((num_qubits - 1, 0))
    return _with_reverse(c_map, both_dir)
