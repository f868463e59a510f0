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

"""Host scalar helpers (reference adaptaqc/utils/utilityfunctions.py)."""
from collections.abc import Iterable
from typing import List, Tuple

import numpy as np


def minimum_of_sinusoidal(value_0, value_pi_by_2, value_minus_pi_by_2):
    """utilityfunctions.py:34-57: (x_min, f(x_min)) of f(x) = a sin(x + b) + c."""
    theta_min = -(np.pi / 2) - np.arctan2(
        2 * value_0 - value_pi_by_2 - value_minus_pi_by_2, value_pi_by_2 - value_minus_pi_by_2
    )
    theta_min = normalized_angles(theta_min)
    intercept_c = 0.5 * (value_pi_by_2 + value_minus_pi_by_2)
    value_pi = (value_pi_by_2 + value_minus_pi_by_2) - value_0
    amplitude_a = 0.5 * (((value_0 - value_pi) ** 2 + (value_pi_by_2 - value_minus_pi_by_2) ** 2) ** 0.5)
    return theta_min, intercept_c - amplitude_a


def normalized_angles(angles):
    single = not isinstance(angles, Iterable)
    if single:
        angles = [angles]
    out = []
    for a in angles:
        while a > np.pi or a < -np.pi:
            a = a - 2 * np.pi if a > np.pi else a + 2 * np.pi
        out.append(a)
    return out[0] if single else out


def is_statevector_backend(backend):
    from ..backends.aer_sv_backend import AerSVBackend

    return isinstance(backend, AerSVBackend)


def remove_permutations_from_coupling_map(coupling_map):
    seen, unique = set(), []
    for pair in coupling_map:
        k = tuple(sorted(pair))
        if k not in seen:
            seen.add(k)
            unique.append(pair)
    return unique


def has_stopped_improving(cost_history, rel_tol=1e-2):
    try:
        poly = np.polyfit(list(range(len(cost_history))), cost_history, 1)
        return poly[0] / np.absolute(np.mean(cost_history)) > -1 * rel_tol
    except np.linalg.LinAlgError:
        return False


def get_distinct_items_and_degeneracies(items: List) -> Tuple[List, List[int]]:
    distinct, degeneracies = [], []
    for item in items:
        for j, d in enumerate(distinct):
            if item == d:
                degeneracies[j] += 1
                break
        else:
            distinct.append(item)
            degeneracies.append(1)
    return distinct, degeneracies


def multi_qubit_gate_depth(qc) -> int:
    return qc.depth(filter_function=lambda instr: len(instr.qubits) > 1)
