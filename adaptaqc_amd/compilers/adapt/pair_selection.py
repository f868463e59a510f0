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

"""Candidate selection (reference adapt_compiler.py:832-837, 984-1065): reuse priorities and the
arg-max over gradient x priority (np.argmax: the first maximum wins)."""
import numpy as np


def pair_reuse_priority(history, pair, k, isql=False):
    """adapt_compiler.py:1037-1065."""
    if len(history) > int(isql) and pair == history[-1]:
        return -1
    if k == 0:
        return 1
    rev = history[::-1]
    try:
        return 1 - np.exp2(-rev.index(pair) / k)
    except ValueError:
        return 1


def qubit_reuse_priority(history, pair, k, isql=False):
    """adapt_compiler.py:1006-1035."""
    if len(history) > int(isql) and pair == history[-1]:
        return -1
    if k == 0:
        return 1
    rev = history[::-1]

    def last_use(q):
        for i, t in enumerate(rev):
            if q in t:
                return i
        return np.inf

    return np.min([1 - np.exp2(-(last_use(q) + 1) / k) for q in pair])


def reuse_priorities(coupling_map, history, k, mode="pair", isql=False):
    """adapt_compiler.py:984-998."""
    if not len(history):
        return [1 for _ in coupling_map]
    if mode == "pair":
        return [pair_reuse_priority(history, qp, k, isql) for qp in coupling_map]
    if mode == "qubit":
        return [qubit_reuse_priority(history, qp, k, isql) for qp in coupling_map]
    raise ValueError(f"Reuse priority mode must be one of: {['pair', 'qubit']}")


def best_gradient_pair(coupling_map, gradients, history, k, mode="pair", isql=False):
    combined = np.multiply(gradients, reuse_priorities(coupling_map, history, k, mode, isql))
    return coupling_map[int(np.argmax(combined))]
