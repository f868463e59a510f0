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

"""AdaptConfig (reference compilers/adapt/adapt_config.py:16-97): same fields and defaults."""
from ...utils.constants import DEFAULT_SUFFICIENT_COST


class AdaptConfig:
    def __init__(self, max_layers: int = int(1e5), sufficient_cost=DEFAULT_SUFFICIENT_COST, max_2q_gates=1e4,
                 cost_improvement_num_layers=10, cost_improvement_tol=1e-2, max_layers_to_modify=100, method="ISL",
                 bad_qubit_pair_memory=10, reuse_exponent=0, reuse_priority_mode="pair", rotosolve_frequency=1,
                 rotoselect_tol=1e-5, rotosolve_tol=1e-3, entanglement_threshold=1e-8):
        self.bad_qubit_pair_memory = bad_qubit_pair_memory
        self.max_layers = max_layers
        self.sufficient_cost = sufficient_cost
        self.max_2q_gates = max_2q_gates
        self.cost_improvement_tol = cost_improvement_tol
        self.cost_improvement_num_layers = int(cost_improvement_num_layers)
        self.max_layers_to_modify = max_layers_to_modify
        self.method = method
        self.rotosolve_frequency = rotosolve_frequency
        self.rotoselect_tol = rotoselect_tol
        self.rotosolve_tol = rotosolve_tol
        self.entanglement_threshold = entanglement_threshold
        self.reuse_exponent = reuse_exponent
        self.reuse_priority_mode = reuse_priority_mode.lower()

    def __repr__(self):
        return f"{self.__class__.__name__}(" + ", ".join(f"{k}={v!r}" for k, v in self.__dict__.items()) + ")"
