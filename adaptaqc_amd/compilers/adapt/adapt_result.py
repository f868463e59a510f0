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

"""AdaptResult (reference compilers/adapt/adapt_result.py:14-70)."""


class AdaptResult:
    def __init__(self, circuit, overlap, exact_overlap, num_1q_gates, num_2q_gates, cnot_depth_history,
                 global_cost_history, local_cost_history, circuit_history, entanglement_measures_history,
                 e_val_history, qubit_pair_history, method_history, time_taken, cost_evaluations, coupling_map,
                 circuit_qasm=None):
        self.circuit = circuit
        self.overlap = overlap
        self.exact_overlap = exact_overlap
        self.num_1q_gates = num_1q_gates
        self.num_2q_gates = num_2q_gates
        self.cnot_depth_history = cnot_depth_history
        self.global_cost_history = global_cost_history
        self.local_cost_history = local_cost_history
        self.circuit_history = circuit_history
        self.entanglement_measures_history = entanglement_measures_history
        self.e_val_history = e_val_history
        self.qubit_pair_history = qubit_pair_history
        self.method_history = method_history
        self.time_taken = time_taken
        self.cost_evaluations = cost_evaluations
        self.coupling_map = coupling_map
        self.circuit_qasm = circuit_qasm

    def __repr__(self):
        return (f"AdaptResult(overlap={self.overlap}, num_2q_gates={self.num_2q_gates}, "
                f"cost_evaluations={self.cost_evaluations}, time_taken={self.time_taken:.2f}s)")
