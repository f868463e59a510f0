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

"""AdaptCompiler host loop (reference compilers/adapt/adapt_compiler.py:48-1163).

Restates the adaptive layer loop around the hot path: pair selection (general_gradient sweep on
the device, or basic / random / expectation / brickwall), Rotoselect on the new layer and
Rotosolve on the last ``max_layers_to_modify`` layers (every cost evaluation on the device),
and, for the MPS backend, absorption of old layers into the cached MPS
(:662-706, :1097-1145).  ISL (the default method) runs the pairwise entanglement sweep on the
device (utils/entanglement_measures.py, csrc/ent.hip).
"""
import logging
import os
import pickle
import timeit
from pathlib import Path

import numpy as np

from ...backends.python_default_backends import SV_SIM
from ...circuit import QuantumCircuit, qasm2_dumps
from ...mps_operations import mps_from_circuit
from ...utils import ansatzes as ans
from ...utils import circuit_operations as co
from ...utils import gradients as gr
from ...utils.constants import ALG_ROTOSELECT, ALG_ROTOSOLVE, CMAP_FULL, generate_coupling_map
from ...utils.utilityfunctions import has_stopped_improving, multi_qubit_gate_depth, \
    remove_permutations_from_coupling_map
from ..approximate_compiler import ApproximateCompiler
from .adapt_config import AdaptConfig
from .adapt_result import AdaptResult
from .pair_selection import reuse_priorities
from ...sharding import as_comm
from ...utils.entanglement_measures import EM_TOMOGRAPHY_CONCURRENCE

logger = logging.getLogger(__name__)


class AdaptCompiler(ApproximateCompiler):
    def __init__(self, target, entanglement_measure=EM_TOMOGRAPHY_CONCURRENCE, backend=SV_SIM, execute_kwargs=None,
                 coupling_map=None, adapt_config: AdaptConfig = None, general_initial_state=False,
                 custom_layer_2q_gate=None, save_circuit_history=False, starting_circuit=None, use_roto_algos=True,
                 use_rotoselect=True, use_advanced_transpilation=False, rotosolve_fraction=1.0,
                 perform_final_minimisation=False, optimise_local_cost=False, soften_global_cost=False,
                 debug_log_full_ansatz=False, initial_single_qubit_layer=False, itensor_chi=None,
                 itensor_cutoff=None, comm=None):
        super().__init__(target=target, initial_state=None, backend=backend, execute_kwargs=execute_kwargs,
                         general_initial_state=general_initial_state, starting_circuit=starting_circuit,
                         optimise_local_cost=optimise_local_cost, rotosolve_fraction=rotosolve_fraction)
        if use_advanced_transpilation or perform_final_minimisation:
            raise NotImplementedError("qiskit transpilation / PyBOBYQA are not available in this build")
        self.save_circuit_history = save_circuit_history
        self.entanglement_measure_method = entanglement_measure
        self.adapt_config = adapt_config if adapt_config is not None else AdaptConfig()
        if coupling_map is None:
            coupling_map = generate_coupling_map(self.total_num_qubits, CMAP_FULL, False, False)
        self.remove_unnecessary_gates_during_adapt = custom_layer_2q_gate is None
        self.use_roto_algos = use_roto_algos
        self.use_rotoselect = use_rotoselect
        self.perform_final_minimisation = False
        self.layer_2q_gate = self.construct_layer_2q_gate(custom_layer_2q_gate)
        self.coupling_map = remove_permutations_from_coupling_map(coupling_map)
        self.coupling_map = [(a, b) for (a, b) in self.coupling_map
                             if a in self.qubit_subset_to_compile and b in self.qubit_subset_to_compile]
        self.qubit_pair_history = []
        self.bad_qubit_pairs = []
        self.pair_selection_method_history = []
        self.entanglement_measures_history = []
        self.e_val_history = []
        self.general_gradient_history = []
        self.time_taken = None
        self.debug_log_full_ansatz = debug_log_full_ansatz
        self.initial_single_qubit_layer = initial_single_qubit_layer
        if self.is_aer_mps_backend:
            self.layers_saved_to_mps = self.full_circuit.copy()
            del self.layers_saved_to_mps.data[1:]
        self.layers_as_gates = []
        self.resume_from_layer = None
        self.prev_checkpoint_time_taken = None
        if self.adapt_config.method == "general_gradient":
            if not self.is_aer_mps_backend:
                raise ValueError("general_gradient method is only implemented for Aer MPS backend")
            self.generators, self.degeneracies = gr.get_generators_and_degeneracies(
                self.layer_2q_gate, use_rotoselect, inverse=True)
            self.inverse_zero_ansatz = self.layer_2q_gate.inverse()
        self.soften_global_cost = soften_global_cost
        # (not in the reference) the ranks of one node share each layer's pair sweep -- general
        # gradient and ISL -- through this communicator (sharding.as_comm: a TorchComm / torch
        # process group over RCCL, or comm.RcclComm); every rank runs the same compile and picks the
        # same pair.  None: one process.
        self.comm = as_comm(comm)
        if self.soften_global_cost and self.optimise_local_cost:
            raise ValueError("soften_global_cost must be False when optimising local cost")

    # -- layers ------------------------------------------------------------------------
    def construct_layer_2q_gate(self, custom_layer_2q_gate):
        if custom_layer_2q_gate is None:  # adapt_compiler.py:224-233
            qc = QuantumCircuit(2)
            co.add_dressed_cnot(qc, 0, 1, True)
            if self.general_initial_state:
                co.add_dressed_cnot(qc, 0, 1, True, v1=False, v2=False)
            return qc
        for ins in custom_layer_2q_gate.data:
            if ins.operation.label is None and ins.operation.name in co.SUPPORTED_1Q_GATES:
                ins.operation.label = ins.operation.name
        return custom_layer_2q_gate

    def get_layer_2q_gate(self, layer_index):
        return self.layer_2q_gate.copy()

    # -- main loop ---------------------------------------------------------------------
    def compile(self, initial_ansatz=None, optimise_initial_ansatz=True, checkpoint_every=0,
                checkpoint_dir="checkpoint/", delete_prev_chkpt=False, freeze_prev_layers=False):
        """adapt_compiler.py:246-482."""
        start_time = timeit.default_timer()
        if self.resume_from_layer is None:
            reset = getattr(self.backend, "reset_learned_capacity", None)
            if reset is not None:  # (capacity learned by earlier compiles on this backend: not ours)
                reset()
            self.time_taken = 0
            start_point = 0
            self.cost_evaluation_counter = 0
            self.global_cost, self.local_cost = None, None
            self.cnot_depth = None
            self.global_cost_history = []
            if self.optimise_local_cost:
                self.local_cost_history = []
            self.circuit_history = []
            self.cnot_depth_history = []
            self.g_range = self.variational_circuit_range
            self.original_lhs_gate_count = self.lhs_gate_count
            if freeze_prev_layers:
                logger.warning("freeze_prev_layers only applies when resuming from a checkpoint")
            # adapt_compiler.py:295-300: a provided ansatz is added (and optimised) first
            self.initial_ansatz_already_successful = False
            if initial_ansatz is not None:
                self._add_initial_ansatz(initial_ansatz, optimise_initial_ansatz)
        else:
            start_point = self.resume_from_layer
            self.time_taken = self.prev_checkpoint_time_taken
            if initial_ansatz is not None:
                logger.warning("An initial ansatz will be ignored when resuming recompilation from a checkpoint")
            if freeze_prev_layers:
                if self.is_aer_mps_backend:
                    num_gates = len(self.full_circuit) - self.rhs_gate_count - 1
                    absorbed = self._absorb_n_gates_into_mps(n=num_gates)
                    co.add_to_circuit(self.layers_saved_to_mps, absorbed)
                    self._update_reference_circuit()
                else:
                    self.lhs_gate_count = self.variational_circuit_range()[1]
        if checkpoint_every > 0:
            Path(checkpoint_dir).mkdir(parents=True, exist_ok=True)

        for layer_count in range(start_point, self.adapt_config.max_layers):
            if getattr(self, "initial_ansatz_already_successful", False):
                break
            if self.optimise_local_cost:
                self.local_cost = self._add_layer(layer_count)
                self.global_cost = self.backend.evaluate_global_cost(self)
                self.local_cost_history.append(self.local_cost)
            else:
                self.global_cost = self._add_layer(layer_count)
            self.global_cost_history.append(self.global_cost)
            self.record_cnot_depth()
            if self.remove_unnecessary_gates_during_adapt and not self.is_aer_mps_backend:
                co.remove_unnecessary_gates_from_circuit(self.full_circuit, False, False, gate_range=self.g_range())
            ref = self.ref_circuit_as_gates if self.is_aer_mps_backend else self.full_circuit
            num_2q_gates, _ = co.find_num_gates(ref, gate_range=self.g_range(ref if self.is_aer_mps_backend else None))
            if self.save_circuit_history:  # adapt_compiler.py:359-366 (MPS: without the MPS op)
                if not self.is_aer_mps_backend:
                    self.circuit_history.append(qasm2_dumps(self.full_circuit))
                else:
                    circuit_copy = self.full_circuit.copy()
                    del circuit_copy.data[0]
                    self.circuit_history.append(qasm2_dumps(circuit_copy))
            cinl = self.adapt_config.cost_improvement_num_layers
            cit = self.adapt_config.cost_improvement_tol
            if len(self.global_cost_history) >= cinl and has_stopped_improving(self.global_cost_history[-cinl:], cit):
                logger.warning("ADAPT-AQC stopped improving")
                self.compiling_finished = True
                break
            if self.global_cost < self.adapt_config.sufficient_cost:
                self.compiling_finished = True
                break
            if num_2q_gates >= self.adapt_config.max_2q_gates:
                self.minimizer.minimize_cost(algorithm_kind=ALG_ROTOSOLVE, max_cycles=10, tol=1e-5,
                                             stop_val=self.adapt_config.sufficient_cost)
                self.compiling_finished = True
                break
            if checkpoint_every > 0 and layer_count % checkpoint_every == 0:
                self.checkpoint(checkpoint_every, checkpoint_dir, delete_prev_chkpt, layer_count, start_time)

        if self.is_aer_mps_backend:
            self.full_circuit = self.ref_circuit_as_gates
        else:
            self.lhs_gate_count = self.original_lhs_gate_count
        co.remove_unnecessary_gates_from_circuit(self.full_circuit, True, True, gate_range=self.g_range())
        soft = self.soften_global_cost
        self.soften_global_cost = False
        final_global_cost = self.backend.evaluate_global_cost(self)
        self.soften_global_cost = soft
        self.global_cost_history.append(final_global_cost)
        if checkpoint_every > 0:  # adapt_compiler.py:432-439: the finished state is checkpointed too
            self.checkpoint(checkpoint_every, checkpoint_dir, delete_prev_chkpt, len(self.qubit_pair_history) - 1,
                            start_time)
        compiled = self.get_compiled_circuit()
        num_2q_gates, num_1q_gates = co.find_num_gates(compiled)
        self.cnot_depth_history.append(multi_qubit_gate_depth(compiled))
        exact_overlap = "Not computable without SV backend"
        if self.is_statevector_backend:
            exact_overlap = co.calculate_overlap_between_circuits(self.circuit_to_compile, compiled)
        if self.save_circuit_history and self.is_aer_mps_backend:
            logger.warning("When using MPS backend, circuit history will not contain the "
                           "set_matrix_product_state instruction at the start of the circuit")
        return AdaptResult(
            circuit=compiled, overlap=1 - final_global_cost, exact_overlap=exact_overlap, num_1q_gates=num_1q_gates,
            num_2q_gates=num_2q_gates, cnot_depth_history=self.cnot_depth_history,
            global_cost_history=self.global_cost_history,
            local_cost_history=self.local_cost_history if self.optimise_local_cost else None,
            circuit_history=self.circuit_history, entanglement_measures_history=self.entanglement_measures_history,
            e_val_history=self.e_val_history, qubit_pair_history=self.qubit_pair_history,
            method_history=self.pair_selection_method_history,
            time_taken=self.time_taken + (timeit.default_timer() - start_time),
            cost_evaluations=self.cost_evaluation_counter, coupling_map=self.coupling_map)

    def checkpoint(self, checkpoint_every, checkpoint_dir, delete_prev_chkpt, layer_count, start_time):
        """adapt_compiler.py:484-506 (the backend drops its device state when pickled)."""
        self.resume_from_layer = layer_count + 1
        self.prev_checkpoint_time_taken = self.time_taken + (timeit.default_timer() - start_time)
        comm = getattr(self, "comm", None)
        if comm is not None and comm.rank != 0:
            return  # (ranks sharing the sweeps run the same compile: rank 0 writes the checkpoint)
        self.comm = None  # (a communicator does not pickle; a resumed compile passes its own)
        try:
            with open(os.path.join(checkpoint_dir, f"{layer_count}.pkl"), "wb") as f:
                pickle.dump(self, f)
        finally:
            self.comm = comm
        if delete_prev_chkpt:
            try:
                os.remove(os.path.join(checkpoint_dir, f"{layer_count - checkpoint_every}.pkl"))
            except FileNotFoundError:
                pass

    def _add_initial_ansatz(self, initial_ansatz, optimise_initial_ansatz):
        """adapt_compiler.py:536-583: the ansatz's inverse goes at the end of the variational
        range, its rotations are optimised by Rotosolve (labels set so that Rotosolve recognises
        them), and it is then frozen: absorbed into the cached MPS on the MPS backend, or moved
        left of the variational range on the statevector backend."""
        for ins in initial_ansatz.data:
            if ins.operation.label is None and ins.operation.name in co.SUPPORTED_1Q_GATES:
                ins.operation.label = ins.operation.name
        co.add_to_circuit(self.full_circuit, co.circuit_by_inverting_circuit(initial_ansatz),
                          self.variational_circuit_range()[1])
        if optimise_initial_ansatz:
            if not self.use_roto_algos:
                raise NotImplementedError("PyBOBYQA is not available in this build")
            cost = self.minimizer.minimize_cost(
                algorithm_kind=ALG_ROTOSOLVE, tol=1e-3,
                stop_val=0 if self.optimise_local_cost else self.adapt_config.sufficient_cost,
                indexes_to_modify=self.variational_circuit_range())
        else:
            cost = self.evaluate_cost()
        self.global_cost = self.backend.evaluate_global_cost(self) if self.optimise_local_cost else cost
        self.cnot_depth = multi_qubit_gate_depth(initial_ansatz)
        if self.global_cost < self.adapt_config.sufficient_cost:
            self.initial_ansatz_already_successful = True
            logger.debug("ADAPT-AQC successfully found approximate circuit using provided ansatz only")
        if self.is_aer_mps_backend:
            absorbed = self._absorb_n_gates_into_mps(n=len(initial_ansatz.data))
            co.add_to_circuit(self.layers_saved_to_mps, absorbed)
            self._update_reference_circuit()
        else:
            self.lhs_gate_count = self.variational_circuit_range()[1]

    def _add_layer(self, index):
        """adapt_compiler.py:585-689."""
        ansatz_start_index = self.variational_circuit_range()[0]
        if self.initial_single_qubit_layer and index == 0:
            idx = self._add_rotation_to_all_qubits()
        else:
            idx = self._add_entangling_layer(index)
        stop_val = 0 if self.optimise_local_cost else self.adapt_config.sufficient_cost
        if self.use_roto_algos:
            alg = ALG_ROTOSELECT if (self.use_rotoselect or (self.initial_single_qubit_layer and index == 0)) \
                else ALG_ROTOSOLVE
            cost = self.minimizer.minimize_cost(algorithm_kind=alg, tol=self.adapt_config.rotoselect_tol,
                                                stop_val=stop_val, indexes_to_modify=idx)
            freq = self.adapt_config.rotosolve_frequency
            if freq != 0 and index > 0 and index % freq == 0:
                multi = self._calculate_multi_layer_optimisation_indices(ansatz_start_index)
                cost = self.minimizer.minimize_cost(algorithm_kind=ALG_ROTOSOLVE, tol=self.adapt_config.rotosolve_tol,
                                                    stop_val=stop_val, indexes_to_modify=multi)
        else:
            raise NotImplementedError("PyBOBYQA is not available in this build")
        if self.is_aer_mps_backend:
            self.layers_as_gates.append(index)
            k = self._calculate_num_layers_to_absorb(index)
            if k > 0:
                isql = self.layers_as_gates[0] == 0 and self.initial_single_qubit_layer
                absorbed = self._absorb_n_gates_into_mps(self._get_num_gates_to_cache(k, isql))
                co.add_to_circuit(self.layers_saved_to_mps, absorbed)
                del self.layers_as_gates[:k]
            self._update_reference_circuit()
        return cost

    def _calculate_num_layers_to_absorb(self, index):
        """adapt_compiler.py:691-706 (rotosolve_frequency = 0 raises ZeroDivisionError, as there)."""
        freq = self.adapt_config.rotosolve_frequency
        nxt = index + (freq - index % freq)
        lowest = nxt - self.adapt_config.max_layers_to_modify + 1
        return len([i for i in self.layers_as_gates if i < lowest])

    def _update_reference_circuit(self):
        rest = self.full_circuit.copy()
        del rest.data[0]
        self.ref_circuit_as_gates = self.layers_saved_to_mps.copy()
        co.add_to_circuit(self.ref_circuit_as_gates, rest)

    def _calculate_multi_layer_optimisation_indices(self, ansatz_start_index):
        n_ent = self.adapt_config.max_layers_to_modify - int(self.initial_single_qubit_layer)
        n_first = self.full_circuit.num_qubits * int(self.initial_single_qubit_layer)
        start = max(ansatz_start_index,
                    self.variational_circuit_range()[1] - len(self.layer_2q_gate.data) * n_ent - n_first)
        first_end = ansatz_start_index + n_first
        if ansatz_start_index < start < first_end:
            start = first_end
        return start, self.variational_circuit_range()[1]

    def _add_entangling_layer(self, index):
        control, target = self._find_appropriate_qubit_pair()
        co.add_to_circuit(self.full_circuit, self.get_layer_2q_gate(index), self.variational_circuit_range()[1],
                          qubit_subset=[control, target])
        self.qubit_pair_history.append((control, target))
        end = self.variational_circuit_range()[1]
        return end - len(self.layer_2q_gate.data), end

    def _add_rotation_to_all_qubits(self):
        layer = QuantumCircuit(self.full_circuit.num_qubits)
        for q in range(self.full_circuit.num_qubits):
            layer.ry(0, q)
        co.add_to_circuit(self.full_circuit, layer, self.variational_circuit_range()[1])
        self.entanglement_measures_history.append([None])
        self.e_val_history.append(None)
        self.general_gradient_history.append(None)
        self.qubit_pair_history.append((None, None))
        self.pair_selection_method_history.append(None)
        end = self.variational_circuit_range()[1]
        return end - self.full_circuit.num_qubits, end

    # -- pair selection ----------------------------------------------------------------
    def _find_appropriate_qubit_pair(self):
        """adapt_compiler.py:775-830."""
        m = self.adapt_config.method
        if m == "random":
            self.pair_selection_method_history.append("random")
            return self.coupling_map[np.random.randint(len(self.coupling_map))]
        if m == "basic":
            self.pair_selection_method_history.append("basic")
            return self.coupling_map[int(np.argmax(self._get_all_qubit_pair_reuse_priorities(1)))]
        if m == "expectation":
            return self._find_best_expectation_qubit_pair()
        if m == "ISL":
            ems = self._get_all_qubit_pair_entanglement_measures()
            self.entanglement_measures_history.append(ems)
            return self._find_best_entanglement_qubit_pair(ems)
        if m == "general_gradient":
            gradients = self._get_all_qubit_pair_gradients()
            self.general_gradient_history.append(gradients)
            self.pair_selection_method_history.append("general_gradient")
            return self._find_best_gradient_qubit_pair(gradients)
        if m == "brickwall":
            n = self.full_circuit.num_qubits
            if n < 2:
                raise ValueError("Cannot pick a pair if there are fewer than two qubits")
            if not self.qubit_pair_history or n == 2 or self.qubit_pair_history[-1][0] is None:
                return (0, 1)
            prev = self.qubit_pair_history[-1]
            nxt = (prev[0] + 2, prev[1] + 2)
            odd = n % 2
            if nxt == (n, n + 1):
                return (1 - odd, 2 - odd)
            if nxt == (n - 1, n):
                return (0 + odd, 1 + odd)
            return nxt
        raise ValueError(f"Invalid compiling method {m}. Method must be one of ISL, expectation, random, basic, "
                         f"general_gradient, brickwall")

    def _get_all_qubit_pair_reuse_priorities(self, k):
        return reuse_priorities(self.coupling_map, self.qubit_pair_history, k, self.adapt_config.reuse_priority_mode,
                                self.initial_single_qubit_layer)

    def _find_best_gradient_qubit_pair(self, gradients):
        prio = self._get_all_qubit_pair_reuse_priorities(self.adapt_config.reuse_exponent)
        return self.coupling_map[int(np.argmax(np.multiply(gradients, prio)))]

    def _get_all_qubit_pair_gradients(self):
        """adapt_compiler.py:839-856 (starting circuit stripped by its length, as there)."""
        if self.starting_circuit is not None:
            rng = (0, len(self.full_circuit) - len(self.starting_circuit))
        else:
            rng = (0, len(self.full_circuit))
        circuit = co.extract_inner_circuit(self.full_circuit, rng)
        return gr.general_grad_of_pairs(circuit, self.inverse_zero_ansatz, self.generators, self.degeneracies,
                                        self.coupling_map, self.starting_circuit, self.backend,
                                        comm=getattr(self, "comm", None))

    def _get_all_qubit_pair_entanglement_measures(self):
        """adapt_compiler.py:955-976: one device state, every pair's RDM and measure in batches."""
        from ...utils.entanglement_measures import pair_entanglement_measures

        self.circ_mps = None  # the reference keeps the host MPS here; the sweep stays on the device
        return pair_entanglement_measures(self.entanglement_measure_method, self, self.coupling_map,
                                          comm=getattr(self, "comm", None))

    def _find_best_entanglement_qubit_pair(self, entanglement_measures):
        """adapt_compiler.py:858-919: entanglement x reuse priority, bad-pair memory, threshold
        fall-back to the expectation method."""
        reuse = self._get_all_qubit_pair_reuse_priorities(self.adapt_config.reuse_exponent)
        if len(self.entanglement_measures_history) >= 2 + int(self.initial_single_qubit_layer):
            prev_index = self.coupling_map.index(self.qubit_pair_history[-1])
            pre_em = self.entanglement_measures_history[-2][prev_index]
            post_em = self.entanglement_measures_history[-1][prev_index]
            if post_em >= pre_em:
                logger.debug(f"Entanglement did not reduce for previous pair {self.coupling_map[prev_index]}. "
                             f"Adding to bad qubit pairs list.")
                self.bad_qubit_pairs.append(self.coupling_map[prev_index])
            if len(self.bad_qubit_pairs) > self.adapt_config.bad_qubit_pair_memory:
                del self.bad_qubit_pairs[0]
        filtered = [em * r for em, r in zip(entanglement_measures, reuse)]
        memory = self.adapt_config.bad_qubit_pair_memory
        for qp in set(self.bad_qubit_pairs):
            reps = len([x for x in self.qubit_pair_history[-1 * memory:] if x == qp])
            if reps >= 1:
                filtered[self.coupling_map.index(qp)] = -1
        if max(filtered) <= self.adapt_config.entanglement_threshold:
            logger.info("No local entanglement detected in non-bad qubit pairs")
            return self._find_best_expectation_qubit_pair()
        self.pair_selection_method_history.append("ISL")
        self.e_val_history.append(None)
        return self.coupling_map[int(np.argmax(filtered))]

    def _find_best_expectation_qubit_pair(self):
        prio = self._get_all_qubit_pair_reuse_priorities(self.adapt_config.reuse_exponent)
        e_vals = self.backend.measure_qubit_expectation_values(self)
        self.e_val_history.append(e_vals)
        sums = [e_vals[c] + e_vals[t] for c, t in self.coupling_map]
        combined = [(2 - s) * p for s, p in zip(sums, prio)]
        self.pair_selection_method_history.append("expectation")
        return self.coupling_map[int(np.argmax(combined))]

    # -- MPS caching -----------------------------------------------------------------
    def _get_num_gates_to_cache(self, n, includes_isql=False):
        return len(self.layer_2q_gate) * (n - int(includes_isql)) + self.full_circuit.num_qubits * int(includes_isql)

    def _absorb_n_gates_into_mps(self, n):
        """adapt_compiler.py:1097-1145: fold the first n gates after the MPS op into it."""
        k = n + 1
        circ = self.full_circuit.copy()
        del circ.data[k:]
        absorbed = circ.copy()
        del absorbed.data[0]
        new_mps = mps_from_circuit(circ, sim=self.backend.simulator)
        mps_circuit = QuantumCircuit(self.full_circuit.num_qubits)
        mps_circuit.set_matrix_product_state(new_mps)
        remaining = len(self.full_circuit.data) - k
        if remaining != 0:
            del self.full_circuit.data[:-remaining]
        else:
            del self.full_circuit.data[:]
        self.full_circuit.data.insert(0, mps_circuit.data[0])
        return absorbed

    def record_cnot_depth(self):
        if self.is_aer_mps_backend:
            circ = co.extract_inner_circuit(self.ref_circuit_as_gates, (1, len(self.ref_circuit_as_gates)))
        else:
            circ = co.extract_inner_circuit(self.full_circuit, (self.original_lhs_gate_count,
                                                                self.variational_circuit_range()[1]))
        self.cnot_depth = multi_qubit_gate_depth(circ)
        self.cnot_depth_history.append(self.cnot_depth)


__all__ = ["AdaptCompiler", "AdaptConfig", "ans"]
