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

"""ApproximateCompiler (reference compilers/approximate_compiler.py:64-527), host side.

Builds ``full_circuit = [target | ansatz | starting_circuit^-1]`` (:435-512), keeps the
MPS target as a leading ``set_matrix_product_state`` instruction when the backend is the MPS
backend (:165-217), and dispatches every cost evaluation to the backend (:514-527).
"""
import logging
from abc import ABC, abstractmethod

from ..backends.aer_mps_backend import AerMPSBackend
from ..backends.python_default_backends import SV_SIM
from ..circuit import QuantumCircuit
from ..mps_operations import check_mps, mps_from_circuit, zero_aer_mps, _preprocess_mps
from ..utils import circuit_operations as co
from ..utils.cost_minimiser import CostMinimiser
from ..utils.utilityfunctions import is_statevector_backend

logger = logging.getLogger(__name__)


def _without_resets(circuit):
    """The initial-state circuit without reset, barrier and delay instructions -- what the
    reference inverts (approximate_compiler.py:481-483: unroll, ``co.remove_reset_gates``,
    ``inverse()``).  Forward, Aer runs the resets from |0..0>, where a reset before any gate on its
    qubit does nothing; a reset after a gate is a non-unitary mid-circuit operation, which the
    pure-state backends here do not run, and raises."""
    from ..circuit import CircuitInstruction, qubit_indices

    out = QuantumCircuit(circuit.num_qubits)
    touched = set()
    for ins in circuit.data:
        name = ins.operation.name
        qs = qubit_indices(circuit, ins)
        if name in ("barrier", "delay"):
            continue
        if name == "reset":
            if any(q in touched for q in qs):
                raise NotImplementedError("initial_state: a reset after a gate on its qubit (mid-circuit reset) "
                                          "is not supported by the pure-state backends")
            continue
        touched.update(qs)
        out.data.append(CircuitInstruction(ins.operation.copy(), list(qs)))
    return out


def initial_state_to_circuit(initial_state):
    """circuit_operations_full_circuit.py:385-410 for circuits; a state vector needs qiskit's
    state-preparation synthesis (``initialize`` unrolled), which is not part of this build."""
    if initial_state is None:
        return None
    if isinstance(initial_state, QuantumCircuit):
        return _without_resets(initial_state)
    if hasattr(initial_state, "num_qubits") and hasattr(initial_state, "data"):  # qiskit-like circuit
        qc = QuantumCircuit(initial_state.num_qubits)
        co.add_to_circuit(qc, initial_state)
        return _without_resets(qc)
    if isinstance(initial_state, (list, tuple)) or hasattr(initial_state, "shape"):
        raise NotImplementedError("a state-vector initial_state needs qiskit's state preparation; pass a circuit")
    raise TypeError("Invalid type of initial_state provided")


class ApproximateCompiler(ABC):
    full_circuit: QuantumCircuit

    def __init__(self, target, backend, execute_kwargs=None, initial_state=None, qubit_subset=None,
                 general_initial_state=False, starting_circuit=None, optimise_local_cost=False,
                 soften_global_cost=False, itensor_chi=None, itensor_cutoff=None, rotosolve_fraction=1.0):
        self.target = target
        self.original_circuit_classical_ops = None
        self.backend = backend if backend is not None else SV_SIM
        self.is_statevector_backend = is_statevector_backend(self.backend)
        self.is_aer_mps_backend = isinstance(self.backend, AerMPSBackend)
        if check_mps(self.target) and not self.is_aer_mps_backend:
            raise Exception("Aer MPS backend must be used when target is an Aer MPS")
        self.circuit_to_compile = self.prepare_circuit()
        self.execute_kwargs = dict(execute_kwargs or {})
        self.execute_kwargs.setdefault("shots", 1)
        self.execute_kwargs.setdefault("optimization_level", 0)
        self.backend_options = {"method": "automatic"}
        if (initial_state is not None or general_initial_state) and self.is_aer_mps_backend:
            # the MPS backend's full circuit starts from the target's MPS (set_matrix_product_state):
            # a state prepared in front of it would be overwritten
            raise NotImplementedError("initial_state / general_initial_state need a statevector backend")
        self.initial_state_circuit = initial_state_to_circuit(initial_state)
        self.total_num_qubits = (self.circuit_to_compile.num_qubits if self.initial_state_circuit is None
                                 else self.initial_state_circuit.num_qubits)  # :289-294
        self.qubit_subset_to_compile = qubit_subset if qubit_subset else list(range(self.total_num_qubits))
        self.general_initial_state = general_initial_state
        self.starting_circuit = self.prepare_starting_circuit(starting_circuit)
        # approximate_compiler.py:133-135 builds this through Aer; it is |0..0> in preprocessed form
        self.zero_mps = _preprocess_mps(zero_aer_mps(self.total_num_qubits))
        self.optimise_local_cost = optimise_local_cost
        self.soften_global_cost = soften_global_cost
        if initial_state is not None and general_initial_state:
            raise ValueError("Can't compile for general initial state when specific initial state is provided")
        self.full_circuit, self.lhs_gate_count, self.rhs_gate_count = self._prepare_full_circuit()
        if not 0 < rotosolve_fraction <= 1:
            raise ValueError("rotosolve_fraction must be in the range (0,1]")
        self.minimizer = CostMinimiser(self.evaluate_cost, self.variational_circuit_range, self.full_circuit,
                                       rotosolve_fraction, evaluator_factory=self._candidate_evaluator)
        self.cost_evaluation_counter = 0
        self.compiling_finished = False

    def prepare_circuit(self):
        if check_mps(self.target):
            qc = QuantumCircuit(len(self.target[0]))
            qc.set_matrix_product_state(self.target)
            return qc
        prepared = self.target.copy()
        if self.is_aer_mps_backend:
            logger.info("Pre-computing target circuit as MPS on the device")
            target_mps = mps_from_circuit(prepared, sim=self.backend.simulator)
            qc = QuantumCircuit(prepared.num_qubits)
            qc.set_matrix_product_state(target_mps)
            return qc
        return prepared

    def prepare_starting_circuit(self, starting_circuit):
        if starting_circuit is None or isinstance(starting_circuit, QuantumCircuit):
            return starting_circuit
        if starting_circuit == "tenpy_product_state":
            return self.product_state_circuit()
        raise ValueError("starting_circuit must be a QuantumCircuit, None, or string: 'tenpy_product_state'")

    def product_state_circuit(self, min_sweeps=10, max_sweeps=50, tol=1e-12):
        """approximate_compiler.py:222-242: the best chi = 1 approximation of the target (the
        reference compresses with tenpy's variational method, chi_max 1, 10-50 sweeps), as one
        single-qubit unitary per qubit in rx / ry / rz (tenpy_chi_1_mps_to_circuit,
        utilityfunctions.py:333-358).  Here the compression runs on the device
        (aqc_mps_product_fit: alternating two-site updates); parity with tenpy is unpinned."""
        from ..mps_operations import device_mps_from_circuit

        if self.is_aer_mps_backend:
            thr = self.backend.simulator.options.matrix_product_state_truncation_threshold
        else:
            thr = 1e-8
        psi = device_mps_from_circuit(self.circuit_to_compile.copy(), trunc_thr=thr)
        svec, fid, sweeps = psi.product_fit(None, min_sweeps, max_sweeps, tol)
        self.starting_state_fidelity = fid
        logger.info(f"Product-state starting circuit: fidelity {fid:.6f} after {sweeps} sweeps")
        return product_state_to_circuit(svec)

    def variational_circuit_range(self, circuit=None):
        if circuit is None:
            circuit = self.full_circuit
        return self.lhs_gate_count, len(circuit.data) - self.rhs_gate_count

    def ansatz_range(self):
        return self.lhs_gate_count, len(self.full_circuit.data)

    @abstractmethod
    def compile(self):
        raise NotImplementedError

    def _prepare_full_circuit(self):
        """approximate_compiler.py:435-512: |0> -- initial state -- circuit_to_compile -- (ansatz) --
        initial state^-1 (or starting_circuit^-1); with general_initial_state the register doubles
        and n Bell pairs (q, q + n) are made before and undone after (arXiv:1811.03147,
        arXiv:1908.04416), so that the overlap with |0..0> measures the whole unitary."""
        n = self.total_num_qubits
        qc = QuantumCircuit(2 * n if self.general_initial_state else n)
        if self.initial_state_circuit is not None:
            co.add_to_circuit(qc, self.initial_state_circuit)
        elif self.general_initial_state:
            for q in range(n):
                qc.h(q)
                qc.cx(q, q + n)
        co.add_to_circuit(qc, self.circuit_to_compile, qubit_subset=self.qubit_subset_to_compile)
        lhs = len(qc.data)
        if self.initial_state_circuit is not None:
            co.add_to_circuit(qc, self.initial_state_circuit.inverse())
        if self.starting_circuit is not None:
            co.add_to_circuit(qc, self.starting_circuit.inverse())
        elif self.general_initial_state:  # (as the reference: not after a starting circuit)
            for q in range(n - 1, -1, -1):
                qc.cx(q, q + n)
                qc.h(q)
        return qc, lhs, len(qc.data) - lhs

    def get_compiled_circuit(self):
        compiled = co.circuit_by_inverting_circuit(
            co.extract_inner_circuit(self.full_circuit, self.variational_circuit_range()))
        if self.starting_circuit is not None:
            co.add_to_circuit(compiled, self.starting_circuit, 0)
        final = QuantumCircuit(self.circuit_to_compile.num_qubits)
        co.add_to_circuit(final, compiled, qubit_subset={i: q for i, q in enumerate(self.qubit_subset_to_compile)})
        return final

    def _candidate_evaluator(self):
        """Cached Rotoselect / Rotosolve candidates (utils/cached_rotations.py) unless disabled
        with ``use_cached_rotations = False``; None selects the reference's generic path."""
        if not getattr(self, "use_cached_rotations", True):
            return None
        from ..utils.cached_rotations import make_evaluator

        return make_evaluator(self)

    def evaluate_cost(self):
        """approximate_compiler.py:514-527."""
        self.cost_evaluation_counter += 1
        if self.optimise_local_cost:
            return self.backend.evaluate_local_cost(self)
        return self.backend.evaluate_global_cost(self)


def product_state_to_circuit(svec):
    """One single-qubit unitary per qubit with column 0 = the qubit's state (U = [[a, conj(b)],
    [b, -conj(a)]], utilityfunctions.py:341-352), written in rz / ry / rz (the reference
    transpiles to the basis rx, ry, rz; any such form prepares the same state up to phase)."""
    n = len(svec)
    qc = QuantumCircuit(n)
    for q, (a, b) in enumerate(svec):
        u = [[a, b.conjugate()], [b, -a.conjugate()]]
        theta, phi, lam = co.zyz_angles(u)
        for name, ang in (("rz", lam), ("ry", theta), ("rz", phi)):
            if abs(ang) > 1e-14:
                qc.append(co.create_1q_gate(name, float(ang)), [q])
    return qc
