"""Duck-typed stand-ins for the qiskit objects the reference hands its backends (qiskit is not
installed): ``Qubit`` objects that are not integers, ``CircuitInstruction(operation, qubits)``,
gates with ``name / params / num_qubits / to_matrix()``, ``QuantumCircuit.find_bit``, ``copy``,
``compose`` -- and a fake of the reference's own module tree for the ABC registration."""
import abc
import sys
import types

import numpy as np


class Qubit:
    def __init__(self, index):
        self._i = index  # private: code must resolve it through find_bit

    def __repr__(self):
        return f"Qubit(QuantumRegister(n, 'q'), {self._i})"


class Gate:
    def __init__(self, name, num_qubits, params=(), matrix=None, label=None):
        self.name = name
        self.num_qubits = num_qubits
        self.params = list(params)
        self._m = matrix
        self.label = label

    def to_matrix(self):
        if self._m is not None:
            return self._m
        from adaptaqc_amd import gates as G

        vals = [float(p) for p in self.params]
        return G.one_qubit(self.name, vals) if self.num_qubits == 1 else G.two_qubit(self.name, vals)


class CircuitInstruction:
    def __init__(self, operation, qubits, clbits=()):
        self.operation = operation
        self.qubits = tuple(qubits)
        self.clbits = tuple(clbits)


class QuantumCircuit:
    def __init__(self, n):
        self.num_qubits = n
        self.qubits = [Qubit(i) for i in range(n)]
        self._loc = {id(q): i for i, q in enumerate(self.qubits)}
        self.data = []

    def find_bit(self, q):
        return types.SimpleNamespace(index=self._loc[id(q)], registers=[])

    def append(self, op, idx):
        self.data.append(CircuitInstruction(op, [self.qubits[i] for i in idx]))

    def copy(self):
        c = QuantumCircuit(self.num_qubits)
        for ins in self.data:
            c.append(ins.operation, [self.find_bit(q).index for q in ins.qubits])
        return c

    def compose(self, other, qubits=None):
        c = self.copy()
        m = list(range(other.num_qubits)) if qubits is None else list(qubits)
        for ins in other.data:
            c.append(ins.operation, [m[other.find_bit(q).index] for q in ins.qubits])
        return c

    def __len__(self):
        return len(self.data)


def from_ir(ir_circuit):
    """A qiskit-shaped copy of an adaptaqc_amd.circuit.QuantumCircuit (set_matrix_product_state
    becomes an instruction named so with the Aer tuple as params[0], as qiskit-aer's)."""
    out = QuantumCircuit(ir_circuit.num_qubits)
    for ins in ir_circuit.data:
        op = ins.operation
        if op.name == "set_matrix_product_state":
            g = Gate("set_matrix_product_state", ir_circuit.num_qubits, [op.params[0]])
        elif op.name == "unitary":
            g = Gate("unitary", op.num_qubits, [], np.asarray(op.params[0]))
        else:
            g = Gate(op.name, op.num_qubits, op.params, label=getattr(op, "label", None))
        out.append(g, list(ins.qubits))
    return out


def fake_reference_modules():
    """Modules shaped like the reference's backend classes (an ABC AQCBackend with AerMPSBackend /
    AerSVBackend subclasses) and the names reference_binding rebinds; installed in sys.modules.

    The ISL sweep's reference path is restated here as the reference's own code runs it, every
    cross-module name resolved at call time through the module objects as in the reference:
    ``AdaptCompiler._get_all_qubit_pair_entanglement_measures`` (adapt_compiler.py:955-976) ->
    ``calculate_entanglement_measure`` (entanglement_measures.py:39-98) ->
    ``co.run_circuit_without_transpilation`` (circuit_operations_running.py:44-69) ->
    ``backend.simulator.run(...).result().get_statevector()`` and ``partial_trace`` (:325-340), or
    ``mpsops.partial_trace`` on the MPS from ``backend.evaluate_circuit``."""
    class AQCBackend(abc.ABC):
        @abc.abstractmethod
        def evaluate_global_cost(self, compiler):
            pass

    class AerMPSBackend(AQCBackend):
        def evaluate_global_cost(self, compiler):
            raise RuntimeError("reference Aer path")

    class AerSVBackend(AQCBackend):
        def evaluate_global_cost(self, compiler):
            raise RuntimeError("reference Aer path")

    def _aer(*a, **k):
        raise RuntimeError("reference Aer path")

    mods = {}
    for name in ("adaptaqc", "adaptaqc.backends", "adaptaqc.backends.aqc_backend", "adaptaqc.backends.aer_mps_backend",
                 "adaptaqc.backends.aer_sv_backend", "adaptaqc.compilers", "adaptaqc.compilers.approximate_compiler",
                 "adaptaqc.compilers.adapt", "adaptaqc.compilers.adapt.adapt_compiler",
                 "adaptaqc.utils", "adaptaqc.utils.gradients", "adaptaqc.utils.entanglement_measures",
                 "adaptaqc.utils.cost_minimiser",
                 "adaptaqc.utils.circuit_operations", "adaptaqc.utils.utilityfunctions",
                 "aqc_research", "aqc_research.mps_operations"):
        mods[name] = types.ModuleType(name)
    em = mods["adaptaqc.utils.entanglement_measures"]
    co = mods["adaptaqc.utils.circuit_operations"]
    uf = mods["adaptaqc.utils.utilityfunctions"]
    mpsops = mods["aqc_research.mps_operations"]
    ac = mods["adaptaqc.compilers.adapt.adapt_compiler"]

    def is_statevector_backend(backend):  # utilityfunctions.py:122-130
        return isinstance(backend, AerSVBackend)

    def run_circuit_without_transpilation(circuit, backend=None, backend_options=None, execute_kwargs=None,
                                          return_statevector=False):  # circuit_operations_running.py:44-69
        if execute_kwargs is None:
            execute_kwargs = {}
        backend_options = {}  # the device backends are not qiskit-aer AerBackends (:55-56)
        job = backend.simulator.run(circuit, **backend_options, **execute_kwargs)
        result = job.result()
        if uf.is_statevector_backend(backend):
            if return_statevector:
                return result.get_statevector()
            raise NotImplementedError("counts_data_from_statevector is not exercised here")
        return result.get_counts()

    def partial_trace(statevector, a, b):  # entanglement_measures.py:325-340 on the host (qi.partial_trace)
        from oracle.entanglement import partial_trace_sv

        return partial_trace_sv(np.asarray(statevector), a, b)

    def calculate_entanglement_measure(method, circuit, qubit_1, qubit_2, backend, backend_options=None,
                                       execute_kwargs=None, mps=None):  # entanglement_measures.py:39-98
        from oracle import entanglement as oe

        if method == "EM_OBSERVABLE_CONCURRENCE_LOWER_BOUND":
            raise RuntimeError("reference shot path")
        if uf.is_statevector_backend(backend):
            statevector = co.run_circuit_without_transpilation(circuit, backend, return_statevector=True)
            rho = em.partial_trace(statevector, qubit_1, qubit_2)
        elif isinstance(backend, AerMPSBackend):
            rho = mpsops.partial_trace(mps, [qubit_1, qubit_2], already_preprocessed=True)
        else:
            raise RuntimeError("reference tomography path")
        return {"EM_TOMOGRAPHY_EOF": oe.eof, "EM_TOMOGRAPHY_CONCURRENCE": oe.concurrence,
                "EM_TOMOGRAPHY_NEGATIVITY": oe.negativity,
                "EM_TOMOGRAPHY_LOG_NEGATIVITY": oe.log_negativity}[method](np.asarray(rho))

    class AdaptCompiler:
        """The attributes and the ISL method of the reference compiler (adapt_compiler.py:137,
        approximate_compiler.py:113, adapt_compiler.py:955-976)."""

        def __init__(self, full_circuit, backend, coupling_map, entanglement_measure="EM_TOMOGRAPHY_CONCURRENCE"):
            self.full_circuit = full_circuit
            self.backend = backend
            self.coupling_map = list(coupling_map)
            self.entanglement_measure_method = entanglement_measure
            self.backend_options = {}
            self.execute_kwargs = {}
            self.soften_global_cost = False
            self.global_cost_history = []
            self.is_aer_mps_backend = isinstance(self.backend, AerMPSBackend)

        def _get_all_qubit_pair_entanglement_measures(self):
            entanglement_measures = []
            if self.is_aer_mps_backend:
                self.circ_mps = self.backend.evaluate_circuit(self)
            else:
                self.circ_mps = None
            for control, target in self.coupling_map:
                entanglement_measures.append(ac.calculate_entanglement_measure(
                    self.entanglement_measure_method, self.full_circuit, control, target, self.backend,
                    self.backend_options, self.execute_kwargs, self.circ_mps))
            return entanglement_measures

    # ---- the Rotoselect / Rotosolve path: cost_minimiser.py:267-368 as the reference runs it, with
    # circuit_operations_basic.py:70-99 (replace_1q_gate), :202 (SUPPORTED_1Q_GATES) and
    # utilityfunctions.py:34-57 (minimum_of_sinusoidal, restated in oracle/adapt_host.py) ----
    cmod = mods["adaptaqc.utils.cost_minimiser"]

    def create_1q_gate(gate_name, angle):  # circuit_operations_basic.py:20-34
        return Gate(gate_name, 1, [angle], label=gate_name)

    def replace_1q_gate(circuit, gate_index, gate_name, angle):
        if gate_name is None:
            return
        ci = circuit.data[gate_index]
        circuit.data[gate_index] = CircuitInstruction(create_1q_gate(gate_name, angle), ci.qubits, ci.clbits)

    def is_supported_1q_gate(gate):
        return gate.name in co.SUPPORTED_1Q_GATES

    class CostMinimiser:
        def __init__(self, cost_finder, variational_circuit_range, full_circuit, rotosolve_fraction=1.0):
            self.cost_finder = cost_finder
            self.variational_circuit_range = variational_circuit_range
            self.full_circuit = full_circuit
            self.rotosolve_fraction = rotosolve_fraction

        def _reduce_cost(self, change_1q_gate_kind=False, indexes_to_modify=None):
            cost = 1
            variational_circuit_range = self.variational_circuit_range()
            if indexes_to_modify is None:
                indexes_to_modify = variational_circuit_range
            else:
                indexes_to_modify = (max(indexes_to_modify[0], variational_circuit_range[0]),
                                     min(indexes_to_modify[1], variational_circuit_range[1]))
            sample = list(range(*indexes_to_modify))
            for index in sample:
                old_gate = self.full_circuit.data[index].operation
                if change_1q_gate_kind and cmod.co.is_supported_1q_gate(old_gate):
                    cost = self.replace_with_best_1q_gate(index)
                elif cmod.co.is_supported_1q_gate(old_gate):
                    angle, cost = self.find_best_angle(index, old_gate.label)
                    cmod.co.replace_1q_gate(self.full_circuit, index, old_gate.label, angle)
                else:
                    continue
            return cost

        def replace_with_best_1q_gate(self, gate_index):
            cmod.co.replace_1q_gate(self.full_circuit, gate_index, "rx", 0)
            cost_identity = self.cost_finder()
            best_gate_name, best_gate_angle, best_gate_cost = None, None, 1
            for gate_name in cmod.SUPPORTED_1Q_GATES:
                min_angle, cost = self.find_best_angle(gate_index, gate_name, cost_identity)
                if cost < best_gate_cost:
                    best_gate_name, best_gate_angle, best_gate_cost = gate_name, min_angle, cost
            cmod.co.replace_1q_gate(self.full_circuit, gate_index, best_gate_name, best_gate_angle)
            return best_gate_cost

        def find_best_angle(self, gate_index, gate_name, cost_for_identity=None):
            circ_instr = self.full_circuit.data[gate_index]
            costs = []
            angles_to_run = [0, cmod.np.pi / 2, -cmod.np.pi / 2]
            if cost_for_identity is not None:
                costs.append(cost_for_identity)
                angles_to_run.remove(0)
            for theta in angles_to_run:
                cmod.co.replace_1q_gate(self.full_circuit, gate_index, gate_name, theta)
                costs.append(self.cost_finder())
            theta_min, cost_min = cmod.minimum_of_sinusoidal(costs[0], costs[1], costs[2])
            self.full_circuit.data[gate_index] = circ_instr
            return theta_min, cost_min

    CostMinimiser.__module__ = "adaptaqc.utils.cost_minimiser"

    class ApproximateCompiler:
        """The attributes evaluate_cost and the backends read (approximate_compiler.py:514-527)."""

        def __init__(self, full_circuit, backend):
            self.full_circuit = full_circuit
            self.backend = backend
            self.cost_evaluation_counter = 0
            self.optimise_local_cost = False
            self.soften_global_cost = False
            self.global_cost_history = []
            self.backend_options = {}
            self.execute_kwargs = {}

        def evaluate_cost(self):
            self.cost_evaluation_counter += 1
            if self.optimise_local_cost:
                return self.backend.evaluate_local_cost(self)
            return self.backend.evaluate_global_cost(self)

    from oracle.adapt_host import minimum_of_sinusoidal

    co.SUPPORTED_1Q_GATES = ["rx", "ry", "rz"]
    co.replace_1q_gate = replace_1q_gate
    co.is_supported_1q_gate = is_supported_1q_gate
    cmod.np = np
    cmod.co = co
    cmod.SUPPORTED_1Q_GATES = co.SUPPORTED_1Q_GATES
    cmod.minimum_of_sinusoidal = minimum_of_sinusoidal
    cmod.CostMinimiser = CostMinimiser
    mods["adaptaqc.compilers.approximate_compiler"].ApproximateCompiler = ApproximateCompiler
    uf.is_statevector_backend = is_statevector_backend
    co.run_circuit_without_transpilation = run_circuit_without_transpilation
    em.partial_trace = partial_trace
    em.calculate_entanglement_measure = calculate_entanglement_measure
    ac.calculate_entanglement_measure = calculate_entanglement_measure  # imported by name (adapt_compiler.py:35)
    ac.AdaptCompiler = AdaptCompiler
    mpsops.partial_trace = _aer
    mods["adaptaqc.backends.aqc_backend"].AQCBackend = AQCBackend
    mods["adaptaqc.backends.aer_mps_backend"].AerMPSBackend = AerMPSBackend
    mods["adaptaqc.backends.aer_sv_backend"].AerSVBackend = AerSVBackend
    mods["adaptaqc.compilers.approximate_compiler"].mps_from_circuit = _aer
    mods["aqc_research.mps_operations"].mps_from_circuit = _aer
    mods["adaptaqc.utils.gradients"].general_grad_of_pairs = _aer
    return mods


class installed_fake_reference:
    """Context manager: the fake reference modules in sys.modules, restored afterwards."""

    def __enter__(self):
        self.mods = fake_reference_modules()
        self.prev = {k: sys.modules.get(k) for k in self.mods}
        sys.modules.update(self.mods)
        return self.mods

    def __exit__(self, *exc):
        from adaptaqc_amd import reference_binding

        reference_binding.uninstall()
        for k, v in self.prev.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
        return False
