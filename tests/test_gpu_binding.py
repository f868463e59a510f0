"""The backends on qiskit-shaped circuits (what the reference's compiler hands them after
reference_binding.install()) give the same results as on this package's IR, and the MPS backend
keeps one device copy of the cached MPS across evaluations."""
import numpy as np
import pytest

from conftest import FakeCompiler
from qiskit_fakes import from_ir, installed_fake_reference

pytestmark = pytest.mark.gpu


def _random_ir(n, seed, layers=4):
    from adaptaqc_amd.circuit import QuantumCircuit

    rng = np.random.default_rng(seed)
    qc = QuantumCircuit(n)
    for layer in range(layers):
        for q in range(n):
            qc.ry(float(rng.uniform(-1, 1)), q)
            qc.rz(float(rng.uniform(-1, 1)), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    qc.cx(0, n - 1)
    return qc


def test_mps_backend_qiskit_shaped_full_circuit():
    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerMPSBackend, mps_sim_with_args
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.mps_operations import mps_from_circuit

    n = 10
    target = _random_ir(n, 1)
    full = QuantumCircuit(n)
    full.set_matrix_product_state(mps_from_circuit(target))
    tail = _random_ir(n, 2, layers=2)
    for ins in tail.data:
        full.data.append(ins.copy())
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        be = AerMPSBackend(mps_sim_with_args(max_chi=8))
        assert isinstance(be, mods["adaptaqc.backends.aer_mps_backend"].AerMPSBackend)
        q_full = from_ir(full)
        c_ir = be.evaluate_global_cost(FakeCompiler(full))
        c_q = be.evaluate_global_cost(FakeCompiler(q_full))
        assert abs(c_ir - c_q) < 1e-13
        base = be._base[1]
        for _ in range(3):  # repeated evaluations: same cached device payload, no re-upload
            assert abs(be.evaluate_global_cost(FakeCompiler(q_full)) - c_q) < 1e-13
            assert be._base[1] is base
        z_ir = be.measure_qubit_expectation_values(FakeCompiler(full))
        z_q = be.measure_qubit_expectation_values(FakeCompiler(q_full))
        np.testing.assert_allclose(z_q, z_ir, atol=1e-13)
        # the patched entry point the reference's compiler calls (approximate_compiler.py:198)
        patched = mods["adaptaqc.compilers.approximate_compiler"].mps_from_circuit
        pre = patched(from_ir(target), return_preprocessed=True, sim=be.simulator)
        assert len(pre) == n and pre[0].shape[0] == 2


def test_sv_backend_qiskit_shaped():
    from adaptaqc_amd.backends import AerSVBackend

    qc = _random_ir(8, 3)
    be = AerSVBackend()
    import os

    os.environ.setdefault("QISKIT_IN_PARALLEL", "FALSE")
    assert abs(be.evaluate_global_cost(FakeCompiler(qc)) - be.evaluate_global_cost(FakeCompiler(from_ir(qc)))) < 1e-14
    np.testing.assert_allclose(be.measure_qubit_expectation_values(FakeCompiler(from_ir(qc))),
                               be.measure_qubit_expectation_values(FakeCompiler(qc)), atol=1e-14)


def test_gradients_qiskit_shaped_inputs():
    """general_grad_of_pairs with the reference's argument types: a qiskit circuit for psi and
    qiskit generator / inverse-ansatz circuits (gradients.py:23-30 signature)."""
    from adaptaqc_amd.utils import ansatzes
    from adaptaqc_amd.utils.gradients import general_grad_of_pairs, get_generators_and_degeneracies

    n = 8
    qc = _random_ir(n, 4)
    layer = ansatzes.identity_resolvable()
    gens, deg = get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
    cmap = [(a, b) for d in range(1, n) for a in range(n - d) for b in [a + d]]
    want = general_grad_of_pairs(qc, layer.inverse(), gens, deg, cmap)
    got = general_grad_of_pairs(from_ir(qc), from_ir(layer.inverse()), [from_ir(g) for g in gens], deg, cmap)
    np.testing.assert_allclose(got, want, atol=1e-14)
    assert max(want) > 1e-3


def _ir_ops(qc):
    """An IR circuit as oracle ops [(name, qubits, params)]."""
    return [(i.operation.name, tuple(i.qubits), tuple(float(p) for p in i.operation.params)) for i in qc.data]


def _oracle_isl(psi, cmap, measure="concurrence"):
    from oracle import entanglement as oe

    return np.array([oe.measure(measure, oe.partial_trace_sv(psi, a, b)) for a, b in cmap])


@pytest.mark.parametrize("measure", ["EM_TOMOGRAPHY_CONCURRENCE", "EM_TOMOGRAPHY_NEGATIVITY"])
def test_reference_isl_sweep_sv(measure):
    """The reference's default configuration (SV backend, ISL, adapt_config.py:25): its ISL loop
    (restated in qiskit_fakes, adapt_compiler.py:955-976 -> entanglement_measures.py:39-98 ->
    circuit_operations_running.py:44-69 -> simulator.run().result().get_statevector() ->
    partial_trace) runs on HipSVBackend after install(), per pair and through the batched wrapper,
    and selects the oracle's pair."""
    import os

    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerSVBackend
    from oracle import sv as osv

    os.environ.setdefault("QISKIT_IN_PARALLEL", "FALSE")
    n = 10
    qc = _random_ir(n, 11)
    cmap = [(a, b) for d in range(1, n) for a in range(n - d) for b in [a + d]]
    name = {"EM_TOMOGRAPHY_CONCURRENCE": "concurrence", "EM_TOMOGRAPHY_NEGATIVITY": "negativity"}[measure]
    want = _oracle_isl(osv.simulate(n, _ir_ops(qc)), cmap, name)
    assert want.max() > 0.05
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        AC = mods["adaptaqc.compilers.adapt.adapt_compiler"].AdaptCompiler
        be = AerSVBackend()
        comp = AC(from_ir(qc), be, cmap, measure)
        per_pair = AC._get_all_qubit_pair_entanglement_measures.__wrapped__(comp)  # the reference's loop
        sim_state = be.simulator._last[2]
        batched = comp._get_all_qubit_pair_entanglement_measures()
        assert comp.circ_mps is None
    np.testing.assert_allclose(per_pair, want, atol=1e-10)
    np.testing.assert_allclose(batched, want, atol=1e-10)
    assert int(np.argmax(per_pair)) == int(np.argmax(want)) == int(np.argmax(batched))
    # one device simulation served all 45 per-pair runs of the unchanged circuit
    assert sim_state is be.simulator._last[2] and len(sim_state._rdms) == len(cmap)


def test_reference_isl_sweep_mps():
    """The reference's ISL loop on HipMPSBackend: evaluate_circuit's MPS (a device-backed
    preprocessed list) through the rebound ``mpsops.partial_trace``, per pair and batched, against
    the oracle; the cached payload is the compiler's leading set_matrix_product_state."""
    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.mps_operations import DevicePreprocessedMPS, mps_from_circuit
    from oracle import sv as osv

    n = 12
    target = _random_ir(n, 21, layers=3)  # shallow enough that pairs keep non-zero concurrence
    tail = _random_ir(n, 22, layers=1)
    full = QuantumCircuit(n)
    full.set_matrix_product_state(mps_from_circuit(target))
    for ins in tail.data:
        full.data.append(ins.copy())
    cmap = [(a, b) for d in range(1, n) for a in range(n - d) for b in [a + d]]
    want = _oracle_isl(osv.simulate(n, _ir_ops(target) + _ir_ops(tail)), cmap)
    assert want.max() > 0.05
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        AC = mods["adaptaqc.compilers.adapt.adapt_compiler"].AdaptCompiler
        be = AerMPSBackend()
        comp = AC(from_ir(full), be, cmap)
        assert comp.is_aer_mps_backend
        per_pair = AC._get_all_qubit_pair_entanglement_measures.__wrapped__(comp)
        assert isinstance(comp.circ_mps, DevicePreprocessedMPS)
        batched = comp._get_all_qubit_pair_entanglement_measures()
        # the host view of the device-backed list is the preprocessed MPS of the same state
        pre = list(comp.circ_mps)
        assert len(pre) == n and all(t.shape[0] == 2 for t in pre)
    np.testing.assert_allclose(per_pair, want, atol=1e-9)
    np.testing.assert_allclose(batched, want, atol=1e-9)
    assert int(np.argmax(per_pair)) == int(np.argmax(want)) == int(np.argmax(batched))
