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


def _angle_gap(a, b):
    """|a - b| modulo 2 pi (rotations at +pi and -pi differ by a global phase only)."""
    return abs((a - b + np.pi) % (2 * np.pi) - np.pi)


def _thin_layer_ir(full, pairs, rng):
    """Thinly-dressed CNOT layers (rz, rz, cx, rz, rz with the kinds as labels,
    circuit_operations_basic.py:135-189) with random angles appended to ``full``."""
    from adaptaqc_amd.circuit import Operation

    for a, b in pairs:
        for q in (a, b):
            full.append(Operation("rz", 1, [float(rng.uniform(-np.pi, np.pi))], "rz"), [q])
        full.cx(a, b)
        for q in (a, b):
            full.append(Operation("rz", 1, [float(rng.uniform(-np.pi, np.pi))], "rz"), [q])


def _oracle_rotoselect(n, aer, full_ir, start, rotoselect, chi):
    """oracle/adapt_host.py's call sequence (cost_minimiser.py:267-368) with the oracle's MPS replay
    as the cost: (final ops, final cost, evaluation log)."""
    from oracle import adapt_host as AH
    from oracle import mps as M

    ops = []
    for ins in full_ir.data[start:]:
        op = ins.operation
        ops.append([op.name, tuple(ins.qubits), [float(p) for p in op.params], op.label])
    base = M.MPS.from_aer(aer) if aer is not None else None

    def cost_fn(o):
        st = M.run_circuit(n, [(x[0], x[1], tuple(x[2])) for x in o], 1e-16, chi, mps=base)
        return 1.0 - abs(M.mps_dot(st.preprocessed(), M.zero_mps(n))) ** 2

    log, seen = [], []

    def rec(o):
        c = cost_fn(o)
        seen.append(c)
        return c

    cost = AH.reduce_cost(ops, rec, rotoselect, (0, len(ops)), log)
    return ops, cost, log, _amplitudes(ops, seen, rotoselect)


def _amplitudes(ops, seen, rotoselect):
    """Per rotation gate (in order): the amplitude of the cost's sinusoid in the chosen gate's angle
    (minimum_of_sinusoidal's a) from the oracle's evaluations -- where it vanishes the cost does not
    depend on the angle and the fitted angle is rounding noise."""
    out, k = [], 0
    for o in ops:
        if o[0] not in ("rx", "ry", "rz"):
            continue
        if rotoselect:
            c = seen[k:k + 7]
            ax = ("rx", "ry", "rz").index(o[0])
            c0, cp, cm = c[0], c[1 + 2 * ax], c[2 + 2 * ax]
            k += 7
        else:
            c0, cp, cm = seen[k:k + 3]
            k += 3
        cpi = cp + cm - c0
        out.append(0.5 * np.hypot(c0 - cpi, cp - cm))
    return out


@pytest.mark.parametrize("rotoselect", [True, False])
def test_reference_rotoselect_batched_mps(rotoselect):
    """the reference's own CostMinimiser (restated in qiskit_fakes) on a 50-qubit
    chi = 64 MPS target with one thinly-dressed layer, after install(): every gate's 7 (Rotoselect) or
    3 (Rotosolve) candidates come from one batched evaluation (cached prefix MPS + the candidates
    replayed through the suffix together), the reference's selection code runs on them.  Same gate
    kinds and angles as the oracle's call sequence (angles 1e-6, costs 1e-6), the reference's
    cost_evaluation_counter, and the same circuit as the reference's per-candidate path through the
    same device backend (1e-9).  The batched gate's latency is reported against this package's
    own compiler path on the same circuit (cached_rotations) and bounded at 1.5x it."""
    import time

    import bench
    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerMPSBackend, mps_sim_with_args
    from adaptaqc_amd.circuit import QuantumCircuit

    n, chi = 50, 64
    rng = np.random.default_rng(77)
    aer = bench.near_product_mps(n, chi, 12)
    full = QuantumCircuit(n)
    full.set_matrix_product_state(aer)
    _thin_layer_ir(full, [(20, 21)], rng)
    want_ops, want_cost, log, amps = _oracle_rotoselect(n, aer, full, 1, rotoselect, chi)
    n_rot = sum(1 for ins in full.data[1:] if ins.operation.name == "rz")
    be = AerMPSBackend(mps_sim_with_args(max_chi=chi))
    # this package's own compiler path on the same circuit (utils/cached_rotations.py), warmed once
    from adaptaqc_amd.utils.cached_rotations import make_evaluator
    from adaptaqc_amd.utils.cost_minimiser import CostMinimiser as OwnCM
    from conftest import FakeCompiler

    def own_run():
        fc = FakeCompiler(full.copy())
        fc.backend = be
        fc.cost_evaluation_counter = 0
        fc.optimise_local_cost = False

        def own_cost():
            fc.cost_evaluation_counter += 1
            return be.evaluate_global_cost(fc)

        own = OwnCM(own_cost, lambda: (1, len(fc.full_circuit.data)), fc.full_circuit,
                    evaluator_factory=lambda: make_evaluator(fc))
        own_cost()
        t0 = time.perf_counter()
        own._reduce_cost(rotoselect, None)
        return time.perf_counter() - t0

    own_run()
    t_own = own_run()
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        CM = mods["adaptaqc.utils.cost_minimiser"].CostMinimiser
        AC = mods["adaptaqc.compilers.approximate_compiler"].ApproximateCompiler
        runs = {}
        for mode in ("per_candidate", "batched"):
            q = from_ir(full)
            comp = AC(q, be)
            cmz = CM(comp.evaluate_cost, lambda q=q: (1, len(q.data)), q)
            comp.evaluate_cost()  # the cached payload on the device
            comp.cost_evaluation_counter = 0
            t0 = time.perf_counter()
            if mode == "batched":
                cost = cmz._reduce_cost(rotoselect, None)
            else:  # the reference's own per-candidate code on the same device backend
                cost = CM._reduce_cost.__wrapped__(cmz, rotoselect, None)
            runs[mode] = (q, cost, comp.cost_evaluation_counter, time.perf_counter() - t0)
        q, cost, count, t_b = runs["batched"]
        assert count == (7 if rotoselect else 3) * n_rot == len(log)
        assert runs["per_candidate"][2] == count
        assert abs(cost - want_cost) < 1e-6, (cost, want_cost)
        assert abs(cost - runs["per_candidate"][1]) < 1e-9
        r = 0
        for k, ins in enumerate(q.data[1:]):
            w = want_ops[k]
            assert ins.operation.name == w[0], (k, ins.operation.name, w[0])
            if ins.operation.params:  # (angles compared modulo 2 pi: +-pi is one rotation up to phase)
                qp = runs["per_candidate"][0].data[1 + k].operation
                # (an angle the cost does not depend on is rounding noise: the batched costs are
                # contracted through the rewritten window, the per-candidate ones over every site,
                # so their last bits differ)
                if amps[r] > 1e-7:
                    assert _angle_gap(float(ins.operation.params[0]), float(qp.params[0])) < 1e-9, (k, amps[r])
                    assert _angle_gap(float(ins.operation.params[0]), w[2][0]) < 1e-6 / amps[r] + 1e-6
                r += 1
    print(f"\nper gate: reference CostMinimiser batched {1e3 * t_b / n_rot:.2f} ms, per-candidate "
          f"{1e3 * runs['per_candidate'][3] / n_rot:.2f} ms, this package's compiler {1e3 * t_own / n_rot:.2f} ms")
    assert t_b <= 1.5 * t_own + 2e-3 * n_rot
    assert t_b < runs["per_candidate"][3]


def _oracle_cost_fn(n, aer, chi, kind, alpha):
    """The oracle's restatement of the MPS backend's costs (aer_mps_backend.py:49-86): global,
    softened global (1 - |<0|psi>|^2 - alpha sum_i |<e_i|psi>|^2) or local (0.5 (1 - mean <Z_i>))."""
    from oracle import mps as M

    base = M.MPS.from_aer(aer)

    def cost_fn(o):
        st = M.run_circuit(n, [(x[0], x[1], tuple(x[2])) for x in o], 1e-16, chi, mps=base)
        pre = st.preprocessed()
        if kind == "local":
            return 0.5 * (1 - np.mean([M.mps_expectation_z(pre, q) for q in range(n)]))
        g = 1.0 - abs(M.mps_dot(pre, M.zero_mps(n))) ** 2
        if kind == "soft":
            g -= alpha * sum(abs(M.extract_amplitude(pre, 2 ** i)) ** 2 for i in range(n))
        return g

    return cost_fn


@pytest.mark.parametrize("kind", ["local", "soft"])
def test_reference_rotoselect_batched_mps_local_and_softened(kind):
    """the local cost (optimise_local_cost) and the softened global cost
    (soften_global_cost) through the reference's own CostMinimiser after install(): every gate's 7
    Rotoselect candidates from one batch (cached prefix MPS, the candidates replayed through the
    suffix together, then every candidate's <Z_i> -- aqc_mps_z_all_batch -- or HW-1 amplitudes --
    aqc_mps_amps_hw1_batch -- in one set of launches).  Against the oracle's call sequence
    (cost_minimiser.py:267-368 restated, oracle/adapt_host.py) with the oracle's costs: gate kinds,
    resolved angles, final cost 1e-6, the reference's evaluation count; against the reference's
    per-candidate path on the same device backend (1e-9).  Per-gate latency bounded at 1.5x the
    global-cost batch of the same layer."""
    import time
    from types import SimpleNamespace

    import bench
    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerMPSBackend, mps_sim_with_args
    from adaptaqc_amd.circuit import QuantumCircuit
    from oracle import adapt_host as AH

    n, chi = 50, 64
    rng = np.random.default_rng(78)
    aer = bench.near_product_mps(n, chi, 13)
    full = QuantumCircuit(n)
    full.set_matrix_product_state(aer)
    _thin_layer_ir(full, [(20, 21)], rng)
    history, sufficient = [0.31], 1e-2
    alpha = abs(history[-1] - sufficient)
    ops = []
    for ins in full.data[1:]:
        op = ins.operation
        ops.append([op.name, tuple(ins.qubits), [float(p) for p in op.params], op.label])
    cost_fn = _oracle_cost_fn(n, aer, chi, kind, alpha)
    log, seen = [], []

    def rec(o):
        c = cost_fn(o)
        seen.append(c)
        return c

    want_cost = AH.reduce_cost(ops, rec, True, (0, len(ops)), log)
    amps = _amplitudes(ops, seen, True)
    n_rot = sum(1 for ins in full.data[1:] if ins.operation.name == "rz")
    be = AerMPSBackend(mps_sim_with_args(max_chi=chi))
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        CM = mods["adaptaqc.utils.cost_minimiser"].CostMinimiser
        AC = mods["adaptaqc.compilers.approximate_compiler"].ApproximateCompiler
        runs = {}
        for mode in ("global", "per_candidate", "batched", "global", "batched"):
            q = from_ir(full)
            comp = AC(q, be)
            comp.optimise_local_cost = kind == "local" and mode != "global"
            comp.soften_global_cost = kind == "soft" and mode != "global"
            comp.global_cost_history = list(history)
            comp.adapt_config = SimpleNamespace(sufficient_cost=sufficient)
            cmz = CM(comp.evaluate_cost, lambda q=q: (1, len(q.data)), q)
            comp.evaluate_cost()  # the cached payload on the device
            comp.cost_evaluation_counter = 0
            t0 = time.perf_counter()
            if mode == "per_candidate":  # the reference's own per-candidate code on the same backend
                cost = CM._reduce_cost.__wrapped__(cmz, True, None)
            else:
                cost = cmz._reduce_cost(True, None)
            runs[mode] = (q, cost, comp.cost_evaluation_counter, time.perf_counter() - t0)
        q, cost, count, t_b = runs["batched"]
        assert count == 7 * n_rot == len(log)
        assert runs["per_candidate"][2] == count
        assert abs(cost - want_cost) < 1e-6, (cost, want_cost)
        assert abs(cost - runs["per_candidate"][1]) < 1e-9
        r = 0
        for k, ins in enumerate(q.data[1:]):
            w = ops[k]
            assert ins.operation.name == w[0], (k, ins.operation.name, w[0])
            if ins.operation.params:
                qp = runs["per_candidate"][0].data[1 + k].operation
                if amps[r] > 1e-7:  # (as above: a cost-independent angle is rounding noise)
                    assert _angle_gap(float(ins.operation.params[0]), float(qp.params[0])) < 1e-9, (k, amps[r])
                    assert _angle_gap(float(ins.operation.params[0]), w[2][0]) < 1e-6 / amps[r] + 1e-6
                r += 1
    t_g = runs["global"][3]
    print(f"\nper gate ({kind}): batched {1e3 * t_b / n_rot:.2f} ms, global-cost batch {1e3 * t_g / n_rot:.2f} ms, "
          f"per-candidate {1e3 * runs['per_candidate'][3] / n_rot:.2f} ms")
    assert t_b <= 1.5 * t_g + 1e-3 * n_rot
    assert t_b < runs["per_candidate"][3]


def test_reference_rotoselect_batched_sv_local_cost():
    """The local cost on the statevector backend through the reference's CostMinimiser: the cached
    prefix state, each candidate's gate and suffix replayed from it, every <Z_i>; against the
    oracle's call sequence with exact SV local costs (1e-10) and the reference's evaluation count."""
    import os

    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerSVBackend
    from oracle import adapt_host as AH
    from oracle import sv as osv

    os.environ.setdefault("QISKIT_IN_PARALLEL", "FALSE")
    n = 10
    full = _random_ir(n, 6, layers=3)
    start = len(full.data)
    _thin_layer_ir(full, [(3, 4), (6, 2)], np.random.default_rng(6))
    ops = []
    for ins in full.data:
        op = ins.operation
        ops.append([op.name, tuple(ins.qubits), [float(p) for p in op.params], op.label])

    def cost_fn(o):
        psi = osv.simulate(n, [(x[0], x[1], tuple(x[2])) for x in o])
        return 0.5 * (1 - np.mean(osv.z_expectations(psi, n)))

    log = []
    want = AH.reduce_cost(ops, cost_fn, True, (start, len(ops)), log)
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        CM = mods["adaptaqc.utils.cost_minimiser"].CostMinimiser
        AC = mods["adaptaqc.compilers.approximate_compiler"].ApproximateCompiler
        q = from_ir(full)
        comp = AC(q, AerSVBackend())
        comp.optimise_local_cost = True
        cmz = CM(comp.evaluate_cost, lambda: (start, len(q.data)), q)
        assert cmz._reduce_cost.__name__ == "_reduce_cost"
        cost = cmz._reduce_cost(True, None)
        assert comp.cost_evaluation_counter == len(log)
        assert abs(cost - want) < 1e-10
        for k in range(start, len(q.data)):
            op = q.data[k].operation
            assert op.name == ops[k][0]
            if op.params:
                assert _angle_gap(float(op.params[0]), ops[k][2][0]) < 1e-8


def test_reference_rotoselect_batched_sv():
    """The same drop-in on the statevector backend (the transition-matrix evaluator): a 10-qubit
    random state plus one thinly-dressed layer, Rotoselect through the reference's CostMinimiser
    after install(): gate kinds / angles / costs as the oracle's call sequence with exact SV costs
    (1e-10), the reference's evaluation count."""
    import os

    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerSVBackend
    from oracle import adapt_host as AH
    from oracle import sv as osv

    os.environ.setdefault("QISKIT_IN_PARALLEL", "FALSE")
    n = 10
    full = _random_ir(n, 5, layers=3)
    start = len(full.data)
    _thin_layer_ir(full, [(3, 4), (6, 2)], np.random.default_rng(5))
    ops = []
    for ins in full.data:
        op = ins.operation
        ops.append([op.name, tuple(ins.qubits), [float(p) for p in op.params], op.label])

    def cost_fn(o):
        return 1.0 - abs(osv.simulate(n, [(x[0], x[1], tuple(x[2])) for x in o])[0]) ** 2

    log = []
    want = AH.reduce_cost(ops, cost_fn, True, (start, len(ops)), log)
    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        CM = mods["adaptaqc.utils.cost_minimiser"].CostMinimiser
        AC = mods["adaptaqc.compilers.approximate_compiler"].ApproximateCompiler
        q = from_ir(full)
        comp = AC(q, AerSVBackend())
        cmz = CM(comp.evaluate_cost, lambda: (start, len(q.data)), q)
        cost = cmz._reduce_cost(True, None)
        assert comp.cost_evaluation_counter == len(log)
        assert abs(cost - want) < 1e-10
        for k in range(start, len(q.data)):
            op = q.data[k].operation
            assert op.name == ops[k][0]
            if op.params:
                assert _angle_gap(float(op.params[0]), ops[k][2][0]) < 1e-8
