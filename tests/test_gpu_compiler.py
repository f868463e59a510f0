"""End-to-end compiler runs on the GPU backends (reference test_adapt_compiler.py style)."""
import os
import pickle

import numpy as np
import pytest

from conftest import to_circuit
from oracle import sv as osv

pytestmark = pytest.mark.gpu


def _random_state_circuit(n, depth, seed):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(depth):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    return ops


def test_readme_example_expectation_method():
    """examples/readme_example.py circuit compiled on the SV backend (config 1 plumbing)."""
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    qc = QuantumCircuit(3)
    qc.rx(1.23, 0)
    qc.cx(0, 1)
    qc.ry(2.5, 1)
    qc.rx(-1.6, 2)
    qc.ccx(2, 1, 0)
    res = AdaptCompiler(qc, adapt_config=AdaptConfig(method="expectation")).compile()
    assert res.overlap > 1 - 1e-2
    assert res.exact_overlap > 1 - 1e-2
    # independent check of the compiled circuit against the oracle
    ops = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in res.circuit.data]
    want = osv.simulate(3, [("rx", (0,), (1.23,)), ("cx", (0, 1), ()), ("ry", (1,), (2.5,)), ("rx", (2,), (-1.6,)),
                            ("ccx", (2, 1, 0), ())])
    got = osv.simulate(3, ops)
    assert abs(np.vdot(want, got)) ** 2 > 1 - 1e-2


def test_general_gradient_mps_compile():
    """general_gradient pair selection (the paper setting) on the MPS backend."""
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig
    from adaptaqc_amd.utils.ansatzes import identity_resolvable

    ops = _random_state_circuit(4, 3, 5)
    qc = to_circuit(4, ops)
    comp = AdaptCompiler(qc, backend=AerMPSBackend(), adapt_config=AdaptConfig(method="general_gradient"),
                         custom_layer_2q_gate=identity_resolvable())
    res = comp.compile()
    assert res.overlap > 1 - 1e-2
    assert all(m == "general_gradient" for m in res.method_history)
    psi = osv.simulate(4, ops)
    got = osv.simulate(4, [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in res.circuit.data])
    assert abs(np.vdot(psi, got)) ** 2 > 1 - 1e-2


@pytest.mark.parametrize("freq,maxmod,expect", [
    (4, 3, [0, 0, 5, 10, 0, 0, 5, 10, 0, 0, 5, 10, 0]),
    (4, 5, [5, 10, 15, 20, 5, 10, 15, 20, 5, 10, 15, 20, 5]),
])
def test_mps_absorption_counts(freq, maxmod, expect):
    """test_adapt_compiler.py:673-718 on the device MPS backend."""
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    qc = to_circuit(4, _random_state_circuit(4, 3, 1))
    comp = AdaptCompiler(qc, backend=AerMPSBackend(),
                         adapt_config=AdaptConfig(rotosolve_frequency=freq, max_layers_to_modify=maxmod, method="basic"))
    got = []
    for i in range(13):
        comp._add_layer(i)
        got.append(len(comp.full_circuit.data) - 1)
    assert got == expect
    # absorbed + live gates reproduce the same state as the reference circuit of all gates
    from adaptaqc_amd.backends import AerSVBackend
    from conftest import FakeCompiler

    mps_cost = comp.backend.evaluate_global_cost(comp)
    sv_cost = AerSVBackend().evaluate_global_cost(FakeCompiler(
        to_circuit(4, _random_state_circuit(4, 3, 1)).compose(_strip_mps(comp.ref_circuit_as_gates))))
    assert abs(mps_cost - sv_cost) < 1e-8


def _strip_mps(circ):
    c = circ.copy()
    del c.data[0]
    return c


def test_sv_and_mps_compiler_costs_agree():
    """test_approximate_compiler.py:78-112 (global and local cost, SV vs MPS)."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.compilers import AdaptCompiler

    qc = to_circuit(4, _random_state_circuit(4, 4, 9))
    for local in (False, True):
        a = AdaptCompiler(qc, backend=AerSVBackend(), optimise_local_cost=local).evaluate_cost()
        b = AdaptCompiler(qc, backend=AerMPSBackend(), optimise_local_cost=local).evaluate_cost()
        assert abs(a - b) < 1e-10


def test_checkpoint_resume(tmp_path):
    """Checkpoints pickle the whole compiler incl. the GPU backend (adapt_compiler.py:484-506)."""
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    qc = to_circuit(4, _random_state_circuit(4, 2, 3))
    comp = AdaptCompiler(qc, backend=AerMPSBackend(), adapt_config=AdaptConfig(method="basic", max_layers=3),
                         save_circuit_history=True)
    first = comp.compile(checkpoint_every=1, checkpoint_dir=str(tmp_path))
    # one QASM circuit per layer, without the MPS op (adapt_compiler.py:359-366)
    assert len(first.circuit_history) == len(first.qubit_pair_history) >= 1
    assert all(h.startswith("OPENQASM 2.0;") and "set_matrix_product_state" not in h for h in first.circuit_history)
    # the finished state is checkpointed as well (adapt_compiler.py:432-439)
    assert os.path.exists(os.path.join(tmp_path, f"{len(first.qubit_pair_history) - 1}.pkl"))
    with open(os.path.join(tmp_path, "1.pkl"), "rb") as f:
        resumed = pickle.load(f)
    assert resumed.resume_from_layer == 2
    resumed.adapt_config.max_layers = 5
    res = resumed.compile()
    assert len(res.qubit_pair_history) >= 3


def _insert_ansatz(comp, seed):
    """Labelled rotations + CX inserted at the end of the variational range (where ADAPT layers go)."""
    from adaptaqc_amd.circuit import Operation
    from adaptaqc_amd.utils import circuit_operations as co

    rng = np.random.default_rng(seed)
    n = comp.full_circuit.num_qubits
    pos = len(comp.full_circuit.data) - comp.rhs_gate_count
    gates = []
    for layer in range(3):
        for q in range(n):
            gates.append((co.create_1q_gate(["rx", "ry", "rz"][rng.integers(3)], rng.uniform(-2, 2)), [q]))
        for q in range(layer % 2, n - 1, 2):
            gates.append((Operation("cx", 2, []), [q, q + 1]))
    gates.append((Operation("cx", 2, []), [0, n - 1]))
    for q in range(n):
        gates.append((co.create_1q_gate("ry", rng.uniform(-2, 2)), [q]))
    for k, (g, qs) in enumerate(gates):
        co.add_gate(comp.full_circuit, g, pos + k, qs)


@pytest.mark.parametrize("backend_kind,cost", [("sv", "global"), ("mps", "global"), ("sv", "local"), ("mps", "local"),
                                               ("mps", "soft")])
@pytest.mark.parametrize("rotoselect", [False, True])
def test_cached_rotations_match_generic(backend_kind, cost, rotoselect):
    """Cached candidates (utils/cached_rotations.py) reproduce the reference's one-simulation-
    per-candidate sweep: same gates, angles (1e-9), costs (1e-10) and evaluation count -- for the
    global cost, the local cost (optimise_local_cost) and the softened global cost (MPS)."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.compilers import AdaptCompiler

    results = []
    for cached in (False, True):
        backend = AerSVBackend() if backend_kind == "sv" else AerMPSBackend()
        comp = AdaptCompiler(to_circuit(4, _random_state_circuit(4, 3, 21)), backend=backend)
        comp.optimise_local_cost = cost == "local"
        comp.soften_global_cost = cost == "soft"
        if cost == "soft":
            comp.global_cost_history = [0.4]  # (set by compile(); the softening reads its last entry)
        comp.use_cached_rotations = cached
        _insert_ansatz(comp, 5)
        rng = comp.variational_circuit_range()
        assert rng[1] - rng[0] > 10
        start_count = comp.cost_evaluation_counter
        reduced = comp.minimizer._reduce_cost(rotoselect, rng)
        gates = [(i.operation.name, tuple(i.qubits), tuple(i.operation.params)) for i in comp.full_circuit.data]
        results.append((reduced, gates, comp.cost_evaluation_counter - start_count, comp.evaluate_cost()))
    (c0, g0, n0, e0), (c1, g1, n1, e1) = results
    assert n0 == n1
    assert abs(c0 - c1) < 1e-10 and abs(e0 - e1) < 1e-10
    assert [x[:2] for x in g0] == [x[:2] for x in g1]
    for a, b in zip(g0, g1):
        if a[0] in ("rx", "ry", "rz"):
            np.testing.assert_allclose(a[2], b[2], atol=1e-9)


def test_compile_cached_vs_generic_same_result():
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    qc = to_circuit(4, _random_state_circuit(4, 2, 13))
    out = []
    for cached in (False, True):
        comp = AdaptCompiler(qc, adapt_config=AdaptConfig(method="basic", max_layers=6))
        comp.use_cached_rotations = cached
        res = comp.compile()
        out.append((res.overlap, [(i.operation.name, tuple(i.qubits)) for i in res.circuit.data],
                    comp.cost_evaluation_counter))
    assert abs(out[0][0] - out[1][0]) < 1e-8
    assert out[0][1] == out[1][1]
    assert out[0][2] == out[1][2]


@pytest.mark.parametrize("backend_kind", ["sv", "mps"])
@pytest.mark.parametrize("rotoselect", [True, False])
def test_cached_rotations_vs_oracle_sequence(backend_kind, rotoselect):
    """The cached path against the oracle's restatement of _reduce_cost / replace_with_best_1q_gate
    / find_best_angle (oracle/adapt_host.py): per gate the same candidate gates in the same order
    (rx(0), then rx, ry, rz at +-pi/2 for Rotoselect; 0, +-pi/2 of the gate's kind for Rotosolve),
    the same costs (1e-10, the oracle's statevector) and the same final gates and angles."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.compilers import AdaptCompiler
    from adaptaqc_amd.utils.cached_rotations import rotation
    from oracle import adapt_host

    n = 4
    backend = AerSVBackend() if backend_kind == "sv" else AerMPSBackend()
    comp = AdaptCompiler(to_circuit(n, _random_state_circuit(n, 3, 21)), backend=backend)
    _insert_ansatz(comp, 5)
    rng = comp.variational_circuit_range()
    # the oracle sees the whole circuit the cost is taken on: target (expanded), ansatz, start^-1
    if backend_kind == "sv":
        prefix_ops = []
        body = comp.full_circuit
        lo = 0
    else:  # MPS: full_circuit[0] is the target MPS; expand it back to the target's gates
        prefix_ops = _random_state_circuit(n, 3, 21)
        body = comp.full_circuit
        lo = 1
    ops0 = [[op[0], tuple(op[1]), list(op[2]), None] for op in prefix_ops]
    off = len(ops0) - lo
    for ins in body.data[lo:]:
        ops0.append([ins.operation.name, tuple(ins.qubits), list(ins.operation.params), ins.operation.label])
    orng = (rng[0] + off, rng[1] + off)

    def cost_fn(o):
        return 1.0 - abs(osv.simulate(n, [(x[0], x[1], tuple(x[2])) for x in o])[0]) ** 2

    calls = []
    orig = [list(x[:2]) + [list(x[2]), x[3]] for x in ops0]
    adapt_host.reduce_cost(ops0, cost_fn, rotoselect, orng, calls)
    recorded = []
    factory = comp.minimizer.evaluator_factory

    def wrapped():
        ev = factory()
        orig = ev.costs

        def costs(index, mats):
            out = orig(index, mats)
            recorded.append((index, [np.asarray(m) for m in mats], list(out)))
            return out

        ev.costs = costs
        return ev

    comp.minimizer.evaluator_factory = wrapped
    count0 = comp.cost_evaluation_counter
    comp.minimizer._reduce_cost(rotoselect, rng)
    per_gate = 7 if rotoselect else 3
    assert comp.cost_evaluation_counter - count0 == len(calls) == per_gate * len(recorded)
    for g, (index, mats, costs) in enumerate(recorded):
        want = calls[per_gate * g: per_gate * (g + 1)]
        assert all(w[0] - off == index for w in want)
        for m, w, c in zip(mats, want, costs):
            np.testing.assert_allclose(m, rotation(w[1], w[2]), atol=1e-15)
            # the candidate circuit as the reference evaluates it: gates before it already at their
            # optimised values, gates after it still at their original ones
            i = w[0]
            trial = ops0[:i] + [[w[1], ops0[i][1], [w[2]], w[1]]] + orig[i + 1:]
            assert abs(c - cost_fn(trial)) < 1e-10
    got = [(i.operation.name, float(i.operation.params[0])) for i in comp.full_circuit.data[rng[0]:rng[1]]
           if i.operation.name in ("rx", "ry", "rz")]
    want = [(o[0], float(o[2][0])) for o in ops0[orng[0]:orng[1]] if o[0] in ("rx", "ry", "rz")]
    assert [x[0] for x in got] == [x[0] for x in want]
    np.testing.assert_allclose([x[1] for x in got], [x[1] for x in want], atol=1e-9)



def _ops_of(circuit):
    return [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in circuit.data]


@pytest.mark.parametrize("backend_kind", ["sv", "mps"])
def test_initial_ansatz_used_and_frozen(backend_kind):
    """compile(initial_ansatz=...) (adapt_compiler.py:295-300, 536-583): the ansatz's rotations are
    optimised first; here it has the target's own structure (angles perturbed), so it alone reaches
    the sufficient cost and no layer is added; the compiled circuit reproduces the target."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    angles = [0.7, -1.1, 0.4, 1.3, -0.6, 0.9]
    target = QuantumCircuit(3)
    ansatz = QuantumCircuit(3)
    for qc, sh in ((target, 0.0), (ansatz, 0.25)):
        qc.ry(angles[0] + sh, 0)
        qc.ry(angles[1] + sh, 1)
        qc.cx(0, 1)
        qc.rz(angles[2] + sh, 1)
        qc.ry(angles[3] + sh, 2)
        qc.cx(1, 2)
        qc.ry(angles[4] + sh, 2)
        qc.rz(angles[5] + sh, 0)
    backend = AerSVBackend() if backend_kind == "sv" else AerMPSBackend()
    comp = AdaptCompiler(target, backend=backend, adapt_config=AdaptConfig(sufficient_cost=1e-4))
    res = comp.compile(initial_ansatz=ansatz)
    assert comp.initial_ansatz_already_successful
    assert res.overlap > 1 - 1e-3
    assert len(res.qubit_pair_history) == 0
    want = osv.simulate(3, _ops_of(target))
    got = osv.simulate(3, _ops_of(res.circuit))
    assert abs(np.vdot(want, got)) ** 2 > 1 - 1e-3


def test_initial_state_circuit_sv():
    """initial_state (approximate_compiler.py:126-139, 458-492): full circuit = S, U, [ansatz],
    S^-1, so the cost of an ansatz V (stored inverted) is 1 - |<s| V^dagger U |s>|^2 with |s> = S|0>
    -- checked against the oracle for the exact V (cost 0) and a perturbed one.  (AdaptCompiler
    passes initial_state=None, adapt_compiler.py:123-134: the option belongs to the base class.)"""
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.compilers.approximate_compiler import ApproximateCompiler
    from adaptaqc_amd.utils import circuit_operations as co

    class _Fixed(ApproximateCompiler):
        def compile(self):
            raise NotImplementedError

    n = 3
    ops = _random_state_circuit(n, 2, 9)
    target = to_circuit(n, ops)
    init_ops = [("h", (0,), ()), ("ry", (1,), (0.8,)), ("cx", (1, 2), ()), ("rx", (2,), (0.3,))]
    init = to_circuit(n, init_ops)
    comp = _Fixed(target, None, initial_state=init)
    assert comp.full_circuit.num_qubits == n and comp.lhs_gate_count == len(init_ops) + len(ops)
    for shift, expect_zero in ((0.0, True), (0.2, False)):
        v_ops = [(nm, qs, tuple(p + shift for p in ps)) for nm, qs, ps in ops]
        c = _Fixed(target, None, initial_state=init)
        co.add_to_circuit(c.full_circuit, co.circuit_by_inverting_circuit(to_circuit(n, v_ops)),
                          c.variational_circuit_range()[1])
        cost = c.evaluate_cost()
        u_s = osv.simulate(n, init_ops + ops)
        v_s = osv.simulate(n, init_ops + v_ops)
        want = 1 - abs(np.vdot(v_s, u_s)) ** 2
        assert abs(cost - want) < 1e-10, (cost, want)
        assert (cost < 1e-10) == expect_zero
    with pytest.raises(ValueError):
        _Fixed(target, None, initial_state=init, general_initial_state=True)


def test_general_initial_state_sv():
    """general_initial_state (approximate_compiler.py:477-508, adapt_compiler.py:224-233): the
    Bell-pair (Choi) form on 2n qubits compiles the whole unitary, |Tr(V^dagger U)| / 2^n ~ 1."""
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    n = 2
    ops = [("ry", (0,), (0.9,)), ("cx", (0, 1), ()), ("rz", (1,), (-0.7,)), ("rx", (0,), (0.4,))]
    target = to_circuit(n, ops)
    comp = AdaptCompiler(target, general_initial_state=True, adapt_config=AdaptConfig(sufficient_cost=1e-4))
    assert comp.full_circuit.num_qubits == 2 * n
    res = comp.compile()
    assert res.overlap > 1 - 1e-3

    def unitary(o):
        cols = []
        for b in range(2 ** n):
            prep = [("x", (q,), ()) for q in range(n) if (b >> q) & 1]
            cols.append(osv.simulate(n, prep + o))
        return np.stack(cols, axis=1)

    u = unitary(ops)
    v = unitary(_ops_of(res.circuit))
    assert abs(np.trace(v.conj().T @ u)) / 2 ** n > 1 - 1e-3
