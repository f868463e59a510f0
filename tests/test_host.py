"""Host-side logic of the product (no GPU): IR, gate conventions, generators, selection, packing."""
import numpy as np
import pytest

from oracle import adapt_host as H
from oracle import gradients as ogr
from oracle import sv as osv


def _as_oracle_ops(qc):
    return [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in qc.data]


def test_gate_matrices_match_oracle():
    from adaptaqc_amd import gates as G
    from oracle import gates as OG

    for name in ("x", "y", "z", "h", "s", "sdg", "t", "tdg", "sx"):
        np.testing.assert_allclose(G.one_qubit(name), OG.matrix(name))
    for name in ("rx", "ry", "rz", "p"):
        np.testing.assert_allclose(G.one_qubit(name, [0.37]), OG.matrix(name, (0.37,)))
    np.testing.assert_allclose(G.one_qubit("u", [0.3, 0.5, -0.2]), OG.matrix("u3", (0.3, 0.5, -0.2)))
    for name in ("cx", "cy", "cz", "swap"):
        np.testing.assert_allclose(G.two_qubit(name), OG.matrix(name))


def test_ccx_decomposition_exact():
    """Host unrolling of ccx (readme_example.py:19) equals the 8x8 Toffoli up to rounding."""
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops
    from adaptaqc_amd.utils.gradients import circuit_unitary

    qc = QuantumCircuit(3)
    qc.ccx(2, 1, 0)
    pieces = QuantumCircuit(3)
    for m, q in device_ops(qc):
        pieces.unitary(m, q)
    u = circuit_unitary(pieces)
    want = np.zeros((8, 8), complex)
    for c in range(8):
        v = np.zeros(8, complex)
        v[c] = 1
        want[:, c] = osv.simulate(3, [("ccx", (2, 1, 0), ())], v)
    np.testing.assert_allclose(u, want, atol=1e-14)


def test_circuit_unitary_matches_oracle():
    from adaptaqc_amd.utils import ansatzes
    from adaptaqc_amd.utils.gradients import circuit_unitary

    for f in (ansatzes.u4, ansatzes.thinly_dressed_cnot, ansatzes.fully_dressed_cnot, ansatzes.heisenberg):
        qc = f()
        for i, ins in enumerate(qc.data):
            if ins.operation.params:
                ins.operation.params = [0.1 * (i + 1)]
        np.testing.assert_allclose(circuit_unitary(qc), ogr.ops_matrix(_as_oracle_ops(qc)), atol=1e-14)


def test_inverse_and_compose():
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.utils.gradients import circuit_unitary

    qc = QuantumCircuit(2)
    qc.rx(0.3, 0)
    qc.u(0.2, 0.4, -0.1, 1)
    qc.s(0)
    qc.cx(1, 0)
    qc.t(1)
    np.testing.assert_allclose(circuit_unitary(qc.inverse()) @ circuit_unitary(qc), np.eye(4), atol=1e-14)
    big = QuantumCircuit(4).compose(qc, [3, 1])
    assert [i.qubits for i in big.data] == [(3,), (1,), (3,), (1, 3), (1,)]


def test_generator_tables_match_reference_counts():
    """test_gradients.py:177-204 through the product's own generator code."""
    from adaptaqc_amd.utils import ansatzes
    from adaptaqc_amd.utils.gradients import get_generators_and_degeneracies

    layers = [ansatzes.fully_dressed_cnot(), ansatzes.heisenberg(), ansatzes.identity_resolvable(),
              ansatzes.thinly_dressed_cnot(), ansatzes.u4()]
    expect = [(8, 12, 12, 36), (5, 5, 15, 15), (4, 6, 12, 18), (4, 4, 12, 12), (11, 15, 21, 45)]
    for layer, e in zip(layers, expect):
        g1, d1 = get_generators_and_degeneracies(layer, rotoselect=False)
        g2, d2 = get_generators_and_degeneracies(layer, rotoselect=True)
        assert (len(g1), sum(d1), len(g2), sum(d2)) == e
        og, od = ogr.get_generators_and_degeneracies(_as_oracle_ops(layer), True, True)
        pg, pd = get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
        assert [_as_oracle_ops(x) for x in pg] == og and pd == od


def test_coupling_maps_and_permutations():
    from adaptaqc_amd.utils.constants import CMAP_FULL, CMAP_LADDER, CMAP_LINEAR, generate_coupling_map
    from adaptaqc_amd.utils.utilityfunctions import remove_permutations_from_coupling_map

    assert generate_coupling_map(50, CMAP_FULL) == H.coupling_map_full(50)
    assert len(generate_coupling_map(50, CMAP_FULL)) == 1225
    assert generate_coupling_map(5, CMAP_LINEAR) == H.coupling_map_linear(5)
    assert generate_coupling_map(6, CMAP_LADDER) == [(0, 1), (2, 3), (4, 5), (1, 2), (3, 4)]
    both = generate_coupling_map(4, CMAP_FULL, both_dir=True)
    assert remove_permutations_from_coupling_map(both) == H.coupling_map_full(4)


def test_reuse_priorities_against_oracle():
    from adaptaqc_amd.compilers.adapt.pair_selection import best_gradient_pair, reuse_priorities

    rng = np.random.default_rng(0)
    cmap = H.coupling_map_full(8)
    for _ in range(20):
        hist = [cmap[i] for i in rng.integers(0, len(cmap), rng.integers(0, 6))]
        for mode in ("pair", "qubit"):
            for k in (0, 1, 2.5):
                np.testing.assert_allclose(reuse_priorities(cmap, hist, k, mode), H.reuse_priorities(cmap, hist, k, mode))
        g = rng.integers(0, 3, len(cmap)).astype(float)
        assert best_gradient_pair(cmap, g, hist, 1) == H.best_gradient_pair(cmap, g, hist, 1)


def test_sinusoid_and_stopping():
    from adaptaqc_amd.utils.utilityfunctions import has_stopped_improving, minimum_of_sinusoidal

    for v in ((0.3, 0.9, 0.1), (0.5, 0.2, 0.6)):
        assert minimum_of_sinusoidal(*v) == H.minimum_of_sinusoidal(*v)
    assert has_stopped_improving([1.0, 1.0, 1.0]) == H.has_stopped_improving([1.0, 1.0, 1.0])
    assert has_stopped_improving([1.0, 0.5, 0.1]) == H.has_stopped_improving([1.0, 0.5, 0.1])


def test_statevector_probabilities():
    from adaptaqc_amd.statevector import Statevector

    psi = osv.simulate(3, [("x", (0,), ()), ("h", (1,), ()), ("ry", (2,), (0.7,))])
    st = Statevector(psi)
    for q in range(3):
        p = st.probabilities([q])
        assert abs((p[0] - p[1]) - osv.z_expectations(psi, 3)[q]) < 1e-14
    p2 = st.probabilities([0, 2])
    assert p2.shape == (4,) and abs(p2.sum() - 1) < 1e-14


def test_op_packing_layout():
    from adaptaqc_amd import _lib
    from adaptaqc_amd import gates as G

    arr = _lib.ops_array([(G.one_qubit("ry", [0.5]), (3,)), (G.two_qubit("cz"), (1, 4))])
    assert arr.itemsize == 272 and arr["nq"].tolist() == [1, 2]
    assert arr[1]["q0"] == 1 and arr[1]["q1"] == 4
    m = arr[0]["m"][:8:2] + 1j * arr[0]["m"][1:8:2]
    np.testing.assert_allclose(m.reshape(2, 2), G.one_qubit("ry", [0.5]))


def test_product_state_vectors():
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.utils.gradients import product_state_vectors

    sc = QuantumCircuit(3)
    sc.ry(0.4, 1)
    sc.rz(0.2, 1)
    s = product_state_vectors(3, sc)
    psi = osv.simulate(3, [("ry", (1,), (0.4,)), ("rz", (1,), (0.2,))])
    np.testing.assert_allclose(np.kron(np.kron(s[2], s[1]), s[0]), psi, atol=1e-15)
    sc.cx(0, 2)
    assert product_state_vectors(3, sc) is None


def test_mps_format_helpers():
    from adaptaqc_amd.mps_operations import _preprocess_mps, check_mps, chi_cap_for, zero_aer_mps

    z = zero_aer_mps(5)
    assert check_mps(z) and not check_mps([np.zeros((2, 1, 1))] * 5)
    pre = _preprocess_mps(z)
    assert all(x.shape == (2, 1, 1) for x in pre)
    assert chi_cap_for(50, 64) == 64 and chi_cap_for(6, None) == 8
    assert chi_cap_for(50, 512) == 512 and chi_cap_for(50, 1024) == 1024
    with pytest.raises(NotImplementedError):
        chi_cap_for(50, 2048)


def test_unbounded_capacity_grows_on_demand():
    """max_chi None: the smallest power of two >= 64 holding the loaded MPS, doubled after each
    overflow up to min(1024, 2^(n/2)); bounded runs never grow."""
    from adaptaqc_amd import mps_operations as mo

    saved = dict(mo._UNBOUNDED_CAP)
    try:
        mo._UNBOUNDED_CAP.clear()
        assert mo.chi_cap_for(20, None) == 64 and mo.chi_cap_for(16, None) == 64
        assert mo.chi_cap_for(20, None, 100) == 128 and mo.chi_cap_for(6, None) == 8
        assert mo.grow_capacity(20, None, 64) and mo.chi_cap_for(20, None) == 128
        assert mo.grow_capacity(20, None, 128) and mo.grow_capacity(20, None, 256)
        assert mo.chi_cap_for(20, None) == 512 and mo.grow_capacity(20, None, 512)
        assert mo.chi_cap_for(20, None) == 1024 and not mo.grow_capacity(20, None, 1024)
        assert mo.chi_cap_for(16, None) == 64 and not mo.grow_capacity(16, 64, 64)
        assert mo.grow_capacity(16, None, 128) and mo.chi_cap_for(16, None) == 256
        assert not mo.grow_capacity(16, None, 256)  # 2^(16/2)
        assert mo.is_capacity_error(RuntimeError("MPS bond capacity (chi_cap) exceeded: increase chi_cap"))
    finally:
        mo._UNBOUNDED_CAP.clear()
        mo._UNBOUNDED_CAP.update(saved)


def test_learned_capacity_is_scoped_to_the_simulator():
    """the capacity an unbounded replay needed belongs to the backend's simulator (not
    the process) and a compile starts afresh: another backend on as many qubits starts at 64."""
    from adaptaqc_amd import mps_operations as mo
    from adaptaqc_amd.backends.aer_mps_backend import AerMPSBackend

    a, b = AerMPSBackend(), AerMPSBackend()
    la, lb = mo.learned_capacities(a.simulator), mo.learned_capacities(b.simulator)
    assert la is not lb and la is not mo._UNBOUNDED_CAP
    assert mo.grow_capacity(20, None, 64, la) and mo.grow_capacity(20, None, 128, la)
    assert mo.chi_cap_for(20, None, 1, la) == 256 and mo.chi_cap_for(20, None, 1, lb) == 64
    a.reset_learned_capacity()
    assert mo.chi_cap_for(20, None, 1, mo.learned_capacities(a.simulator)) == 64


def test_backends_pickle_without_device_state():
    import pickle

    from adaptaqc_amd.backends.python_default_backends import MPS_SIM, SV_SIM

    for be in (SV_SIM, MPS_SIM):
        clone = pickle.loads(pickle.dumps(be))
        assert type(clone) is type(be)
    assert MPS_SIM.simulator.options.matrix_product_state_truncation_threshold == 1e-16


def test_isinstance_switches():
    """approximate_compiler.py:113 and utilityfunctions.py:122-130 switch on these types."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend, HipMPSBackend, HipSVBackend
    from adaptaqc_amd.utils.utilityfunctions import is_statevector_backend

    assert is_statevector_backend(HipSVBackend()) and not is_statevector_backend(HipMPSBackend())
    assert isinstance(HipMPSBackend(), AerMPSBackend) and issubclass(HipSVBackend, AerSVBackend)


def test_isl_pair_selection_host_logic(monkeypatch):
    """adapt_compiler.py:858-919 on synthetic histories: reuse priority, bad pairs, threshold."""
    from adaptaqc_amd.backends import AerSVBackend
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig

    qc = QuantumCircuit(3)
    qc.h(0)
    comp = AdaptCompiler(qc, backend=AerSVBackend(), adapt_config=AdaptConfig(bad_qubit_pair_memory=2))
    cmap = comp.coupling_map
    monkeypatch.setattr(comp, "_find_best_expectation_qubit_pair", lambda: "expectation")
    ems = [0.1 * (i + 1) for i in range(len(cmap))]
    comp.entanglement_measures_history.append(ems)
    assert comp._find_best_entanglement_qubit_pair(ems) == cmap[-1]
    comp.qubit_pair_history.append(cmap[-1])
    # entanglement of the chosen pair did not go down -> bad pair, masked while in memory
    comp.entanglement_measures_history.append(list(ems))
    pick = comp._find_best_entanglement_qubit_pair(ems)
    assert cmap[-1] in comp.bad_qubit_pairs and pick != cmap[-1]
    # everything below the threshold -> expectation fall-back
    tiny = [1e-12] * len(cmap)
    comp.entanglement_measures_history.append(tiny)
    comp.qubit_pair_history.append(pick)
    assert comp._find_best_entanglement_qubit_pair(tiny) == "expectation"


def test_ops_batch_marshalling():
    """device.OpsBatch: one pointer and count per op list, pointing at the held arrays (so in-place
    angle updates are seen by the next apply), lists converted like apply_batch's."""
    import ctypes

    from adaptaqc_amd import _lib, gates
    from adaptaqc_amd.device import OpsBatch

    lists = [[(gates.one_qubit("rx", [0.1 * k]), (0,)), (gates.TWO_QUBIT["cx"], (0, 1))] for k in range(5)]
    lists.append([])
    arrs = [_lib.ops_array(o) for o in lists[:3]] + lists[3:]
    b = OpsBatch(arrs)
    assert len(b) == 6
    assert list(b.counts) == [2, 2, 2, 2, 2, 0]
    assert b.arrays[0] is arrs[0]  # held, not copied: in-place updates stay visible
    for k in range(3):
        assert b.ptrs[k] == arrs[k].ctypes.data
    assert b.ptrs[5] in (None, 0)
    assert isinstance(b.ptrs, ctypes.Array)


def test_device_preprocessed_mps_list_protocol():
    """DevicePreprocessedMPS fills lazily; every list operation -- the C-level ones
    included (copy, ==, reversed, +, count / index, in-place edits) -- sees the filled contents."""
    from adaptaqc_amd.mps_operations import DevicePreprocessedMPS

    host = [10, 11, 12, 13]  # (stand-ins for the site tensors: the list protocol is what is tested)

    class FakeDevice:
        n = 4

        def preprocessed(self):
            return list(host)

    def fresh():
        return DevicePreprocessedMPS(FakeDevice())

    assert len(fresh()) == 4
    assert fresh().copy() == host
    assert fresh() == host and not (fresh() != host)
    assert list(reversed(fresh())) == host[::-1]
    assert fresh() + [1] == host + [1]
    assert [1] + fresh() == [1] + host
    assert fresh() * 2 == host * 2
    assert fresh().count(12) == 1 and fresh().index(13) == 3
    assert 11 in fresh() and 99 not in fresh()
    d = fresh()
    d.append(7)
    assert len(list(d)) == 5 and d[4] == 7
    d = fresh()
    d[0] = None
    assert d[0] is None and d[1] == 11
    assert repr(fresh()) == repr(host)


def test_partial_trace_cache_invalidates_on_site_replacement(monkeypatch):
    """partial_trace's cache is keyed on the host list and its site objects; replacing
    a site recomputes, and the device copy is not retained."""
    from adaptaqc_amd import mps_operations as mo

    calls = []

    class FakeDev:
        n = 3

        def pair_rdms(self, pairs):
            calls.append(len(pairs))
            return np.stack([np.eye(4, dtype=complex) * len(calls)] * len(pairs))

    monkeypatch.setattr(mo, "_as_device", lambda mps, pre: FakeDev())
    monkeypatch.setattr(mo, "_pt_cache", {"obj": None, "sites": None, "rdms": None})
    mps = [np.zeros((2, 1, 1), complex) for _ in range(3)]
    r1 = mo.partial_trace(mps, [0, 2], True)
    r2 = mo.partial_trace(mps, [1, 0], True)
    assert len(calls) == 1 and r1[0, 0] == 1 and r2[0, 0] == 1
    mps[1] = np.zeros((2, 1, 1), complex)
    r3 = mo.partial_trace(mps, [0, 1], True)
    assert len(calls) == 2 and r3[0, 0] == 2
    assert "dev" not in mo._pt_cache


def test_initial_state_resets_stripped():
    """ADVICE r3 / approximate_compiler.py:481-483: resets (and barriers, delays) leave the
    initial-state circuit before it is used and inverted; a reset after a gate on its qubit
    raises (non-unitary mid-circuit operation)."""
    from adaptaqc_amd.circuit import Operation, QuantumCircuit
    from adaptaqc_amd.compilers.approximate_compiler import initial_state_to_circuit

    qc = QuantumCircuit(3)
    qc.append(Operation("reset", 1), [0])
    qc.h(0)
    qc.append(Operation("barrier", 3), [0, 1, 2])
    qc.cx(0, 1)
    qc.append(Operation("reset", 1), [2])
    out = initial_state_to_circuit(qc)
    assert [i.operation.name for i in out.data] == ["h", "cx"]
    assert [i.operation.name for i in out.inverse().data] == ["cx", "h"]
    bad = QuantumCircuit(2)
    bad.h(0)
    bad.append(Operation("reset", 1), [0])
    with pytest.raises(NotImplementedError):
        initial_state_to_circuit(bad)
