"""Candidate-sweep parity on MI355X vs the oracle (gradients.py:23-124)."""
import numpy as np
import pytest

from conftest import to_circuit
from oracle import adapt_host
from oracle import gradients as ogr
from oracle import mps as M
from oracle import sv as osv

pytestmark = pytest.mark.gpu


def _layer(kind):
    from adaptaqc_amd.utils import ansatzes

    return ansatzes.identity_resolvable() if kind == "identity_resolvable" else ansatzes.thinly_dressed_cnot()


def _inputs(kind):
    from adaptaqc_amd.utils.gradients import get_generators_and_degeneracies

    layer = _layer(kind)
    gens, deg = get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
    return layer.inverse(), gens, deg


@pytest.mark.parametrize("kind", ["identity_resolvable", "thinly_dressed"])
def test_fixture_all_pairs(random_mps, goldens, kind):
    """1225-pair sweep on the 50-qubit paper fixtures vs oracle goldens."""
    from adaptaqc_amd.device import DeviceMPS
    from adaptaqc_amd.utils.gradients import grads_for_state

    cmap = [tuple(x) for x in goldens["cmap"]]
    inv0, gens, deg = _inputs(kind)
    for seed in (1, 2, 64, 100):
        d = DeviceMPS(50, 4)
        d.load_aer(random_mps[seed])
        g = np.array(grads_for_state(d, 50, inv0, gens, deg, cmap))
        ref = goldens[f"s{seed}_grad_{kind}"]
        scale = np.max(np.abs(ref))
        np.testing.assert_allclose(g, ref, rtol=0, atol=1e-9 * scale)


def test_analytic_two_qubit_gradient():
    """test_gradients.py:39-73: sqrt(Im(conj(a) b)^2 + Re(conj(a) c)^2), places=10."""
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.utils.gradients import general_grad_of_pairs, get_generators_and_degeneracies

    rng = np.random.default_rng(0)
    qc = QuantumCircuit(2)
    ops = []
    for _ in range(5):
        th = rng.uniform(-3, 3, 3)
        qc.ry(th[0], 0)
        qc.rz(th[1], 1)
        qc.cx(1, 0)
        qc.rx(th[2], 0)
        ops += [("ry", (0,), (th[0],)), ("rz", (1,), (th[1],)), ("cx", (1, 0), ()), ("rx", (0,), (th[2],))]
    s = osv.simulate(2, ops)
    a, b, c = s[0], s[1], s[2]
    expected = np.sqrt(np.imag(np.conj(a) * b) ** 2 + np.real(np.conj(a) * c) ** 2)
    ans = QuantumCircuit(2)
    ans.rx(0, 0)
    ans.ry(0, 1)
    gens, deg = get_generators_and_degeneracies(ans, rotoselect=False, inverse=True)
    got = general_grad_of_pairs(qc, ans.inverse(), gens, deg, coupling_map=[(0, 1)])[0]
    assert abs(got - expected) < 1e-10


def test_no_ansatz_zero_gradient():
    """test_gradients.py:14-37."""
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.utils.gradients import general_grad_of_pairs, get_generators_and_degeneracies

    rng = np.random.default_rng(2)
    qc = QuantumCircuit(5)
    for _ in range(5):
        for q in range(5):
            qc.rx(rng.uniform(-3, 3), q)
        qc.cx(0, 3)
        qc.cx(4, 1)
    start = QuantumCircuit(5)
    for q in range(5):
        start.ry(rng.uniform(-3, 3), q)
    ans = QuantumCircuit(2)
    gens, deg = get_generators_and_degeneracies(ans)
    g = general_grad_of_pairs(qc, ans, gens, deg, [(0, 1), (1, 2), (2, 3), (3, 4)], starting_circuit=start)
    np.testing.assert_array_almost_equal(g, [0, 0, 0, 0])


@pytest.mark.parametrize("kind", ["identity_resolvable", "thinly_dressed"])
def test_product_start_random_state_vs_reference_structure(kind):
    """12-qubit state near |s>, tenpy-like product starting circuit, full map."""
    from adaptaqc_amd.utils.gradients import general_grad_of_pairs

    rng = np.random.default_rng(21)
    n = 12
    ops = []
    for layer in range(4):
        for q in range(n):
            ops.append(("ry", (q,), (0.3 * rng.standard_normal(),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    start_ops = [("ry", (q,), (0.2 * q,)) for q in range(n)] + [("rz", (q,), (0.1,)) for q in range(0, n, 3)]
    cmap = adapt_host.coupling_map_full(n)
    inv0, gens, deg = _inputs(kind)
    got = general_grad_of_pairs(to_circuit(n, ops), inv0, gens, deg, cmap, starting_circuit=to_circuit(n, start_ops))
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in _layer(kind).data]
    o_gens, o_deg = ogr.get_generators_and_degeneracies(o_layer, True, True)
    psi = M.run_circuit(n, ops).preprocessed()
    ref = ogr.general_grad_of_pairs_ref(psi, n, ogr.inverse_ops(o_layer), o_gens, o_deg, cmap, start_ops)
    np.testing.assert_allclose(got, ref, atol=1e-11)
    assert np.max(ref) > 1e-3  # non-trivial gradients


def test_entangled_starting_circuit_device_route():
    from adaptaqc_amd.utils.gradients import general_grad_of_pairs

    n = 6
    rng = np.random.default_rng(4)
    ops = [("ry", (q,), (rng.uniform(-1, 1),)) for q in range(n)] + [("cx", (0, 1), ()), ("cx", (2, 4), ())]
    start = [("h", (0,), ()), ("cx", (0, 5), ()), ("ry", (3,), (0.4,))]
    cmap = adapt_host.coupling_map_full(n)
    inv0, gens, deg = _inputs("thinly_dressed")
    got = general_grad_of_pairs(to_circuit(n, ops), inv0, gens, deg, cmap, starting_circuit=to_circuit(n, start))
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in _layer("thinly_dressed").data]
    o_gens, o_deg = ogr.get_generators_and_degeneracies(o_layer, True, True)
    psi = M.run_circuit(n, ops).preprocessed()
    ref = ogr.general_grad_of_pairs_ref(psi, n, ogr.inverse_ops(o_layer), o_gens, o_deg, cmap, start)
    np.testing.assert_allclose(got, ref, atol=1e-11)


def test_sharded_pairs_equal_full(random_mps):
    """Per-rank pair subsets (first-qubit sharding) reproduce the full sweep bit for bit."""
    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch
    from adaptaqc_amd.sharding import PairShard
    from adaptaqc_amd.utils.gradients import layer_operators

    n = 50
    cmap = adapt_host.coupling_map_full(n)
    inv0, gens, deg = _inputs("identity_resolvable")
    u0, gm = layer_operators(inv0, gens)
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1
    d = DeviceMPS(n, 4)
    d.load_aer(random_mps[35])
    full = pair_grads_batch([d], svec, cmap, u0, np.stack(gm), deg)[0]
    for world in (2, 3, 8):
        got = np.zeros(len(cmap))
        for r in range(world):
            sh = PairShard(cmap, n, r, world)
            part = pair_grads_batch([d], svec, sh.local_pairs, u0, np.stack(gm), deg)[0]
            got[sh.local_index] = part
        np.testing.assert_array_equal(got, full)


def test_argmax_c_abi_tie_break():
    import ctypes

    from adaptaqc_amd import _lib

    rng = np.random.default_rng(0)
    for trial in range(20):
        s = rng.integers(0, 4, 1225).astype(float)
        p = rng.choice([-1.0, 0.5, 1.0], 1225)
        best = ctypes.c_int()
        _lib.check(_lib.lib().aqc_argmax_scaled(_lib.ptr(s), _lib.ptr(p), len(s), 0, ctypes.byref(best)))
        assert best.value == int(np.argmax(s * p))


def test_argmax_rows_batch_matches_numpy():
    """aqc_argmax_scaled_batch (the state-sharded bench's per-state selection, sharding.best_pairs):
    every row's first maximum, including ties and a padded row stride, against np.argmax."""
    import torch

    from adaptaqc_amd.sharding import best_pairs

    rng = np.random.default_rng(3)
    S, ld, count = 37, 1230, 1225
    s = rng.integers(0, 5, (S, ld)).astype(float)
    p = rng.choice([0.25, 0.5, 1.0], count)
    s[5, :] = 2.0  # a whole row tied: index 0 unless p decides
    best, score = best_pairs(torch.as_tensor(s, device="cuda"), p)
    torch.cuda.synchronize()
    want = np.argmax(s[:, :count] * p, axis=1)
    assert best.cpu().numpy().tolist() == want.tolist()
    np.testing.assert_array_equal(score.cpu().numpy(), (s[:, :count] * p)[np.arange(S), want])


def _near_zero_state(n, chi, seed, alpha=0.6):
    """bench.near_product_mps: every bond at min(2^k, 2^(n-k), chi), gradients far from zero."""
    from bench import near_product_mps

    return near_product_mps(n, chi, seed, alpha)


def test_config4_full_size_chi128_vs_oracle():
    """Config 4 size: 50 qubits, chi = 128, identity_resolvable generators, |s> = |0..0>, all 1225
    pairs vs the oracle's environment form (itself pinned to the reference structure)."""
    import bench
    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch
    from adaptaqc_amd.utils import ansatzes

    n, chi = 50, 128
    aer = _near_zero_state(n, chi, 3)
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(aer)
    assert d.dims().max() == chi
    cmap = adapt_host.coupling_map_full(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    got = pair_grads_batch([d], svec, cmap, u0, gm, deg)[0]
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in ansatzes.identity_resolvable().data]
    o_gens, o_deg = ogr.get_generators_and_degeneracies(o_layer, True, True)
    psi = M.MPS.from_aer(aer).preprocessed()
    ref = ogr.general_grad_of_pairs_env(psi, n, ogr.inverse_ops(o_layer), o_gens, o_deg, cmap)
    assert np.max(ref) > 1e-3
    np.testing.assert_allclose(got, ref, atol=1e-10)


def test_unbounded_cap512_general_gradient():
    """an unbounded MPS (max_chi None, the reference's default MPS_SIM) at
    n = 18 that has grown to capacity 512 (chi_cap_for's limit min(512, 2^(n/2))); general_grad_of_pairs
    on it runs the capacity-agnostic segmented sweep (one state, and a batch of two split into
    single states) and matches the oracle's environment form."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS
    from adaptaqc_amd.mps_operations import chi_cap_for
    from adaptaqc_amd.utils.gradients import grads_for_state, layer_operators, pair_grads_batch

    n = 18
    assert chi_cap_for(n, None, 300) == 512
    rng = np.random.default_rng(18)
    ops = []
    for layer in range(3):
        for q in range(n):
            ops.append(("ry", (q,), (float(rng.uniform(-np.pi, np.pi)),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    inv0, gens, deg = _inputs("identity_resolvable")
    cmap = [(a, a + d) for d in range(1, n) for a in range(n - d)]
    states = []
    for k in range(2):
        d = DeviceMPS(n, 512, 1e-16, None)
        d.apply(device_ops(to_circuit(n, ops[: len(ops) - 5 * k])))
        states.append(d)
    one = np.array(grads_for_state(states[0], n, inv0, gens, deg, cmap))
    u0, gmats = layer_operators(inv0, gens)
    svec = np.zeros((n, 2), dtype=complex)
    svec[:, 0] = 1.0
    both = np.array(pair_grads_batch(states, svec, cmap, u0, np.stack(gmats), np.asarray(deg, dtype=float)))
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in _layer("identity_resolvable").data]
    og, od = ogr.get_generators_and_degeneracies(o_layer, True, True)
    for k in range(2):
        ref = ogr.general_grad_of_pairs_env(M.run_circuit(n, ops[: len(ops) - 5 * k]).preprocessed(), n,
                                            ogr.inverse_ops(o_layer), og, od, cmap)
        got = one if k == 0 else both[1]
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-10 * max(1.0, np.max(np.abs(ref))))
    np.testing.assert_allclose(both[0], one, rtol=0, atol=1e-13)
    # the chi = 1 product fit (starting_circuit="tenpy_product_state") at the same capacity
    f = states[0].product_fit(None, 10, 50, 1e-12)[1]
    assert 0.0 < f <= 1.0 + 1e-12
    assert _lib.load() is not None
