"""Pin the CPU oracle against the reference's own known-answer tests and fixtures."""
import numpy as np

from oracle import adapt_host as H
from oracle import gradients as gr
from oracle import mps as M
from oracle import sv


def _L(spec):
    return [(nm, q, () if nm == "cx" else (0.0,)) for nm, q in spec]


FD = _L([("rz", (0,)), ("ry", (0,)), ("rz", (0,)), ("rz", (1,)), ("ry", (1,)), ("rz", (1,)), ("cx", (0, 1)),
         ("rz", (0,)), ("ry", (0,)), ("rz", (0,)), ("rz", (1,)), ("ry", (1,)), ("rz", (1,))])
HB = _L([("rz", (1,)), ("cx", (1, 0)), ("rz", (0,)), ("ry", (1,)), ("cx", (0, 1)), ("ry", (1,)), ("cx", (1, 0)),
         ("rz", (0,))])
IR = _L([("rx", (0,)), ("rx", (1,)), ("cx", (0, 1)), ("rx", (0,)), ("rx", (1,)), ("cx", (0, 1)), ("rx", (0,)),
         ("rx", (1,))])
TD = _L([("rx", (0,)), ("rx", (1,)), ("cx", (0, 1)), ("rx", (0,)), ("rx", (1,))])
U4 = _L([("rz", (0,)), ("ry", (0,)), ("rz", (0,)), ("rz", (1,)), ("ry", (1,)), ("rz", (1,)), ("cx", (1, 0)),
         ("rz", (0,)), ("ry", (1,)), ("cx", (0, 1)), ("ry", (1,)), ("cx", (1, 0)), ("rz", (0,)), ("ry", (0,)),
         ("rz", (0,)), ("rz", (1,)), ("ry", (1,)), ("rz", (1,))])


def test_cost_table():
    """test_approximate_compiler.py:114-150."""
    zero = []
    neel = [("x", (0,), ()), ("x", (2,), ())]
    ghz = [("h", (0,), ())] + [("cx", (0, i + 1), ()) for i in range(3)]
    had = [("h", (i,), ()) for i in range(4)]
    got = []
    for ops in (zero, neel, ghz, had):
        psi = sv.simulate(4, ops)
        got += [sv.global_cost(psi), sv.local_cost(psi, 4)]
    np.testing.assert_allclose(got, [0, 0, 1, 0.5, 0.5, 0.5, 15 / 16, 0.5], atol=1e-14)


def test_sv_z_known_answer():
    """test_utilityfunctions.py:86-95."""
    psi = sv.simulate(3, [("x", (0,), ()), ("h", (1,), ())])
    np.testing.assert_array_almost_equal(sv.z_expectations(psi, 3), [-1, 0, 1], decimal=15)


def test_mps_z_known_answer():
    """test_utilityfunctions.py:201-211."""
    z0 = M.run_circuit(4, []).preprocessed()
    np.testing.assert_allclose([M.mps_expectation_z(z0, q) for q in range(4)], [1, 1, 1, 1])
    h = M.run_circuit(4, [("h", (q,), ()) for q in range(4)]).preprocessed()
    np.testing.assert_allclose([M.mps_expectation_z(h, q) for q in range(4)], [0, 0, 0, 0], atol=1e-7)


def test_neel_overlap_exactly_one():
    """test_utilityfunctions.py:287-315: product state vs itself through a different route."""
    a = M.run_circuit(3, [("x", (1,), ())]).preprocessed()
    b = M.run_circuit(3, [("h", (1,), ()), ("z", (1,), ()), ("h", (1,), ())]).preprocessed()
    assert abs(abs(M.mps_dot(a, b)) ** 2 - 1) < 1e-14


def test_analytic_gradient():
    """test_gradients.py:39-73 (places=10)."""
    rng = np.random.default_rng(0)
    ops = []
    for _ in range(5):
        ops += [("ry", (0,), (rng.uniform(-3, 3),)), ("rz", (1,), (rng.uniform(-3, 3),)), ("cx", (1, 0), ()),
                ("rx", (0,), (rng.uniform(-3, 3),))]
    s = sv.simulate(2, ops)
    a, b, c = s[0], s[1], s[2]
    expected = np.sqrt(np.imag(np.conj(a) * b) ** 2 + np.real(np.conj(a) * c) ** 2)
    ans = [("rx", (0,), (0.0,)), ("ry", (1,), (0.0,))]
    gens, deg = gr.get_generators_and_degeneracies(ans, False, True)
    psi = M.run_circuit(2, ops).preprocessed()
    got = gr.general_grad_of_pairs_ref(psi, 2, gr.inverse_ops(ans), gens, deg, [(0, 1)])[0]
    assert abs(got - expected) < 1e-10
    got_env = gr.general_grad_of_pairs_env(psi, 2, gr.inverse_ops(ans), gens, deg, [(0, 1)])[0]
    assert abs(got_env - expected) < 1e-10


def test_generator_count_table():
    """test_gradients.py:177-204."""
    expect = [(8, 12, 12, 36), (5, 5, 15, 15), (4, 6, 12, 18), (4, 4, 12, 12), (11, 15, 21, 45)]
    for layer, (d1, t1, d2, t2) in zip((FD, HB, IR, TD, U4), expect):
        g1, deg1 = gr.get_generators_and_degeneracies(layer, False)
        g2, deg2 = gr.get_generators_and_degeneracies(layer, True)
        assert (len(g1), sum(deg1), len(g2), sum(deg2)) == (d1, t1, d2, t2)


def test_known_generators():
    """test_gradients.py:96-130 and :132-155."""
    ans = [("rx", (0,), (0.0,)), ("cx", (0, 1), ())]
    g, _ = gr.get_generators_and_degeneracies(ans, rotoselect=True, inverse=False)
    assert g == [[("x", (0,), ()), ("cx", (0, 1), ())], [("y", (0,), ()), ("cx", (0, 1), ())],
                 [("z", (0,), ()), ("cx", (0, 1), ())]]
    gi, _ = gr.get_generators_and_degeneracies(ans, rotoselect=True, inverse=True)
    assert gi == [[("cx", (0, 1), ()), ("x", (0,), ())], [("cx", (0, 1), ()), ("y", (0,), ())],
                  [("cx", (0, 1), ()), ("z", (0,), ())]]
    ans2 = [("rx", (0,), (0.0,)), ("ry", (1,), (0.0,)), ("cx", (0, 1), ()), ("rz", (0,), (0.0,)),
            ("rx", (1,), (0.0,)), ("cx", (1, 0), ()), ("ry", (0,), (0.0,)), ("rz", (1,), (0.0,)), ("cx", (1, 0), ())]
    assert gr.get_generator(ans2, 3, "ry") == [("cx", (0, 1), ()), ("y", (0,), ())]


def test_degenerate_generators():
    """test_gradients.py:157-175."""
    ans = [("rx", (0,), (0.0,)), ("cx", (0, 1), ()), ("ry", (1,), (0.0,)), ("cx", (0, 1), ()), ("rx", (0,), (0.0,))]
    g, d = gr.get_generators_and_degeneracies(ans)
    assert g == [[("x", (0,), ())], [("cx", (0, 1), ()), ("y", (1,), ()), ("cx", (0, 1), ())]]
    assert d == [2, 1]


def test_mps_matches_sv_and_truncation_monotone():
    rng = np.random.default_rng(3)
    n = 7
    ops = []
    for layer in range(5):
        for q in range(n):
            ops.append(("ry", (q,), (rng.uniform(-3, 3),)))
        for _ in range(3):
            a, b = rng.choice(n, 2, replace=False)
            ops.append(("cx", (int(a), int(b)), ()))
    psi = sv.simulate(n, ops)
    st = M.run_circuit(n, ops)
    np.testing.assert_allclose(M.mps_to_vector(st.preprocessed()), psi, atol=1e-12)
    st2 = M.run_circuit(n, ops, 1e-16, 2)
    assert max(x.shape[2] for x in st2.preprocessed()) <= 2
    ov = abs(M.mps_dot(st2.preprocessed(), st2.preprocessed()))
    assert abs(ov - 1) < 1e-10  # renormalised


def test_truncation_rank_rule():
    s = np.array([0.9, 0.4, 1e-5, 1e-9, 1e-12])
    assert M.truncation_rank(s, 1e-16, None) == 3  # CHOP: 1e-9^2 = 1e-18 and 1e-24 are <= 1e-16
    assert M.truncation_rank(s, 1e-8, None) == 2
    assert M.truncation_rank(s, 1e-16, 2) == 2
    assert M.truncation_rank(np.array([1e-9]), 1e-16, None) == 1


def test_fixtures_are_normalised(random_mps):
    """paper/random_mps: 54 fixtures, 50 qubits, chi = 2, norm 1."""
    assert len(random_mps) == 54
    for seed in (1, 17, 100):
        pre = M.MPS.from_aer(random_mps[seed]).preprocessed()
        assert len(pre) == 50 and max(x.shape[2] for x in pre) == 2
        assert abs(M.mps_dot(pre, pre) - 1) < 1e-12


def test_goldens_reproduce(goldens, random_mps):
    """The committed goldens are what the oracle computes (guards accidental oracle drift)."""
    pre = M.MPS.from_aer(random_mps[1]).preprocessed()
    assert abs(M.mps_dot(pre, M.zero_mps(50)) - complex(goldens["s1_ov0"])) < 1e-15
    layer = IR
    gens, deg = gr.get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
    cmap = H.coupling_map_full(50)[:60]
    got = gr.general_grad_of_pairs_env(pre, 50, gr.inverse_ops(layer), gens, deg, cmap)
    np.testing.assert_allclose(got, goldens["s1_grad_identity_resolvable"][:60], rtol=1e-12, atol=0)


def test_absorption_gate_counts():
    """test_adapt_compiler.py:673-718: gates left un-absorbed after each layer (5 gates/layer)."""
    for freq, maxmod, expect in ((4, 3, [0, 0, 5, 10, 0, 0, 5, 10, 0, 0, 5, 10, 0]),
                                 (4, 5, [5, 10, 15, 20, 5, 10, 15, 20, 5, 10, 15, 20, 5])):
        as_gates = []
        got = []
        for i in range(13):
            as_gates.append(i)
            k = H.num_layers_to_absorb(i, as_gates, freq, maxmod)
            del as_gates[:k]
            got.append(5 * len(as_gates))
        assert got == expect


def test_reuse_priorities_and_argmax():
    cmap = H.coupling_map_full(4)
    hist = [(0, 1), (2, 3), (0, 2)]
    pp = H.reuse_priorities(cmap, hist, 1, "pair")
    assert pp[cmap.index((0, 2))] == -1
    assert abs(pp[cmap.index((0, 1))] - (1 - 2 ** -2)) < 1e-15
    qp = H.reuse_priorities(cmap, hist, 1, "qubit")
    assert qp[cmap.index((0, 2))] == -1
    grads = np.ones(len(cmap))
    assert H.best_gradient_pair(cmap, grads, hist, 0) == cmap[0]


def test_minimum_of_sinusoidal():
    for a, b, c in ((0.3, 1.1, -0.4), (1.0, -2.0, 0.5)):
        f = lambda x: a * np.sin(x + b) + c
        th, val = H.minimum_of_sinusoidal(f(0), f(np.pi / 2), f(-np.pi / 2))
        assert abs(val - (c - abs(a))) < 1e-12 and abs(f(th) - val) < 1e-12


def test_entanglement_oracle_known_answers():
    """oracle/entanglement.py: MPS contraction == SV partial trace; Bell / Werner / product."""
    from oracle import entanglement as OE
    from oracle import mps as M
    from oracle import sv as osv

    rng = np.random.default_rng(3)
    n = 6
    ops = []
    for layer in range(5):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-3, 3),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    ops.append(("cx", (0, 4), ()))
    psi = osv.simulate(n, ops)
    pre = M.run_circuit(n, ops, 1e-16, None).preprocessed()
    for a in range(n):
        for b in range(a + 1, n):
            np.testing.assert_allclose(OE.mps_rdm(pre, a, b), OE.partial_trace_sv(psi, a, b), atol=1e-13)
    bell = np.array([1, 0, 0, 1]) / np.sqrt(2)
    rho = np.outer(bell, bell.conj())
    assert abs(OE.concurrence(rho) - 1) < 1e-12 and abs(OE.eof(rho) - 1) < 1e-12
    assert abs(OE.negativity(rho) - 0.5) < 1e-12 and abs(OE.log_negativity(rho) - 1) < 1e-12
    w = 0.8 * rho + 0.2 / 4 * np.eye(4)
    assert abs(OE.concurrence(w) - 0.7) < 1e-12
    prod = np.kron([1, 0], [np.cos(0.3), np.sin(0.3)])
    assert OE.concurrence(np.outer(prod, prod)) == 0.0
    # qubit ordering of the 2-qubit partial trace: x = 2*bit(hi) + bit(lo)
    psi2 = np.zeros(8, complex)
    psi2[0b100] = 1.0  # qubit 2 = 1
    np.testing.assert_allclose(np.diag(OE.partial_trace_sv(psi2, 0, 2)).real, [0, 0, 1, 0])
