"""ISL entanglement sweep on MI355X vs the oracle (oracle/entanglement.py).

Reference pins: test_entanglement_measures.py:93-112 (SV == MPS concurrence / negativity / EoF at
1e-6 through the compiler's all-pair sweep), :48-52 (concurrence of a random pure 2-qubit
state equals the closed form |<psi|sy sy|psi*>|, qiskit's formula), and known answers (Bell,
Werner, product states).
"""
import numpy as np
import pytest

from conftest import to_circuit
from oracle import entanglement as OE
from oracle import mps as M
from oracle import sv as osv

pytestmark = pytest.mark.gpu


def _random_ops(n, depth, seed, long_range=True):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(depth):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
        if long_range:
            a, b = rng.choice(n, 2, replace=False)
            ops.append(("cx", (int(a), int(b)), ()))
    return ops


def _all_pairs(n):
    return [(a, b) for a in range(n) for b in range(a + 1, n)]


def test_sv_rdms_vs_oracle():
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    n = 9
    ops = _random_ops(n, 5, 1)
    psi = osv.simulate(n, ops)
    st = DeviceSV(n)
    st.apply(device_ops(to_circuit(n, ops)))
    pairs = _all_pairs(n) + [(5, 2), (8, 0)]  # reversed pairs give the same (min, max) ordering
    rho = st.pair_rdms(pairs)
    for (a, b), r in zip(pairs, rho):
        np.testing.assert_allclose(r, OE.partial_trace_sv(psi, a, b), atol=1e-13)


@pytest.mark.parametrize("chi", [None, 8])
def test_mps_rdms_vs_oracle(chi):
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    n = 10
    ops = _random_ops(n, 6, 2)
    ref = M.run_circuit(n, ops, 1e-16, chi)
    d = DeviceMPS(n, 32, 1e-16, chi)
    d.apply(device_ops(to_circuit(n, ops)))
    pre = ref.preprocessed()
    pairs = _all_pairs(n)
    rho = d.pair_rdms(pairs)
    for (a, b), r in zip(pairs, rho):
        np.testing.assert_allclose(r, OE.mps_rdm(pre, a, b), atol=1e-11)
    if chi is None:  # untruncated: equals the statevector partial trace
        psi = osv.simulate(n, ops)
        for (a, b), r in zip(pairs, rho):
            np.testing.assert_allclose(r, OE.partial_trace_sv(psi, a, b), atol=1e-11)


def test_mps_rdms_fifty_qubits_chi64():
    """config-3 sized state (50 q, chi = 64): a spread of pairs against the oracle contraction."""
    import bench
    from adaptaqc_amd.device import DeviceMPS

    q = bench.random_vidal_mps(50, 64, 1000)
    d = DeviceMPS(50, 64, 1e-16, 64)
    d.load_aer(q)
    pre = M.MPS.from_aer(q).preprocessed()
    pairs = [(0, 1), (0, 49), (3, 17), (24, 25), (12, 37), (48, 49), (30, 2)]
    rho = d.pair_rdms(pairs)
    for (a, b), r in zip(pairs, rho):
        want = OE.mps_rdm(pre, a, b)
        np.testing.assert_allclose(r, want, atol=1e-12)
        assert abs(np.trace(r) - 1) < 1e-12


def _random_density(seed, rank):
    rng = np.random.default_rng(seed)
    g = rng.standard_normal((4, rank)) + 1j * rng.standard_normal((4, rank))
    rho = g @ g.conj().T
    return rho / np.trace(rho)


def test_measures_vs_oracle():
    from adaptaqc_amd.device import entanglement_measures

    rhos = [_random_density(s, r) for s in range(12) for r in (1, 2, 4)]
    bell = np.array([1, 0, 0, 1]) / np.sqrt(2)
    rhos.append(np.outer(bell, bell.conj()))
    for p in (0.2, 1 / 3, 0.5, 0.9):
        rhos.append(p * np.outer(bell, bell.conj()) + (1 - p) / 4 * np.eye(4))
    prod = np.kron([np.cos(0.4), np.sin(0.4)], [1, 1j]) / np.sqrt(2)
    rhos.append(np.outer(prod, prod.conj()))
    # 1e-7: for rank-deficient rho the zero eigenvalues of rho rho~ come out as +-1e-17 in any
    # implementation and the reference formula takes their square roots (:290-291), so C
    # carries ~1e-8.5 of rounding noise on both sides (the reference's own SV == MPS test
    # allows 1e-6); full-rank states agree far tighter
    for method in OE.METHODS:
        got = entanglement_measures(np.stack(rhos), method)
        want = [OE.measure(method, r) for r in rhos]
        np.testing.assert_allclose(got, want, atol=1e-7)


def test_known_answers_and_pure_state_formula():
    from adaptaqc_amd.utils import entanglement_measures as em

    bell = np.array([1, 0, 0, 1]) / np.sqrt(2)
    rho = np.outer(bell, bell.conj())
    assert abs(em.concurrence(rho) - 1) < 1e-12
    assert abs(em.eof(rho) - 1) < 1e-10
    assert abs(em.negativity(rho) - 0.5) < 1e-12
    assert abs(em.log_negativity(rho) - 1) < 1e-12
    p = 0.8
    w = p * rho + (1 - p) / 4 * np.eye(4)
    assert abs(em.concurrence(w) - (3 * p - 1) / 2) < 1e-12
    rng = np.random.default_rng(0)
    for _ in range(5):  # pure states: C = |<psi| sy sy |psi*>|
        psi = rng.standard_normal(4) + 1j * rng.standard_normal(4)
        psi /= np.linalg.norm(psi)
        c = abs(psi.conj() @ OE.SY_SY @ psi.conj())
        assert abs(em.concurrence(np.outer(psi, psi.conj())) - c) < 1e-7  # sqrt-of-rounding floor


def test_calculate_entanglement_measure_api():
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.mps_operations import mps_from_circuit
    from adaptaqc_amd.utils import entanglement_measures as em

    ops = _random_ops(4, 3, 7)
    qc = to_circuit(4, ops)
    psi = osv.simulate(4, ops)
    want = OE.concurrence(OE.partial_trace_sv(psi, 0, 2))
    assert abs(em.calculate_entanglement_measure(em.EM_TOMOGRAPHY_CONCURRENCE, qc, 0, 2, AerSVBackend()) - want) < 1e-10
    mps = mps_from_circuit(qc.copy(), return_preprocessed=True)
    got = em.calculate_entanglement_measure(em.EM_TOMOGRAPHY_CONCURRENCE, qc, 0, 2, AerMPSBackend(), mps=mps)
    assert abs(got - want) < 1e-10
    np.testing.assert_allclose(em.partial_trace(psi, 2, 0), OE.partial_trace_sv(psi, 0, 2), atol=1e-13)
    with pytest.raises(ValueError):
        em.calculate_entanglement_measure("nope", qc, 0, 1, AerSVBackend())
    with pytest.raises(NotImplementedError):
        em.calculate_entanglement_measure(em.EM_OBSERVABLE_CONCURRENCE_LOWER_BOUND, qc, 0, 1, AerSVBackend())


def test_sv_and_mps_all_pair_measures_agree():
    """test_entanglement_measures.py:93-112: SV == MPS through the compiler's sweep (1e-6)."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.compilers import AdaptCompiler
    from adaptaqc_amd.utils import entanglement_measures as em

    qc = to_circuit(3, _random_ops(3, 4, 11))
    for method in (em.EM_TOMOGRAPHY_CONCURRENCE, em.EM_TOMOGRAPHY_NEGATIVITY, em.EM_TOMOGRAPHY_EOF):
        sv = AdaptCompiler(qc, entanglement_measure=method, backend=AerSVBackend())
        mps = AdaptCompiler(qc, entanglement_measure=method, backend=AerMPSBackend())
        np.testing.assert_allclose(sv._get_all_qubit_pair_entanglement_measures(),
                                   mps._get_all_qubit_pair_entanglement_measures(), atol=1e-6)


def test_readme_example_default_isl():
    """examples/readme_example.py with the default AdaptConfig (method ISL, SV backend)."""
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.compilers import AdaptCompiler

    qc = QuantumCircuit(3)
    qc.rx(1.23, 0)
    qc.cx(0, 1)
    qc.ry(2.5, 1)
    qc.rx(-1.6, 2)
    qc.ccx(2, 1, 0)
    comp = AdaptCompiler(qc)
    res = comp.compile()
    assert res.overlap > 1 - 1e-2
    assert "ISL" in comp.pair_selection_method_history
    ops = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in res.circuit.data]
    want = osv.simulate(3, [("rx", (0,), (1.23,)), ("cx", (0, 1), ()), ("ry", (1,), (2.5,)), ("rx", (2,), (-1.6,)),
                            ("ccx", (2, 1, 0), ())])
    assert abs(np.vdot(want, osv.simulate(3, ops))) ** 2 > 1 - 1e-2


def test_isl_compile_on_mps():
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.compilers import AdaptCompiler

    ops = _random_ops(5, 2, 3, long_range=False)
    res = AdaptCompiler(to_circuit(5, ops), backend=AerMPSBackend()).compile()
    assert res.overlap > 1 - 1e-2
    got = osv.simulate(5, [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in res.circuit.data])
    assert abs(np.vdot(osv.simulate(5, ops), got)) ** 2 > 1 - 1e-2


@pytest.mark.parametrize("cap", [100, 192, 384, 512])
def test_env_chains_every_capacity_vs_oracle(cap):
    """z_all_batch and pair RDMs at capacities outside the split chains' four (192, 320,
    384 and 448 once ran k_env_split<128>, whose slices overran the scratch) and at 512: two states
    of bond 96 loaded into capacity `cap`, against the oracle's contractions."""
    import bench
    from adaptaqc_amd.device import DeviceMPS, z_all_batch

    n = 14
    qs = [bench.random_vidal_mps(n, 96, 40 + s) for s in range(2)]
    ds = []
    for q in qs:
        d = DeviceMPS(n, cap, 1e-16, None)
        d.load_aer(q)
        ds.append(d)
    z = z_all_batch(ds)
    pairs = [(0, 1), (2, 9), (6, 7), (0, 13), (12, 13)]
    for s, q in enumerate(qs):
        pre = M.MPS.from_aer(q).preprocessed()
        np.testing.assert_allclose(z[s], [M.mps_expectation_z(pre, i) for i in range(n)], atol=1e-11)
        for (a, b), r in zip(pairs, ds[s].pair_rdms(pairs)):
            np.testing.assert_allclose(r, OE.mps_rdm(pre, a, b), atol=1e-11)


@pytest.mark.parametrize("cap", [64, 128])
def test_env_chain_timeout_reruns_single_workgroup(cap):
    """A split chain whose hand-off times out (spin limit 0: every wait not already satisfied) is
    re-run with one workgroup per chain instead of failing the call, counted by
    aqc_env_fallbacks; the values equal the default run's."""
    import ctypes

    import bench
    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceMPS, z_all_batch

    n = 12
    ds = []
    for s in range(3):
        d = DeviceMPS(n, cap, 1e-16, None)
        d.load_aer(bench.random_vidal_mps(n, 48, 70 + s))
        ds.append(d)
    lib = _lib.load()
    cnt = ctypes.c_longlong(0)
    _lib.check(lib.aqc_env_fallbacks(ctypes.byref(cnt)))
    want = z_all_batch(ds)
    want_rdm = ds[0].pair_rdms([(0, 5), (3, 4)])
    _lib.check(lib.aqc_env_set_spin_limit(0.0))
    try:
        got = z_all_batch(ds)
        got_rdm = ds[0].pair_rdms([(0, 5), (3, 4)])
    finally:
        _lib.check(lib.aqc_env_set_spin_limit(-1.0))
    _lib.check(lib.aqc_env_fallbacks(ctypes.byref(cnt)))
    assert cnt.value >= 1
    np.testing.assert_allclose(got, want, atol=1e-12)
    np.testing.assert_allclose(got_rdm, want_rdm, atol=1e-12)
    _lib.check(lib.aqc_env_set_single(1))
    try:
        single = z_all_batch(ds)
    finally:
        _lib.check(lib.aqc_env_set_single(0))
    np.testing.assert_allclose(single, want, atol=1e-12)
