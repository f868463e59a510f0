"""MPS engine parity on MI355X vs the oracle (1e-6 for truncated MPS; tighter where exact)."""
import numpy as np
import pytest

from conftest import FakeCompiler, golden_ops, to_circuit
from oracle import mps as M
from oracle import sv as osv

pytestmark = pytest.mark.gpu


def _dev_from_aer(q, cap=None, thr=1e-16, max_chi=None):
    from adaptaqc_amd.device import DeviceMPS

    n = len(q[0])
    lmax = max(np.asarray(a).shape[1] for a, _ in q[0])
    d = DeviceMPS(n, cap or max(lmax, 4), thr, max_chi)
    d.load_aer(q)
    return d


def test_fixture_measurements(random_mps, goldens):
    """paper/random_mps fixtures: <psi|0>, <Z_i>, HW-1 amplitudes vs oracle goldens."""
    for seed in (1, 2, 64, 100):
        d = _dev_from_aer(random_mps[seed])
        ov = d.overlap_zero()
        ref = complex(goldens[f"s{seed}_ov0"])
        assert abs(ov - ref) <= 1e-12 * max(1.0, abs(ref)) + 1e-30
        np.testing.assert_allclose(d.z_all(), goldens[f"s{seed}_z"], atol=1e-10)
        np.testing.assert_allclose(d.amps_hw1(), goldens[f"s{seed}_hw1"], atol=1e-14)


def test_vidal_round_trip_unchanged(random_mps):
    """test_utilityfunctions.py:317-338: Gamma/lambda unchanged through set/save."""
    q = random_mps[17]
    d = _dev_from_aer(q)
    gam, lam = d.to_aer()
    for (a, b), (a2, b2) in zip(q[0], gam):
        np.testing.assert_allclose(a, a2)
        np.testing.assert_allclose(b, b2)
    for x, y in zip(q[1], lam):
        np.testing.assert_allclose(x, y)


@pytest.mark.parametrize("chi", [0, 4])
def test_golden_circuits(goldens, chi):
    """Seeded 8-qubit circuits with non-adjacent gates; chi=4 makes truncation bind."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    for seed in range(3):
        ops = golden_ops(goldens, seed)
        d = DeviceMPS(8, 16, 1e-16, chi or None)
        d.apply(device_ops(to_circuit(8, ops)))
        assert abs(d.overlap_zero() - complex(goldens[f"circ{seed}_chi{chi}_ov0"])) < 1e-10
        np.testing.assert_allclose(d.z_all(), goldens[f"circ{seed}_chi{chi}_z"], atol=1e-9)
        np.testing.assert_array_equal(d.dims(), goldens[f"circ{seed}_chi{chi}_dims"])


def test_mps_equals_statevector_without_truncation():
    """SV == MPS when nothing is truncated (test_approximate_compiler.py:78-112 style)."""
    from adaptaqc_amd.circuit import device_ops

    rng = np.random.default_rng(7)
    n = 10
    ops = []
    for layer in range(6):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-np.pi, np.pi),)))
        for _ in range(4):
            a, b = rng.choice(n, 2, replace=False)
            ops.append(("cx", (int(a), int(b)), ()))
    psi = osv.simulate(n, ops)
    from adaptaqc_amd.device import DeviceMPS

    d = DeviceMPS(n, 32)
    d.apply(device_ops(to_circuit(n, ops)))
    pre = d.preprocessed()
    vec = np.array([M.extract_amplitude(pre, i) for i in range(2 ** n)])
    np.testing.assert_allclose(vec, psi, atol=1e-11)


def test_backend_costs_sv_vs_mps():
    """Global / local cost of SV and MPS backends agree (reference: 5 decimals; here 1e-10)."""
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.circuit import QuantumCircuit

    rng = np.random.default_rng(3)
    n = 6
    qc = QuantumCircuit(n)
    for _ in range(5):
        for q in range(n):
            qc.ry(rng.uniform(-1, 1), q)
            qc.rz(rng.uniform(-1, 1), q)
        for q in range(0, n - 1):
            qc.cx(q, q + 1)
    sv_comp = FakeCompiler(qc)
    sv = AerSVBackend()
    mps_b = AerMPSBackend()
    mps_circ = QuantumCircuit(n)
    from adaptaqc_amd.mps_operations import mps_from_circuit

    mps_circ.set_matrix_product_state(mps_from_circuit(qc))
    mps_comp = FakeCompiler(mps_circ)
    assert abs(sv.evaluate_global_cost(sv_comp) - mps_b.evaluate_global_cost(mps_comp)) < 1e-10
    assert abs(sv.evaluate_local_cost(sv_comp) - mps_b.evaluate_local_cost(mps_comp)) < 1e-10


def test_soften_global_cost():
    """aer_mps_backend.py:58-70: C - alpha * sum_i |<e_i|psi>|^2."""
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.mps_operations import mps_from_circuit

    qc = QuantumCircuit(5)
    for q in range(5):
        qc.ry(0.3 + 0.1 * q, q)
    qc.cx(0, 3)
    circ = QuantumCircuit(5)
    circ.set_matrix_product_state(mps_from_circuit(qc))
    be = AerMPSBackend()
    comp = FakeCompiler(circ, soften=True, history=[0.4], sufficient_cost=0.01)
    psi = osv.simulate(5, [("ry", (q,), (0.3 + 0.1 * q,)) for q in range(5)] + [("cx", (0, 3), ())])
    c = 1 - abs(psi[0]) ** 2
    expect = c - abs(0.4 - 0.01) * sum(abs(psi[1 << i]) ** 2 for i in range(5))
    assert abs(be.evaluate_global_cost(comp) - expect) < 1e-12


def test_hadamard_and_zero_z():
    """test_utilityfunctions.py:201-211."""
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.mps_operations import mps_from_circuit

    be = AerMPSBackend()
    for gates, expect in (("", [1, 1, 1, 1]), ("h", [0, 0, 0, 0])):
        qc = QuantumCircuit(4)
        if gates:
            qc.h([0, 1, 2, 3])
        circ = QuantumCircuit(4)
        circ.set_matrix_product_state(mps_from_circuit(qc))
        np.testing.assert_allclose(be.measure_qubit_expectation_values(FakeCompiler(circ)), expect, atol=1e-7)


def test_chi64_fifty_qubits_vs_oracle():
    """50 qubits, max_chi = 64 binding: device replay vs oracle replay of the same ops."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    n, chi = 50, 64
    rng = np.random.default_rng(11)
    ops = []
    for layer in range(14):
        for q in range(n):
            ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
            ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    ops += [("cx", (3, 9), ()), ("cx", (30, 22), ())]
    ref = M.run_circuit(n, ops, 1e-16, chi)
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.apply(device_ops(to_circuit(n, ops)))
    dims = d.dims()
    ref_dims = [1] + [x.shape[2] for x in ref.preprocessed()]
    np.testing.assert_array_equal(dims, ref_dims)
    pre_ref = ref.preprocessed()
    ov_ref = M.mps_dot(pre_ref, M.zero_mps(n))
    ov = d.overlap_zero()
    assert abs(ov - ov_ref) <= 1e-6 * abs(ov_ref) + 1e-18
    zr = np.array([M.mps_expectation_z(pre_ref, q) for q in range(0, n, 7)])
    np.testing.assert_allclose(d.z_all()[0:n:7], zr, atol=1e-6)


def test_batch_apply_matches_single():
    from adaptaqc_amd.device import DeviceMPS, apply_batch, overlap_zero_batch
    from adaptaqc_amd import _lib

    rng = np.random.default_rng(5)
    n = 12
    states, lists = [], []
    for s in range(4):
        ops = []
        for _ in range(20):
            a, b = rng.choice(n, 2, replace=False)
            th = rng.uniform(-3, 3, 2)
            ops.append((np.array([[np.cos(th[0]), -np.sin(th[0])], [np.sin(th[0]), np.cos(th[0])]], complex), (int(a),)))
            ops.append((np.kron(np.eye(2), np.eye(2))[[0, 1, 3, 2]] .astype(complex), (int(a), int(b))))
        lists.append(_lib.ops_array(ops))
        states.append(DeviceMPS(n, 16, 1e-16, 8))
    apply_batch(states, lists)
    ov = overlap_zero_batch(states)
    for s in range(4):
        d = DeviceMPS(n, 16, 1e-16, 8)
        d.apply(lists[s])
        assert abs(d.overlap_zero() - ov[s]) < 1e-13


@pytest.mark.parametrize("gram", [1, 0])
def test_svd_paths_vs_oracle(goldens, gram):
    """Both two-site SVD paths -- the Gram path with the register Jacobi behind it (default), and
    the register Jacobi alone -- reproduce the oracle (small, ragged and full-width theta)."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    _lib.check(_lib.lib().aqc_mps_set_svd_path(gram, 64))
    try:
        for seed in range(3):
            for chi in (0, 4):
                d = DeviceMPS(8, 16, 1e-16, chi or None)
                d.apply(device_ops(to_circuit(8, golden_ops(goldens, seed))))
                assert abs(d.overlap_zero() - complex(goldens[f"circ{seed}_chi{chi}_ov0"])) < 1e-10
                np.testing.assert_array_equal(d.dims(), goldens[f"circ{seed}_chi{chi}_dims"])
        rng = np.random.default_rng(21)
        for n, chi in ((12, 32), (16, 64)):
            ops = []
            for layer in range(8):
                for q in range(n):
                    ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
                    ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
                for q in range(layer % 2, n - 1, 2):
                    ops.append(("cx", (q, q + 1), ()))
            ops.append(("cx", (1, n - 2), ()))
            ref = M.run_circuit(n, ops, 1e-16, chi)
            d = DeviceMPS(n, chi, 1e-16, chi)
            d.apply(device_ops(to_circuit(n, ops)))
            np.testing.assert_array_equal(d.dims(), [1] + [x.shape[2] for x in ref.preprocessed()])
            ov_ref = M.mps_dot(ref.preprocessed(), M.zero_mps(n))
            assert abs(d.overlap_zero() - ov_ref) <= 1e-8 * abs(ov_ref) + 1e-18
    finally:
        _lib.check(_lib.lib().aqc_mps_set_svd_path(1, 64))


def test_copy_batch_matches_single_copies(random_mps):
    from adaptaqc_amd.device import DeviceMPS, copy_batch

    srcs = [_dev_from_aer(random_mps[s], cap=16) for s in (1, 2, 64)]
    dst = [DeviceMPS(len(random_mps[1][0]), 16) for _ in range(5)]
    pick = [srcs[k % 3] for k in range(5)]
    copy_batch(dst, pick)
    for d, s in zip(dst, pick):
        assert abs(d.overlap_zero() - s.overlap_zero()) == 0.0
        np.testing.assert_array_equal(d.dims(), s.dims())
        for (a, b), (a2, b2) in zip(d.to_aer()[0], s.to_aer()[0]):
            np.testing.assert_array_equal(a, a2)
            np.testing.assert_array_equal(b, b2)


def test_jacobi_stop_rule_vs_oracle():
    """A looser sweep stop (last sweep's rotations all |t| <= 1e-6 or 1e-5) keeps a 16-qubit chi = 64
    replay (max_chi binding, 2 chi = 128 thetas) within 1e-9 of the oracle's overlap."""
    import ctypes

    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    rng = np.random.default_rng(33)
    n, chi = 16, 64
    ops = []
    for layer in range(10):
        for q in range(n):
            ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
            ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    ops.append(("cx", (2, n - 3), ()))
    ref = M.run_circuit(n, ops, 1e-16, chi)
    ov_ref = M.mps_dot(ref.preprocessed(), M.zero_mps(n))
    L = _lib.lib()
    _lib.check(L.aqc_mps_set_svd_path(0, 64))  # the register Jacobi itself
    try:
        for tiny in (1e-8, 1e-6, 1e-5):
            _lib.check(L.aqc_mps_set_jacobi_stop(ctypes.c_double(tiny)))
            d = DeviceMPS(n, chi, 1e-16, chi)
            d.apply(device_ops(to_circuit(n, ops)))
            np.testing.assert_array_equal(d.dims(), [1] + [x.shape[2] for x in ref.preprocessed()])
            assert abs(d.overlap_zero() - ov_ref) <= 1e-9 * abs(ov_ref) + 1e-18, tiny
    finally:
        _lib.check(L.aqc_mps_set_jacobi_stop(ctypes.c_double(0.0)))
        _lib.check(L.aqc_mps_set_svd_path(1, 64))


@pytest.mark.parametrize("sort", [False, True])
def test_fused_chain_matches_lockstep_and_oracle(sort):
    """Batched applies at 2 chi = 128 run each state's op list in one fused workgroup (k_chain);
    the result equals the lock-step launches' (1e-12) and the oracle's (1e-9) on 40 states of a
    16-qubit chi = 64 brickwork + long-range gates (swap routing, max_chi binding)."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS, apply_batch, overlap_zero_batch

    n, chi, ns = 16, 64, 40
    rng = np.random.default_rng(41)
    circuits = []
    for s in range(ns):
        ops = []
        for layer in range(6 + s % 5):
            for q in range(n):
                ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
            for q in range(layer % 2, n - 1, 2):
                ops.append(("cx", (q, q + 1), ()))
        a = int(rng.integers(0, n - 1))
        ops.append(("cx", (a, int(rng.integers(a + 1, n))), ()))
        for q in range(0, n, 3):  # trailing 1-qubit gates: standalone one-site ops in the chain
            ops.append(("rx", (q,), (rng.uniform(-np.pi, np.pi),)))
        circuits.append(ops)
    lists = [device_ops(to_circuit(n, ops)) for ops in circuits]
    L = _lib.lib()
    res, stats = {}, {}
    try:
        for fused in (1, 0):
            _lib.check(L.aqc_mps_set_fused_chain(fused))
            st = [DeviceMPS(n, chi, 1e-16, chi) for _ in range(ns)]
            _lib.gram_stats()
            apply_batch(st, lists, sort=sort)
            stats[fused] = _lib.gram_stats()
            res[fused] = (overlap_zero_batch(st), [d.dims() for d in st])
    finally:
        _lib.check(L.aqc_mps_set_fused_chain(1))
    # The two paths form theta' with different kernels (the chain's VALU pass, the lock-step MFMA
    # GEMM), equal to the last bits.  Rank-deficient updates (these |0>-started circuits have many)
    # keep their values above CHOP's band on the Gram path under the certificate, down to its
    # floor lambda_K > 1e-9 lambda_1, where the kept subspace carries eps lambda_1 / lambda_K of
    # error: there last-bit input differences reach the overlaps at ~1e-11, and the paths agree to
    # the Gram path's accuracy (as each does with the oracle below) instead of bit for bit.
    assert stats[1]["certificates"] == stats[0]["certificates"], stats
    tol = 1e-12 if stats[1]["certificates"] == 0 else 1e-9
    np.testing.assert_allclose(res[1][0], res[0][0], rtol=tol, atol=1e-16)
    for a, b in zip(res[1][1], res[0][1]):
        np.testing.assert_array_equal(a, b)
    for s in (0, 7, 39):
        ref = M.run_circuit(n, circuits[s], 1e-16, chi)
        ov_ref = M.mps_dot(ref.preprocessed(), M.zero_mps(n))
        assert abs(res[1][0][s] - ov_ref) <= 1e-9 * abs(ov_ref) + 1e-18


def test_device_memory_cache_reuses_blocks_and_results_unchanged():
    """Handles take their buffers from the library's device-memory cache: creating and dropping
    the same shape again is served from the cache (no hipMalloc), the handed-out bytes return to
    their starting value, and a state built in a reused block is the oracle's (the block is
    re-initialised, nothing of the previous owner leaks in)."""
    import ctypes

    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    L = _lib.lib()

    def stats():
        out = (ctypes.c_double * 5)()
        _lib.check(L.aqc_pool_stats(out))
        return list(out)

    n, chi = 12, 16
    ops = []
    rng = np.random.default_rng(5)
    for layer in range(5):
        for q in range(n):
            ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    dops = device_ops(to_circuit(n, ops))
    want = M.mps_dot(M.run_circuit(n, ops, 1e-16, chi).preprocessed(), M.zero_mps(n))
    for it in range(21):  # (the first pass allocates the shape's blocks: handle, environments)
        if it == 1:
            s0 = stats()
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.apply(dops)
        assert abs(d.overlap_zero() - want) < 1e-10
        d.close()
    s1 = stats()
    assert s1[4] == s0[4], (s0, s1)          # no new hipMalloc for the repeated shape
    assert s1[3] >= s0[3] + 20, (s0, s1)     # every creation served from the cache
    assert s1[1] == s0[1] and s1[2] == s0[2]  # nothing left handed out


@pytest.mark.gpu
@pytest.mark.parametrize("n,cap", [(14, 64), (16, 128), (18, 256)])
def test_z_all_batch_split_environments_vs_oracle(n, cap):
    """<Z_i> of a batch of random states whose capacity splits over the four-workgroup environment
    chains (k_env_split: 16, 32 and 64 columns per workgroup, bonds at the capacity in the middle):
    every value against the oracle's full contraction at 1e-12, and the batch against one state at
    a time."""
    import bench
    from adaptaqc_amd.device import DeviceMPS, z_all_batch

    states, want = [], []
    for seed in range(3):
        q = bench.random_vidal_mps(n, cap, 40 + seed)
        d = DeviceMPS(n, cap, 1e-16, cap)
        d.load_aer(q)
        states.append(d)
        pre = M.MPS.from_aer(q).preprocessed()
        want.append([M.mps_expectation_z(pre, i) for i in range(n)])
    got = z_all_batch(states)
    np.testing.assert_allclose(got, np.array(want), atol=1e-12)
    np.testing.assert_allclose(states[1].z_all(), got[1], atol=1e-13)


@pytest.mark.gpu
def test_z_all_batch_two_rounds_of_chains():
    """30 states at capacity 64: the environment chains run in two rounds (28 states, then 2), on the
    XCD-grouped grid with its padding (56 and 4 chains, padded to 56 and 8): every state's <Z_i>
    equal to its own single-state call, and three of them against the oracle at 1e-12."""
    import bench
    from adaptaqc_amd.device import DeviceMPS, z_all_batch

    n, cap = 14, 64
    states, aers = [], []
    for seed in range(30):
        q = bench.random_vidal_mps(n, cap, 300 + seed)
        d = DeviceMPS(n, cap, 1e-16, cap)
        d.load_aer(q)
        states.append(d)
        aers.append(q)
    got = z_all_batch(states)
    for k in range(30):
        np.testing.assert_allclose(states[k].z_all(), got[k], atol=1e-13)
    for k in (0, 27, 29):
        pre = M.MPS.from_aer(aers[k]).preprocessed()
        np.testing.assert_allclose(got[k], [M.mps_expectation_z(pre, i) for i in range(n)], atol=1e-12)
