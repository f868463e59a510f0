"""Large-bond MPS updates (2 chi > 128: multi-workgroup block Jacobi, bjacobi.hip) vs the oracle.

BASELINE configs 4 and 5 run at chi = 128 and chi = 256; here the same kernels on states small
enough for the numpy oracle (LAPACK SVDs): random Vidal MPS whose middle bonds sit at the cap,
then adjacent, swap-routed and truncating two-site gates.  Tolerance: the truncated-MPS bar of
BASELINE.json (1e-6), on the fidelity between the device and oracle states, on <Z_i>, and exact
bond dimensions.
"""
import numpy as np
import pytest

from bench import random_vidal_mps  # noqa: E402
from conftest import to_circuit
from oracle import mps as M

pytestmark = pytest.mark.gpu


def _check(n, chi, ops, seed):
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    aer = random_vidal_mps(n, chi, seed)
    ref = M.run_circuit(n, ops, 1e-16, chi, mps=M.MPS.from_aer(aer))
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(aer)
    d.apply(device_ops(to_circuit(n, ops)))
    dims = d.dims()
    pre_ref = ref.preprocessed()
    np.testing.assert_array_equal(dims, [1] + [x.shape[2] for x in pre_ref])
    pre = d.preprocessed()
    fid = abs(M.mps_dot(pre_ref, pre))
    nrm = abs(M.mps_dot(pre, pre))
    assert abs(nrm - 1.0) < 1e-10
    assert abs(fid - 1.0) < 1e-6, fid
    qs = list(range(0, n, 3))
    zr = np.array([M.mps_expectation_z(pre_ref, q) for q in qs])
    np.testing.assert_allclose(d.z_all()[qs], zr, atol=1e-6)
    return dims


def _blas_threads():
    """numpy's BLAS on up to 16 threads for the oracle's large SVDs and contractions (importing bench
    may have pinned it to one for the CPU baseline's workers)."""
    import os

    from threadpoolctl import threadpool_limits

    return threadpool_limits(limits=min(16, os.cpu_count() or 1))


def _gates(n, rng, pairs):
    ops = []
    for a, b in pairs:
        for q in (a, b):
            ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
            ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
        ops.append(("cx", (a, b), ()))
    return ops


@pytest.mark.parametrize("n,chi", [(16, 128), (18, 256)])
def test_block_jacobi_adjacent_and_routed(n, chi):
    """Middle bonds at the cap: adjacent gates (truncation 2chi -> chi binds) and a routed gate."""
    rng = np.random.default_rng(chi)
    m = n // 2
    ops = _gates(n, rng, [(m - 1, m), (m, m + 1), (m + 1, m - 2)])
    dims = _check(n, chi, ops, seed=chi + 1)
    assert dims.max() == chi


def test_block_jacobi_ragged_bonds():
    """Bonds below the cap and non-multiples of the 16-column block (chi_l != chi_r)."""
    rng = np.random.default_rng(3)
    n, chi = 16, 100  # bonds 64 | 100 100 100 | 64: 200-row thetas (12.5 blocks), 128 x 200 (transposed)
    ops = _gates(n, rng, [(7, 8), (6, 7), (8, 9), (2, 3), (0, 1)])
    _check(n, chi, ops, seed=9)


def test_concurrent_disjoint_updates_match_sequential():
    """One brickwork layer applied in one call (disjoint updates share a wave, separate
    workspaces) equals the same gates applied one call at a time, bit for bit."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    n, chi = 16, 128
    rng = np.random.default_rng(8)
    ops = _gates(n, rng, [(a, a + 1) for a in range(0, n - 1, 2)])
    aer = random_vidal_mps(n, chi, 12)
    one = DeviceMPS(n, chi, 1e-16, chi)
    one.load_aer(aer)
    one.apply(device_ops(to_circuit(n, ops)))
    seq = DeviceMPS(n, chi, 1e-16, chi)
    seq.load_aer(aer)
    for k in range(0, len(ops), 5):  # ry, rz, ry, rz, cx per pair
        seq.apply(device_ops(to_circuit(n, ops[k:k + 5])))
    np.testing.assert_array_equal(one.dims(), seq.dims())
    for (a, b), (c, d) in zip(one.to_aer()[0], seq.to_aer()[0]):
        np.testing.assert_array_equal(a, c)
        np.testing.assert_array_equal(b, d)


def test_config5_full_size_vs_oracle():
    """Config 5 at full size: 100 qubits, chi = 256, 24 disjoint updates at the cap in one wave,
    against the oracle's replay (numpy LAPACK SVDs of the 512 x 512 thetas): exact bond dims,
    Schmidt values within 1e-9, normalised descending bonds, fidelity within 1e-6."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    n, chi = 100, 256
    rng = np.random.default_rng(5)
    aer = random_vidal_mps(n, chi, 5)
    ops = _gates(n, rng, [(a, a + 1) for a in range(26, 74, 2)])
    ref = M.run_circuit(n, ops, 1e-16, chi, mps=M.MPS.from_aer(aer))
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(aer)
    d.apply(device_ops(to_circuit(n, ops)))
    pre_ref = ref.preprocessed()
    np.testing.assert_array_equal(d.dims(), [1] + [x.shape[2] for x in pre_ref])
    gam, lam = d.to_aer()
    for b in range(27, 74, 2):  # the truncated bonds
        np.testing.assert_allclose(lam[b - 1], ref.l[b - 1], atol=1e-9, err_msg=f"bond {b}")
    for l in lam:
        assert abs(np.sum(l ** 2) - 1.0) < 1e-10
        assert np.all(np.diff(l) <= 1e-14)
    pre = d.preprocessed()
    fid = abs(M.mps_dot(pre_ref, pre)) / np.sqrt(abs(M.mps_dot(pre, pre)) * abs(M.mps_dot(pre_ref, pre_ref)))
    assert abs(fid - 1.0) < 1e-6, fid


def test_unbounded_chi_above_256_deep_circuit():
    """The reference's default MPS_SIM has no bond-dimension cap (python_default_backends.py:19,
    aer_mps_backend.py:27-42).  A 20-qubit brickwork of depth 18 at max_chi = None grows the middle
    bonds past 256 (oracle: ..., 256, 314, 482, 262, ...); the device replay (the capacity grown on
    demand to 512 -- each overflow re-runs the replay at twice the capacity -- two-site SVDs of up
    to 1024 x 1024) matches the oracle's bond dimensions exactly and its state to 1e-6 fidelity,
    with <0..0|psi> and <Z> beside it."""
    from adaptaqc_amd import mps_operations as mo
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.mps_operations import device_mps_from_circuit

    n, depth = 20, 18
    rng = np.random.default_rng(5)
    ops = []
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            a, b = float(rng.uniform(-np.pi, np.pi)), float(rng.uniform(-np.pi, np.pi))
            ops += [("ry", (q,), (a,)), ("rz", (q,), (b,))]
            qc.ry(a, q)
            qc.rz(b, q)
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
            qc.cx(q, q + 1)
    ref = M.run_circuit(n, ops)
    pre_ref = ref.preprocessed()
    want_dims = [1] + [x.shape[2] for x in pre_ref]
    assert max(want_dims) > 256
    mo._UNBOUNDED_CAP.pop(n, None)  # (start from the smallest capacity: the replay must grow)
    d = device_mps_from_circuit(qc)
    assert d.chi_cap == 512 and mo._UNBOUNDED_CAP[n] == 512
    np.testing.assert_array_equal(d.dims(), want_dims)
    pre = d.preprocessed()
    fid = abs(M.mps_dot(pre_ref, pre))
    assert abs(fid - 1.0) < 1e-6, fid
    assert abs(d.overlap_zero() - M.mps_dot(pre_ref, M.zero_mps(n))) < 1e-9
    qs = [0, 7, 10, 13, 19]
    zr = np.array([M.mps_expectation_z(pre_ref, q) for q in qs])
    np.testing.assert_allclose(d.z_all()[qs], zr, atol=1e-6)


def _golden_cap1024():
    import os

    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cap1024.npz"))


def _product_overlaps(d, phi):
    """<phi_k|psi> on the device without a cap^3 environment chain: a copy of psi rotated qubit by
    qubit by W_q (W_q phi_q = |0>: exact one-qubit gates, no truncation), then <0..0|W psi> =
    <phi|psi> through the zero-chain overlap (overlap_zero returns <psi|0..0>)."""
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops
    from adaptaqc_amd.device import DeviceMPS

    out = []
    c = DeviceMPS(d.n, d.chi_cap, 1e-16, None)
    for p in phi:
        qc = QuantumCircuit(d.n)
        for q, (a, b) in enumerate(p):
            qc.unitary(np.array([[np.conj(a), np.conj(b)], [-b, a]]), [q])
        c.copy_from(d)
        c.apply(device_ops(qc))
        out.append(np.conj(c.overlap_zero()))
    return np.array(out)


def _mps_sv_overlap(pre, psi):
    """<psi|mps> of a preprocessed MPS against a dense little-endian statevector (host)."""
    t = np.asarray(psi).conj().reshape(-1, 1)
    for a in pre:
        t = np.einsum("xsl,slr->xr", t.reshape(t.shape[0] // 2, 2, t.shape[1]), a, optimize=True)
    return complex(t.reshape(-1)[0])


def test_unbounded_chi_above_512_threshold_1e8():
    """VERDICT r5 missing #1: the reference's default MPS_SIM has no bond cap
    (python_default_backends.py:19, aer_mps_backend.py:27-42) and the paper runs it at threshold 1e-8
    (examples/advanced_mps_example.py:46).  A 21-qubit brickwork of depth 24 at max_chi = None,
    threshold 1e-8 grows the middle bonds past 512 (oracle: ..., 256, 511, 800, 704, 509, 256, ...):
    the device replay grows its capacity on demand to 1024 (two-site blocks up to 1600 x 1024 on the
    multi-workgroup Gram path, the Gram side C = min(2 chi_l, 2 chi_r) <= 1024).  Against the
    oracle's goldens (tests/golden/make_cap1024_golden.py): exact bond dimensions, the Schmidt values
    of bonds 9-11 within 1e-9, <0..0|psi> and four product-state overlaps within 1e-10, <Z> within
    1e-6, and the fidelity against the exact state (the device statevector) within 1e-6 of the
    oracle's."""
    import time

    from adaptaqc_amd import mps_operations as mo
    from adaptaqc_amd.backends import mps_sim_with_args
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops
    from adaptaqc_amd.device import DeviceSV
    from adaptaqc_amd.mps_operations import device_mps_from_circuit

    gd = _golden_cap1024()
    n, depth = 21, 24
    rng = np.random.default_rng(5)
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            qc.ry(float(rng.uniform(-np.pi, np.pi)), q)
            qc.rz(float(rng.uniform(-np.pi, np.pi)), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    sim = mps_sim_with_args(mps_truncation_threshold=1e-8)
    t0 = time.perf_counter()
    d = device_mps_from_circuit(qc, sim)
    print(f"device replay (capacity grown to {d.chi_cap}): {time.perf_counter() - t0:.2f} s", flush=True)
    assert d.chi_cap == 1024 and mo.learned_capacities(sim)[n] == 1024
    np.testing.assert_array_equal(d.dims(), gd["brick_dims"])
    gam, lam = d.to_aer()
    for b in (9, 10, 11):  # the bonds above 512 and beside them: Schmidt values
        np.testing.assert_allclose(lam[b], gd[f"brick_lam{b}"], atol=1e-9, err_msg=f"bond {b}")
    assert abs(d.overlap_zero() - complex(gd["brick_ov0"])) < 1e-10
    np.testing.assert_allclose(_product_overlaps(d, gd["brick_phi"]), gd["brick_phi_ov"], atol=1e-10)
    np.testing.assert_allclose(d.z_all()[gd["brick_zq"]], gd["brick_z"], atol=1e-6)
    sv = DeviceSV(n)
    sv.apply(device_ops(qc))
    fid = abs(_mps_sv_overlap(d.preprocessed(), sv.get())) ** 2
    print(f"fidelity vs exact {fid:.12f} (oracle {float(gd['brick_fid_exact']):.12f})", flush=True)
    assert abs(fid - float(gd["brick_fid_exact"])) < 1e-6


def test_capacity_1024_gram_side_above_1024_block_jacobi():
    """A two-site block whose both sides exceed 1024 (2 chi_l = 2 chi_r = 1040 at capacity 1024): the
    Gram path declines it (C > 1024) and the block Jacobi (16-column blocks of 2048 rows) factors it;
    max_chi = 1024 truncates.  Against the oracle's goldens (tests/golden/make_cap1024_golden.py):
    exact bond dimensions, the new bond's Schmidt values within 1e-9, four product-state overlaps
    within 1e-10."""
    import time

    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    gd = _golden_cap1024()
    n, chi = 22, 520
    t0 = time.perf_counter()
    with _blas_threads():  # (the chi = 520 canonical form: ~10 s on 8 threads)
        aer = random_vidal_mps(n, chi, 8)
    print(f"input state: {time.perf_counter() - t0:.1f} s", flush=True)
    rng = np.random.default_rng(8)
    ops = []
    for q in (10, 11):
        ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
        ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
    ops.append(("cx", (10, 11), ()))
    d = DeviceMPS(n, 1024, 1e-16, 1024)
    d.load_aer(aer)
    t0 = time.perf_counter()
    d.apply(device_ops(to_circuit(n, ops)))
    np.testing.assert_array_equal(d.dims(), gd["bj_dims"])
    print(f"1040 x 1040 update (block Jacobi): {time.perf_counter() - t0:.2f} s", flush=True)
    gam, lam = d.to_aer()
    np.testing.assert_allclose(lam[10], gd["bj_lam10"], atol=1e-9)
    np.testing.assert_allclose(_product_overlaps(d, gd["bj_phi"]), gd["bj_phi_ov"], atol=1e-10)
