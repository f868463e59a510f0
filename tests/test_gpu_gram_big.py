"""Multi-workgroup Gram-path SVD for 2 chi > 128 (gram_big.hip) against the oracle and against the
block Jacobi it replaces.

The tridiagonalisation spreads each job's G over several workgroups that exchange one vector per
column through global memory; these tests check the decompositions it feeds into the two-site
update (bond dims exact, Schmidt values 1e-9, fidelity 1e-6 -- BASELINE.json's truncated-MPS bar),
that the path was actually taken (its counters), that the block Jacobi (the Gram path switched
off) gives the same state, and that a rank-deficient theta declines to the block Jacobi.
"""
import numpy as np
import pytest

from bench import random_vidal_mps  # noqa: E402
from conftest import to_circuit
from oracle import mps as M

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[1, 0], ids=["tail", "exchange_to_end"])
def gb_tail(request):
    """The last 128 columns of the tridiagonalisation in one workgroup (k_gb_tail, the default) or
    over all of the job's workgroups with the per-column exchange to the end."""
    from adaptaqc_amd import _lib

    _lib.check(_lib.load().aqc_gb_set_tail(request.param))
    try:
        yield request.param
    finally:
        _lib.check(_lib.load().aqc_gb_set_tail(1))


def _gates(n, rng, pairs):
    ops = []
    for a, b in pairs:
        for q in (a, b):
            ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
            ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
        ops.append(("cx", (a, b), ()))
    return ops


def _run(n, chi, ops, seed, gram=1):
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    _lib.check(_lib.load().aqc_mps_set_svd_path(gram, 64))
    try:
        _lib.gram_big_stats()
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.load_aer(random_vidal_mps(n, chi, seed))
        d.apply(device_ops(to_circuit(n, ops)))
        stats = _lib.gram_big_stats()
    finally:
        _lib.check(_lib.load().aqc_mps_set_svd_path(1, 64))
    return d, stats


def _vs_oracle(d, n, chi, ops, seed):
    ref = M.run_circuit(n, ops, 1e-16, chi, mps=M.MPS.from_aer(random_vidal_mps(n, chi, seed)))
    pre_ref = ref.preprocessed()
    np.testing.assert_array_equal(d.dims(), [1] + [x.shape[2] for x in pre_ref])
    pre = d.preprocessed()
    fid = abs(M.mps_dot(pre_ref, pre)) / np.sqrt(abs(M.mps_dot(pre, pre)) * abs(M.mps_dot(pre_ref, pre_ref)))
    assert abs(fid - 1.0) < 1e-6, fid
    return ref


@pytest.mark.parametrize("n,chi", [(18, 128), (20, 256)])
def test_gram_big_taken_and_matches_oracle(n, chi, gb_tail):
    """Adjacent truncating updates at the cap (2 chi = 256 / 512): every one takes the Gram path
    (no floor declines, no exchange timeouts) and the state matches the oracle."""
    rng = np.random.default_rng(chi + 3)
    m = n // 2
    ops = _gates(n, rng, [(m - 1, m), (m, m + 1), (m - 2, m - 1)])
    d, st = _run(n, chi, ops, seed=chi + 4)
    assert st["calls"] == 3 and st["taken"] == 3 and st["timeouts"] == 0, st
    ref = _vs_oracle(d, n, chi, ops, chi + 4)
    _, lam = d.to_aer()
    for b in (m - 1, m, m + 1):
        np.testing.assert_allclose(lam[b - 1], ref.l[b - 1], atol=1e-9, err_msg=f"bond {b}")


def test_gram_big_equals_block_jacobi():
    """One wave of 8 disjoint updates at 2 chi = 512 (config 5's state) through the Gram path and
    through the block Jacobi (Gram path off): same bond dimensions, Schmidt values within 1e-9,
    states within 1e-6."""
    n, chi = 100, 256
    rng = np.random.default_rng(11)
    ops = _gates(n, rng, [(a, a + 1) for a in range(40, 56, 2)])
    g, st = _run(n, chi, ops, seed=5, gram=1)
    assert st["taken"] == 8, st
    b, st0 = _run(n, chi, ops, seed=5, gram=0)
    assert st0["taken"] == 0, st0
    np.testing.assert_array_equal(g.dims(), b.dims())
    _, lg = g.to_aer()
    _, lb = b.to_aer()
    for x, y in zip(lg, lb):
        np.testing.assert_allclose(x, y, atol=1e-9)
    pg, pb = g.preprocessed(), b.preprocessed()
    assert abs(abs(M.mps_dot(pg, pb)) / np.sqrt(abs(M.mps_dot(pg, pg)) * abs(M.mps_dot(pb, pb))) - 1.0) < 1e-6


def test_gram_big_rank_deficient_certified():
    """A 2 chi = 256 update whose middle bond keeps only 4 non-zero Schmidt values (the rest set to
    zero): theta' has rank <= 16 and the eigenvalues past it sit at the noise floor, inside CHOP's
    error band.  The kept count assumes them chopped and k_gb_cert proves it (||X - X V V^H||_F^2 <
    CHOP / 2), so the Gram path keeps the update (round 4 declined it to the block Jacobi, which the
    exchange-timeout test below still covers); the result matches the oracle on the same input."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS

    n, chi = 16, 128
    gam, lam = random_vidal_mps(n, chi, 21)
    lam = [np.array(x, dtype=float) for x in lam]
    b = 7  # the bond between sites 7 and 8
    lam[b][4:] = 0.0
    lam[b] /= np.linalg.norm(lam[b])
    aer = (gam, lam)
    rng = np.random.default_rng(2)
    ops = _gates(n, rng, [(7, 8)])
    _lib.gram_big_stats()
    d = DeviceMPS(n, chi, 1e-16, None)
    d.load_aer(aer)
    d.apply(device_ops(to_circuit(n, ops)))
    st = _lib.gram_big_stats()
    assert st["taken"] == 1 and st["certificates"] == 1 and st["certified"] == 1, st
    assert st["declined_floor"] == 0 and st["timeouts"] == 0, st
    ref = M.run_circuit(n, ops, 1e-16, None, mps=M.MPS.from_aer(aer))
    pre_ref = ref.preprocessed()
    np.testing.assert_array_equal(d.dims(), [1] + [x.shape[2] for x in pre_ref])
    pre = d.preprocessed()
    fid = abs(M.mps_dot(pre_ref, pre)) / np.sqrt(abs(M.mps_dot(pre, pre)) * abs(M.mps_dot(pre_ref, pre_ref)))
    assert abs(fid - 1.0) < 1e-6, fid


def test_gram_big_config5_wave(gb_tail):
    """Config 5's wave (100 qubits, chi = 256, 24 disjoint updates at the cap): all 24 on the Gram
    path in one call."""
    n, chi = 100, 256
    rng = np.random.default_rng(5)
    ops = _gates(n, rng, [(a, a + 1) for a in range(26, 74, 2)])
    d, st = _run(n, chi, ops, seed=5)
    assert st["taken"] == 24 and st["timeouts"] == 0, st
    _vs_oracle(d, n, chi, ops, 5)


def test_gram_big_exchange_timeout_declines_to_block_jacobi(gb_tail):
    """The counter-wait limit at 0 (aqc_gb_set_spin_limit): a workgroup that finds its job's count
    short at any column declines the job (status 3).  The declined jobs run the
    block Jacobi after the status read-back and the state still matches the oracle (exact bond dims,
    fidelity 1e-6)."""
    from adaptaqc_amd import _lib

    n, chi = 18, 128
    rng = np.random.default_rng(chi + 3)
    m = n // 2
    ops = _gates(n, rng, [(m - 1, m), (m, m + 1), (m - 2, m - 1)])
    _lib.check(_lib.load().aqc_gb_set_spin_limit(0.0))
    try:
        d, st = _run(n, chi, ops, seed=chi + 4)
    finally:
        _lib.check(_lib.load().aqc_gb_set_spin_limit(-1.0))
    assert st["calls"] == 3 and st["timeouts"] >= 1, st
    assert st["taken"] + st["timeouts"] == 3, st
    _vs_oracle(d, n, chi, ops, chi + 4)


def test_gram_big_late_workgroup_start(gb_tail):
    """the tridiagonalisation's workgroups of one job may start late (CUs held by
    other work).  A staggered CU-holding load on another stream (aqc_debug_hog: blocks release
    their CUs over 2 ... 30 ms) is queued first, so the jobs' workgroups are dispatched one CU at a
    time; reflector row 0 must not be overwritten before every workgroup has read it.  Same result
    as the oracle, no timeout (30 ms is well inside the 100 ms limit)."""
    from adaptaqc_amd import _lib

    n, chi = 20, 256
    rng = np.random.default_rng(chi + 3)
    m = n // 2
    ops = _gates(n, rng, [(m - 1, m), (m, m + 1), (m - 2, m - 1)])
    lib = _lib.lib()
    _lib.check(lib.aqc_debug_hog(2048, 30.0))
    d, st = _run(n, chi, ops, seed=chi + 4)
    assert st["calls"] == 3 and st["taken"] == 3 and st["timeouts"] == 0, st
    _vs_oracle(d, n, chi, ops, chi + 4)


def test_gram_big_two_stages_equal_one_stage():
    """Config 5's state, 16 disjoint updates at 2 chi = 512 (two rounds: a round's second stage
    beside the next round's first) with the exchange in two stages (16 then 4 workgroups per job)
    and in one: the same bond dimensions and Schmidt values within 1e-12 (the stages differ only in
    the lane grouping of the row sums)."""
    from adaptaqc_amd import _lib

    n, chi = 100, 256
    rng = np.random.default_rng(17)
    ops = _gates(n, rng, [(a, a + 1) for a in range(34, 66, 2)])
    res = []
    for stages in (2, 1):
        _lib.check(_lib.load().aqc_gb_set_stages(stages))
        try:
            d, st = _run(n, chi, ops, seed=6)
        finally:
            _lib.check(_lib.load().aqc_gb_set_stages(2))
        assert st["taken"] == 16 and st["timeouts"] == 0, st
        res.append(d)
    np.testing.assert_array_equal(res[0].dims(), res[1].dims())
    _, l0 = res[0].to_aer()
    _, l1 = res[1].to_aer()
    for x, y in zip(l0, l1):
        np.testing.assert_allclose(x, y, atol=1e-12)


def test_gram_big_tail_equals_exchange_to_end():
    """Config 5's state, 8 disjoint updates at 2 chi = 512 with the single-workgroup tail and with
    the exchange to the end: the same arithmetic on the same data, so the same bond dimensions and
    Schmidt values within 1e-12."""
    from adaptaqc_amd import _lib

    n, chi = 100, 256
    rng = np.random.default_rng(13)
    ops = _gates(n, rng, [(a, a + 1) for a in range(40, 56, 2)])
    res = []
    for tail in (1, 0):
        _lib.check(_lib.load().aqc_gb_set_tail(tail))
        try:
            d, st = _run(n, chi, ops, seed=6)
        finally:
            _lib.check(_lib.load().aqc_gb_set_tail(1))
        assert st["taken"] == 8, st
        res.append(d)
    np.testing.assert_array_equal(res[0].dims(), res[1].dims())
    _, l0 = res[0].to_aer()
    _, l1 = res[1].to_aer()
    for x, y in zip(l0, l1):
        np.testing.assert_allclose(x, y, atol=1e-12)
