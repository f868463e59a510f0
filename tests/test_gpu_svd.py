"""The two-site SVD kernel on its own (aqc_svd_debug) against LAPACK / scipy on the same theta.

Shapes follow the two-site update: theta is (2 chi_l) x (2 chi_r), column-major.  The QR phase is
pinned to scipy's pivoted QR (zgeqp3: same reflector convention, pivot = largest trailing norm),
the decomposition to numpy's SVD; tolerances are relative to sigma_max.

Contract (k_jacobi_reg): singular values above the noise floor (1e-11 sigma_max) to
1e-13 sigma_max absolute; columns whose squared norm falls below 1e-24 ||W||^2 are frozen, so
values under the floor are only bounded by it -- the two-site update discards every
sigma < 1e-8 (CHOP, s^2 < 1e-16) anyway.  Singular vectors are checked where sigma > 1e-8.
"""
import ctypes

import numpy as np
import pytest
import scipy.linalg as sla

pytestmark = pytest.mark.gpu

SHAPES = [(4, 4), (2, 8), (16, 8), (32, 32), (24, 64), (64, 64), (128, 64), (64, 128), (128, 128)]


def _theta(m, n, seed, rank=None):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((m, n)) + 1j * rng.standard_normal((m, n))
    a *= (0.8 ** np.arange(n))[None, :]  # graded columns, like lambda-weighted thetas
    if rank is not None:
        u, s, vh = np.linalg.svd(a, full_matrices=False)
        s[rank:] = 0.0
        a = (u * s) @ vh
    return a / np.linalg.norm(a)


def _check_sigma(sig, s_ref):
    sig = np.sort(sig)[::-1]
    live = s_ref > 1e-11 * s_ref[0]
    np.testing.assert_allclose(sig[live], s_ref[live], atol=1e-13 * s_ref[0])
    assert np.all(sig[~live] <= 2e-11 * s_ref[0])


def _run(theta, variant, stop_after_qr=False):
    from adaptaqc_amd import _lib

    m, n = theta.shape
    c, l = min(m, n), max(m, n)
    lw = c
    th = np.asfortranarray(theta.astype(np.complex128)).ravel(order="F").copy()
    w = np.zeros(c * lw, np.complex128)
    sig = np.zeros(c)
    perm = np.zeros(c, np.int32)
    sw = ctypes.c_int()
    _lib.check(_lib.lib().aqc_svd_debug(th.ctypes.data, m, n, variant, int(stop_after_qr), w.ctypes.data,
                                        sig.ctypes.data, perm.ctypes.data, ctypes.byref(sw)))
    return w.reshape(c, lw).T, sig, perm, sw.value  # columns of W as columns


@pytest.mark.parametrize("m,n", SHAPES)
def test_jacobi_singular_values(m, n):
    th = _theta(m, n, m * 1000 + n)
    s_ref = np.linalg.svd(th, compute_uv=False)
    for variant in (2,):
        w, sig, _, sweeps = _run(th, variant)
        _check_sigma(sig, s_ref)
        assert sweeps < 40


@pytest.mark.parametrize("m,n", SHAPES)
def test_qr_phase_matches_scipy(m, n):
    th = _theta(m, n, m * 7 + n)
    w_in = th.conj().T if m < n else th
    q, r, p = sla.qr(w_in, pivoting=True, mode="economic")
    for variant in (2,):
        x, _, perm, _ = _run(th, variant, stop_after_qr=True)
        np.testing.assert_array_equal(perm, p)
        np.testing.assert_allclose(x, r.conj().T, atol=1e-13)


@pytest.mark.parametrize("m,n", SHAPES)
def test_qr_jacobi_vectors(m, n):
    """With QR the output columns are the other side's singular vectors times sigma."""
    th = _theta(m, n, m * 31 + n)
    u, s, vh = np.linalg.svd(th, full_matrices=False)
    k = int(np.sum(s > 1e-8 * s[0]))
    for variant in (2,):
        w, sig, _, _ = _run(th, variant)
        order = np.argsort(-sig, kind="stable")
        w, sig = w[:, order], sig[order]
        if m >= n:  # W = theta: output = V sigma, so theta (W / sigma^2) = U
            vcols = w[:, :k] / sig[:k]
            np.testing.assert_allclose(np.abs(vcols.conj().T @ vh[:k].conj().T), np.eye(k), atol=1e-10)
        else:       # W = theta^H: output = U sigma
            ucols = w[:, :k] / sig[:k]
            np.testing.assert_allclose(np.abs(ucols.conj().T @ u[:, :k]), np.eye(k), atol=1e-10)


def test_rank_deficient_and_zero_columns():
    for rank in (1, 3, 17):
        th = _theta(64, 64, rank, rank=rank)
        s_ref = np.linalg.svd(th, compute_uv=False)
        for variant in (2,):
            _, sig, _, _ = _run(th, variant)
            _check_sigma(sig, s_ref)


# ---- the Gram / tridiagonal fast path (aqc_svd_debug variant 7, svd_gram.h) -------------------
def _gram_ticks():
    """Phase ticks accumulated since the last call (the call resets them)."""
    from adaptaqc_amd import _lib

    t = np.zeros(12)
    _lib.check(_lib.lib().aqc_svd_gram_ticks(_lib.ptr(t)))
    return t


def _spectrum_theta(m, n, s, seed):
    rng = np.random.default_rng(seed)
    c = min(m, n)
    u, _ = np.linalg.qr(rng.standard_normal((m, c)) + 1j * rng.standard_normal((m, c)))
    v, _ = np.linalg.qr(rng.standard_normal((n, c)) + 1j * rng.standard_normal((n, c)))
    return (u * s[None, :]) @ v.conj().T


@pytest.mark.parametrize("m,n", [(128, 128), (128, 96), (96, 128), (128, 72), (80, 80)])
def test_gram_path_vs_numpy(m, n):
    """Spectrum decaying as 0.93^i (lambda_64 / lambda_1 ~ 1e-4 > 1e-9): the Gram path runs to the
    end (its back-transformation ticks advance) and returns the top K = 64 triplets: sigma to
    1e-12 sigma_1, the kept right subspace of X (theta or theta^H, L >= C) to 1e-10, W = V Sigma."""
    c = min(m, n)
    theta = _spectrum_theta(m, n, 0.93 ** np.arange(c), 7 + m + n)
    _gram_ticks()
    w, sig, _, _ = _run(theta, 7)
    assert _gram_ticks()[4] > 0, "the Gram path declined"
    K = min(64, c)
    x = theta if m >= n else theta.conj().T
    _, s_ref, vh = np.linalg.svd(x)
    order = np.argsort(-sig)
    got = sig[order]
    np.testing.assert_allclose(got[:K], s_ref[:K], rtol=0, atol=1e-12 * s_ref[0])
    assert np.all(got[K:] == 0.0)
    V = w[:, order[:K]] / got[None, :K]
    Vr = vh[:K].conj().T
    assert np.linalg.norm(V @ V.conj().T - Vr @ Vr.conj().T, 2) < 1e-10
    assert np.max(np.abs(V.conj().T @ V - np.eye(K))) < 1e-11


@pytest.mark.parametrize("m,n,decay", [(128, 128, 0.97), (128, 96, 0.97), (96, 128, 0.95), (128, 80, 0.98)])
def test_gram_path_wide_k_vs_numpy(m, n, decay):
    """max_chi unbounded (debug max_chi 0) and no tail threshold: every value above the CHOP is kept,
    K = C > 64 -- the wide S5 (waves 0-1, pivots in the work scratch) and S6 in two passes.  Sigma
    to 1e-12 sigma_1, each W column an eigenvector of X^H X (residual 1e-11 sigma_1^2), V unitary."""
    from adaptaqc_amd import _lib

    c = min(m, n)
    theta = _spectrum_theta(m, n, decay ** np.arange(c), 3 + m + n)
    L = _lib.lib()
    _lib.check(L.aqc_mps_set_svd_path(1, 0))
    try:
        _gram_ticks()
        w, sig, _, _ = _run(theta, 7)
        assert _gram_ticks()[4] > 0, "the Gram path declined"
    finally:
        _lib.check(L.aqc_mps_set_svd_path(1, 64))
    x = theta if m >= n else theta.conj().T
    s_ref = np.linalg.svd(x, compute_uv=False)
    order = np.argsort(-sig)
    got = sig[order]
    np.testing.assert_allclose(got, s_ref, rtol=0, atol=1e-12 * s_ref[0])
    V = w[:, order] / got[None, :]
    G = x.conj().T @ x
    res = np.linalg.norm(G @ V - V * got[None, :] ** 2, axis=0)
    assert res.max() < 1e-11 * s_ref[0] ** 2, res.max()
    assert np.max(np.abs(V.conj().T @ V - np.eye(c))) < 1e-11


@pytest.mark.parametrize("kind", ["graded", "rank10", "zero_tail_cluster"])
def test_gram_path_declines_to_jacobi(kind):
    """Where kept values reach the noise floor of the Gram form the path declines and the register
    Jacobi answers: graded (lambda_K <= 1e-9 lambda_1) at once; zero_tail_cluster (120 values of
    sigma^2 = 1e-12, inside the eigenvalue brackets' band around CHOP) after its certificate
    (||X - X V V^H||^2 < CHOP / 2) fails.  rank10 (118 exact zeros) passes the certificate and stays
    on the Gram path.  sigma as the Jacobi contract (_check_sigma) either way."""
    from adaptaqc_amd import _lib

    m = n = 128
    if kind == "graded":
        theta = _theta(m, n, 3)  # 0.8^i columns: sigma_64 / sigma_1 ~ 1e-6
    elif kind == "rank10":
        theta = _theta(m, n, 4, rank=10)
    else:
        s = np.concatenate([np.ones(8), 1e-6 * np.ones(120)])
        theta = _spectrum_theta(m, n, s, 5)
    _lib.gram_stats()
    w, sig, _, _ = _run(theta, 7)
    st = _lib.gram_stats()
    if kind == "rank10":
        assert st["taken"] == 1 and st["certificates"] == 1 and st["certified"] == 1, st
    else:
        assert st["taken"] == 0 and st["declined_floor"] == 1, st
        assert st["certificates"] == (1 if kind == "zero_tail_cluster" else 0) and st["certified"] == 0, st
    _check_sigma(sig, np.linalg.svd(theta, compute_uv=False))


@pytest.mark.parametrize("n", [32, 64, 128])
@pytest.mark.parametrize("kind", ["2x1+graded", "8x1+1e-3", "4x1+4x0.5+graded", "8x1+1e-6"])
def test_jacobi_degenerate_clusters(n, kind):
    """Exactly degenerate singular values (Bell-pair-like Schmidt spectra): every lane of a column
    group must agree on each rotation (lane-consistent 16-lane DPP sums, aqc_internal.h row_sum16);
    with the sums associated differently in alternate quads the near-degenerate pairs rotated in
    opposite senses on different rows and the clusters never converged (1e-8 .. 4e-6 errors)."""
    k = {"2x1+graded": 2, "8x1+1e-3": 8, "4x1+4x0.5+graded": 8, "8x1+1e-6": 8}[kind]
    if kind == "2x1+graded":
        s = np.concatenate([np.ones(2), 0.5 * 0.9 ** np.arange(n - 2)])
    elif kind == "8x1+1e-3":
        s = np.concatenate([np.ones(8), 1e-3 * np.ones(n - 8)])
    elif kind == "8x1+1e-6":
        s = np.concatenate([np.ones(8), 1e-6 * np.ones(n - 8)])
    else:
        s = np.concatenate([np.ones(4), 0.5 * np.ones(4), 0.2 * 0.9 ** np.arange(n - 8)])
    theta = _spectrum_theta(n, n, s, 5 + n)
    ref = np.linalg.svd(theta, compute_uv=False)
    for variant in (2,):
        _, sig, _, sweeps = _run(theta, variant)
        np.testing.assert_allclose(np.sort(sig)[::-1][:k], ref[:k], rtol=0, atol=1e-13)
        _check_sigma(sig, ref)
        assert sweeps < 40


