"""The headline (bench.py, config 3) path itself against the oracle: the exact bench input --
50-qubit chi = 64 states, a thinly-dressed layer at pair distances 1, 2, 5, 25 replayed with Aer
swap routing and sorted back -- through the fused per-state chain (k_chain, >= 32 states), and
the 1225-pair chi = 64 gradient sweep on states whose gradients are far from zero."""
import numpy as np
import pytest

import bench
from oracle import adapt_host
from oracle import gradients as ogr
from oracle import mps as M

pytestmark = pytest.mark.gpu


def _gram_expectation(svd_logs, max_chi):
    """From the oracle's per-update singular values: (updates, must take the Gram path, must
    decline it).  The path runs when lambda_K > 1e-9 lambda_1 (lambda = s^2, K = min(C, max_chi));
    the device's eigenvalues carry eps ||G|| absolute error, so only decisions a decade clear of the
    floor are asserted."""
    calls = take = decline = 0
    for s in svd_logs:
        calls += 1
        k = min(len(s), max_chi)
        ratio = (s[k - 1] / s[0]) ** 2 if s[0] > 0 else 0.0
        if k <= 64 and ratio > 1e-8:
            take += 1
        elif k > 64 or ratio < 1e-10:
            decline += 1
    return calls, take, decline


@pytest.mark.parametrize("kind", ["near-product", "random"])
def test_bench_overlap_workload_fused_chain_vs_oracle(kind):
    """10 states x 4 distances = 40 evaluations in one apply + sort batch (k_chain), every one
    against the oracle replay: exact bond dimensions and overlap within 1e-6 (truncated-MPS
    tolerance of BASELINE.json).  The Gram-path counters (aqc_svd_gram_stats) must show every
    update going through the SVD, the Gram path taken wherever the oracle's spectrum puts lambda_K
    a decade above its 1e-9 lambda_1 floor and declined wherever it is a decade below."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceMPS, apply_batch, check_batch, copy_batch, overlap_zero_batch

    n, chi, B = bench.N_QUBITS, bench.CHI, 10
    distinct = bench.bench_states(n, chi, 4, kind)
    src = []
    for k in range(B):
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.load_aer(distinct[k % len(distinct)])
        src.append(d)
    rng = np.random.default_rng(17)
    angles = [rng.uniform(-np.pi, np.pi, 4) for _ in range(B * len(bench.DISTANCES))]
    ops = [_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + d, angles[s * 4 + i]))
           for s in range(B) for i, d in enumerate(bench.DISTANCES)]
    work = [DeviceMPS(n, chi, 1e-16, chi) for _ in ops]
    assert len(work) >= 32  # the fused per-state chain's batch size (kChainMinStates)
    copy_batch(work, [src[k // 4] for k in range(len(work))])
    # the random-state case runs the bench's pipelined form: queued apply, read-back, deferred check
    pipelined = kind == "random"
    _lib.gram_stats()  # reset
    apply_batch(work, ops, sort=True, wait=not pipelined)
    ov = overlap_zero_batch(work)
    if pipelined:
        check_batch(work)
    gram = _lib.gram_stats()
    logs = []
    nontrivial = 0
    for k in range(len(work)):
        s, i = divmod(k, len(bench.DISTANCES))
        d = bench.DISTANCES[i]
        st = M.MPS.from_aer(distinct[s % len(distinct)])
        st.svd_log = []
        ref = M.run_circuit(n, bench.thin_layer_oracle_ops(bench.LAYER_A, bench.LAYER_A + d, angles[k]), 1e-16, chi,
                            mps=st)
        logs += [sv for _, sv in st.svd_log]
        pre = ref.preprocessed()
        np.testing.assert_array_equal(work[k].dims(), [1] + [x.shape[2] for x in pre])
        ov_ref = M.mps_dot(pre, M.zero_mps(n))
        assert abs(ov[k] - ov_ref) <= 1e-6, (k, d, ov[k], ov_ref)
        nontrivial += abs(ov_ref) > 1e-3
    if kind == "near-product":
        assert nontrivial == len(work)  # checkable (non-trivial) overlaps
    calls, take, decline = _gram_expectation(logs, chi)
    assert gram["calls"] == calls, (gram, calls)
    assert take <= gram["taken"] <= calls - decline, (gram, take, decline)
    assert gram["declined_floor"] + gram["declined_shape"] + gram["taken"] == gram["calls"]
    assert take > 0


def _designed_pair_state(n, p, a_sv, b_sv, seed):
    """A 50-qubit Vidal MPS (random chi = 64 elsewhere) whose sites p, p+1 are rewritten so that
    a CX on (p, p+1) produces theta' = diag(A, B) block-diagonally (unit lambdas around and between
    the two sites, Gamma_{p+1} = [I, 0], Gamma_p = [A, B]); A and B are random-unitary conjugates of
    the given singular values.  Not canonical -- the device and the oracle run the same arithmetic
    on it, which is all the comparison needs."""
    rng = np.random.default_rng(seed)

    def haar(m):
        z = (rng.normal(size=(m, m)) + 1j * rng.normal(size=(m, m))) / np.sqrt(2)
        q, r = np.linalg.qr(z)
        return q * (np.diag(r) / np.abs(np.diag(r)))

    gam, lam = bench.random_vidal_mps(n, 64, 9000 + seed)
    gam, lam = list(gam), list(lam)
    A = haar(64) @ np.diag(a_sv) @ haar(64).conj().T
    Bm = haar(64) @ np.diag(b_sv) @ haar(64).conj().T
    gam[p] = (A, Bm)
    gam[p + 1] = (np.eye(64, dtype=complex), np.zeros((64, 64), complex))
    lam[p - 1] = np.ones(64)
    lam[p] = np.ones(64)
    lam[p + 1] = np.ones(64)
    return gam, lam


def test_k_chain_near_degenerate_cut_and_gram_decline_vs_oracle():
    """32 states through k_chain whose first update's theta' is built to stress the Gram path
    (SURVEY 7 hard part 2): 16 with a near-degenerate cut sigma_64 = sigma_65 (1 + delta), delta
    1e-4 ... 1e-8 (the Gram path is taken: its kept subspace carries eps sigma_1^2 / (sigma_64^2 -
    sigma_65^2) error), and 16 with lambda_64 < 1e-9 lambda_1 (the Gram path declines inside
    k_chain and the register Jacobi runs).  Each against the oracle (LAPACK SVD): exact bond dims,
    the truncated two-site block within 1e-6, and the state's fidelity with the oracle's within
    1e-6."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd import gates as Gd
    from adaptaqc_amd.device import DeviceMPS, apply_batch

    n, p = bench.N_QUBITS, 24
    lin = np.linspace(1.0, 0.5, 65)
    states, kinds = [], []
    for s in range(16):
        delta = [1e-4, 1e-6, 1e-7, 1e-8][s % 4]
        a = lin[:64]
        b = lin[1:65] * (1 + delta)  # b_j = a_{j+1} (1 + delta): sigma_64 = a_33 (1 + delta), sigma_65 = a_33
        states.append(_designed_pair_state(n, p, a, b, s))
        kinds.append(("cut", delta))
    r = 0.6
    for s in range(16):
        merged = np.sqrt(r ** np.arange(1, 129))  # s_i^2 ~ r^i: lambda_64 / lambda_1 = r^63 ~ 1e-14
        states.append(_designed_pair_state(n, p, merged[0::2], merged[1::2], 100 + s))
        kinds.append(("decline", r))
    # the designs hold on the oracle's theta'
    cx = ("cx", (p, p + 1), ())
    for (kind, par), aer in zip(kinds, states):
        st = M.MPS.from_aer(aer)
        sv = np.linalg.svd(st.theta_matrix(p, M.G.matrix("cx", ()).reshape(2, 2, 2, 2).transpose(1, 0, 3, 2)),
                           compute_uv=False)
        if kind == "cut":
            assert abs(sv[63] / sv[64] - 1 - par) < 1e-2 * par + 1e-12
        else:
            assert (sv[63] / sv[0]) ** 2 < 1e-12
    dev = []
    for aer in states:
        d = DeviceMPS(n, 64, 1e-16, 64)
        d.load_aer(aer)
        dev.append(d)
    ops = [_lib.ops_array([(Gd.TWO_QUBIT["cx"], (p, p + 1))]) for _ in dev]
    _lib.gram_stats()
    apply_batch(dev, ops, sort=True)
    gram = _lib.gram_stats()
    assert gram["calls"] == 32 and gram["taken"] == 16 and gram["declined_floor"] == 16, gram
    for k, ((kind, par), aer) in enumerate(zip(kinds, states)):
        st = M.MPS.from_aer(aer)
        ref = M.run_circuit(n, [cx], 1e-16, 64, mps=st)
        got = M.MPS.from_aer(dev[k].to_aer())
        assert [x.shape[2] for x in got.g[:-1]] == [x.shape[2] for x in ref.g[:-1]], kind
        t_ref, t_got = ref.theta_matrix(p), got.theta_matrix(p)
        assert np.max(np.abs(t_got - t_ref)) < 1e-6, (kind, par, np.max(np.abs(t_got - t_ref)))
        pr, pg = ref.preprocessed(), got.preprocessed()
        fid = M.mps_dot(pr, pg) / M.mps_dot(pr, pr)
        assert abs(fid - 1) < 1e-6, (kind, par, fid)


def test_bench_gradients_chi64_nontrivial_vs_oracle():
    """1225-pair identity_resolvable sweep (rotoselect generators, |s> = |0..0>) on two bench
    states at chi = 64: all pairs against the oracle's environment form, 6 pairs against the
    reference structure (per-pair, per-generator MPS build + dot), and the arg-max pair."""
    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch

    n, chi = bench.N_QUBITS, bench.CHI
    cmap = adapt_host.coupling_map_full(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    _, og, od, inv0 = bench.oracle_layer()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    qs = bench.bench_states(n, chi, 2)
    ds = []
    for q in qs:
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.load_aer(q)
        assert d.dims().max() == chi
        ds.append(d)
    got = pair_grads_batch(ds, svec, cmap, u0, gm, deg)
    for s, q in enumerate(qs):
        psi = M.MPS.from_aer(q).preprocessed()
        want = np.array(ogr.general_grad_of_pairs_env(psi, n, inv0, og, od, cmap))
        assert np.max(want) > 1e-2
        np.testing.assert_allclose(got[s], want, rtol=0, atol=1e-10)
        idx = np.random.default_rng(s).choice(len(cmap), 6, replace=False)
        ref = ogr.general_grad_of_pairs_ref(psi, n, inv0, og, od, [cmap[i] for i in idx], (), 1e-16, chi)
        np.testing.assert_allclose(got[s][idx], ref, rtol=0, atol=1e-10)
        assert int(np.argmax(got[s])) == int(np.argmax(want))
