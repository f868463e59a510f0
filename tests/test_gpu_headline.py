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


@pytest.mark.parametrize("kind", ["near-product", "random"])
def test_bench_overlap_workload_fused_chain_vs_oracle(kind):
    """10 states x 4 distances = 40 evaluations in one apply + sort batch (k_chain); one
    evaluation per distance, each from a different source state, against the oracle replay:
    exact bond dimensions and overlap within 1e-6 (truncated-MPS tolerance of BASELINE.json)."""
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
    copy_batch(work, [src[k // 4] for k in range(len(work))])
    # the random-state case runs the bench's pipelined form: queued apply, read-back, deferred check
    pipelined = kind == "random"
    apply_batch(work, ops, sort=True, wait=not pipelined)
    ov = overlap_zero_batch(work)
    if pipelined:
        check_batch(work)
    checked = 0
    for i, d in enumerate(bench.DISTANCES):
        k = 4 * i + i  # state i (source i % 4), distance d
        st = M.MPS.from_aer(distinct[i % len(distinct)])
        ref = M.run_circuit(n, bench.thin_layer_oracle_ops(bench.LAYER_A, bench.LAYER_A + d, angles[k]), 1e-16, chi,
                            mps=st)
        pre = ref.preprocessed()
        np.testing.assert_array_equal(work[k].dims(), [1] + [x.shape[2] for x in pre])
        ov_ref = M.mps_dot(pre, M.zero_mps(n))
        assert abs(ov[k] - ov_ref) <= 1e-6, (d, ov[k], ov_ref)
        if kind == "near-product":
            assert abs(ov_ref) > 1e-3  # a checkable (non-trivial) overlap
        checked += 1
    assert checked == 4


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
