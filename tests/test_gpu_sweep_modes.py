"""Sweep chain kernels (aqc_sweep_set_chain_mode): first qubits grouped 8 to a workgroup on the
matrix cores vs one chain per workgroup, on batches of near-product states (non-trivial
gradients), at exact (64, 128) and inexact (100) bond capacities, full and sharded pair sets, and
the grouped batch against the oracle's environment form."""
import ctypes

import numpy as np
import pytest

from oracle import adapt_host
from oracle import gradients as ogr
from oracle import mps as M

pytestmark = pytest.mark.gpu


def _mode(m):
    from adaptaqc_amd import _lib

    _lib.check(_lib.lib().aqc_sweep_set_chain_mode(ctypes.c_int(m)))


def _states(n, chi, cap, seeds):
    import bench
    from adaptaqc_amd.device import DeviceMPS

    out = []
    for s in seeds:
        d = DeviceMPS(n, cap, 1e-16, cap)
        d.load_aer(bench.near_product_mps(n, chi, s))
        out.append(d)
    return out


@pytest.mark.parametrize("chi,cap", [(128, 128), (64, 64), (100, 100)])
def test_grouped_equals_per_chain(chi, cap):
    import bench
    from adaptaqc_amd.device import pair_grads_batch
    from adaptaqc_amd.sharding import PairShard

    n = 50
    cmap = adapt_host.coupling_map_full(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    st = _states(n, chi, cap, [11, 12, 13])
    try:
        _mode(1)
        ref = pair_grads_batch(st, svec, cmap, u0, gm, deg)
        _mode(2)
        got = pair_grads_batch(st, svec, cmap, u0, gm, deg)
        assert np.max(ref) > 1e-3
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.max(ref))
        # a rank's shard: groups of fewer than 8 first qubits, non-contiguous first qubits
        for world, r in ((3, 1), (8, 0), (8, 7)):
            sh = PairShard(cmap, n, r, world)
            part = pair_grads_batch(st, svec, sh.local_pairs, u0, gm, deg)
            np.testing.assert_allclose(part, ref[:, sh.local_index], rtol=0, atol=1e-12 * np.max(ref))
    finally:
        _mode(0)


def test_grouped_batch_vs_oracle_chi128():
    """Config 4 shape through the automatic (grouped) kernel: 2 states, 1225 pairs, vs oracle."""
    import bench
    from adaptaqc_amd.device import pair_grads_batch
    from adaptaqc_amd.utils import ansatzes

    n, chi = 50, 128
    cmap = adapt_host.coupling_map_full(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    seeds = [21, 22]
    st = _states(n, chi, chi, seeds)
    got = pair_grads_batch(st, svec, cmap, u0, gm, deg)
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in ansatzes.identity_resolvable().data]
    o_gens, o_deg = ogr.get_generators_and_degeneracies(o_layer, True, True)
    psi = M.MPS.from_aer(bench.near_product_mps(n, chi, seeds[1])).preprocessed()
    ref = ogr.general_grad_of_pairs_env(psi, n, ogr.inverse_ops(o_layer), o_gens, o_deg, cmap)
    assert np.max(ref) > 1e-3
    np.testing.assert_allclose(got[1], ref, atol=1e-10)


@pytest.mark.parametrize("n,chi,cap", [(50, 128, 128), (50, 64, 64), (50, 100, 100), (23, 16, 16), (7, 4, 8)])
def test_segmented_single_sweep_equals_chain_form(n, chi, cap):
    """The segmented single-state sweep (aqc_sweep_set_chain_mode 3, sweep_seg.h: prefix / suffix
    products inside sqrt(n) segments, boundary environments, batched GEMM hops) gives the chain
    form's gradients on full and sharded pair sets -- with the pair ends in either order -- and the
    same arg-max; at 50 qubits chi = 128 also against the oracle's environment form."""
    import bench
    from adaptaqc_amd.device import pair_grads_batch
    from adaptaqc_amd.sharding import PairShard
    from adaptaqc_amd.utils import ansatzes

    cmap = adapt_host.coupling_map_full(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    st = _states(n, chi, cap, [31])
    try:
        _mode(1)
        ref = pair_grads_batch(st, svec, cmap, u0, gm, deg)
        _mode(3)
        got = pair_grads_batch(st, svec, cmap, u0, gm, deg)
        assert np.max(ref) > 1e-4
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-11 * np.max(ref))
        assert int(np.argmax(got[0])) == int(np.argmax(ref[0]))
        for world, r in ((3, 1), (8, 7)):
            sh = PairShard(cmap, n, r, world)
            if not sh.local_pairs:
                continue
            part = pair_grads_batch(st, svec, sh.local_pairs, u0, gm, deg)
            np.testing.assert_allclose(part, ref[:, sh.local_index], rtol=0, atol=1e-11 * np.max(ref))
        flipped = [(b, a) for a, b in cmap[::7]]
        part = pair_grads_batch(st, svec, flipped, u0, gm, deg)
        _mode(1)
        part_ref = pair_grads_batch(st, svec, flipped, u0, gm, deg)
        np.testing.assert_allclose(part, part_ref, rtol=0, atol=1e-11 * np.max(ref))
    finally:
        _mode(0)
    if n == 50 and chi == 128:
        o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in ansatzes.identity_resolvable().data]
        o_gens, o_deg = ogr.get_generators_and_degeneracies(o_layer, True, True)
        psi = M.MPS.from_aer(bench.near_product_mps(n, chi, 31)).preprocessed()
        want = ogr.general_grad_of_pairs_env(psi, n, ogr.inverse_ops(o_layer), o_gens, o_deg, cmap)
        np.testing.assert_allclose(got[0], want, rtol=0, atol=1e-10)
