"""Batched reload of cached MPS (aqc_mps_copy_batch): after a first full copy, a reload from the
same unchanged source rewrites only the Gamma sites changed since.  Every case must leave the
destination equal to the source exactly (as a full copy would), whatever happened in between:
updates on the destination, on the source, a different source, set_vidal, single copies."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, CHI = 20, 32


def _state(seed):
    import bench
    from adaptaqc_amd.device import DeviceMPS

    d = DeviceMPS(N, CHI, 1e-16, CHI)
    d.load_aer(bench.near_product_mps(N, CHI, seed))
    return d


def _layer(a, b, seed):
    import bench

    ang = np.random.default_rng(seed).uniform(-np.pi, np.pi, 4)
    return bench.thin_layer_ops(a, b, ang)


def _same(x, y):
    gx, lx = x.to_aer()
    gy, ly = y.to_aer()
    assert np.array_equal(x.dims(), y.dims())
    for (a0, a1), (b0, b1) in zip(gx, gy):
        assert np.array_equal(a0, b0) and np.array_equal(a1, b1)
    for a, b in zip(lx, ly):
        assert np.array_equal(a, b)


def test_partial_reload_matches_source():
    from adaptaqc_amd.device import apply_batch, copy_batch

    src = [_state(1), _state(2)]
    dst = [_state(9), _state(9)]
    copy_batch(dst, src)  # first copy: full
    for x, y in zip(dst, src):
        _same(x, y)
    for rnd in range(3):
        # updates on the copies (one far range with swap routing, one short), sorted back
        apply_batch(dst, [_layer(3, 11 + rnd, 10 + rnd), _layer(15, 16, 20 + rnd)], sort=True)
        copy_batch(dst, src)  # partial reload
        for x, y in zip(dst, src):
            _same(x, y)
    # nothing changed since the last reload: nothing to copy, still equal
    copy_batch(dst, src)
    for x, y in zip(dst, src):
        _same(x, y)


def test_reload_after_source_or_destination_changes():
    from adaptaqc_amd.device import apply_batch, copy_batch

    a, b = _state(3), _state(4)
    d = _state(5)
    copy_batch([d], [a])
    apply_batch([d], [_layer(2, 4, 1)], sort=True)
    # the source changes: the next reload must copy everything it changed
    apply_batch([a], [_layer(12, 17, 2)], sort=True)
    copy_batch([d], [a])
    _same(d, a)
    # a different source
    apply_batch([d], [_layer(6, 7, 3)], sort=True)
    copy_batch([d], [b])
    _same(d, b)
    # set_vidal on the destination, then a reload from the same source
    import bench

    d.load_aer(bench.near_product_mps(N, CHI, 77))
    copy_batch([d], [b])
    _same(d, b)
    # a single copy from another handle in between
    d.copy_from(a)
    _same(d, a)
    apply_batch([d], [_layer(0, 1, 4)], sort=True)
    copy_batch([d], [b])
    _same(d, b)
    # unsorted destination (updates without the sort): the reload restores order and sites
    apply_batch([d], [_layer(1, 18, 5)], sort=False)
    copy_batch([d], [b])
    _same(d, b)
