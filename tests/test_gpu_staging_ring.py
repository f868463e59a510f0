"""The pinned staging ring under calls of growing and alternating sizes (mps.hip StagingLease):
queued (async) applies whose job arrays outgrow the ring's sets between small calls -- a set that
grows brings the whole ring to its size while the other sets' earlier uploads may still be read --
give the same overlaps as the same replays run one state at a time and waited for."""
import numpy as np
import pytest

from adaptaqc_amd import _lib
from adaptaqc_amd.device import DeviceMPS, apply_batch, copy_batch, overlap_zero_batch

pytestmark = pytest.mark.gpu


def _ops(n, layers, seed):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(layers):
        for q in range(layer % 2, n - 1, 2):
            a = rng.standard_normal((4, 4)) + 1j * rng.standard_normal((4, 4))
            u, _ = np.linalg.qr(a)
            ops.append((u, (q, q + 1)))
    return _lib.ops_array(ops)


def _one_at_a_time(n, ops_list):
    out = []
    for ops in ops_list:
        s = DeviceMPS(n, 64, 1e-16, 64)
        apply_batch([s], [ops], sort=True)
        out.append(overlap_zero_batch([s])[0])
    return np.array(out)


def test_ring_growth_between_queued_calls():
    n = 10
    small = [_ops(n, 1, 100 + i) for i in range(2)]          # a few jobs
    large = [_ops(n, 12, 200 + i) for i in range(40)]        # >= 32 states: the chain path, many jobs
    larger = [_ops(n, 24, 300 + i) for i in range(48)]
    want_small, want_large, want_larger = (_one_at_a_time(n, x) for x in (small, large, larger))

    for rep in range(3):  # every set of the ring meets every size at least once
        ss = [DeviceMPS(n, 64, 1e-16, 64) for _ in small]
        sl = [DeviceMPS(n, 64, 1e-16, 64) for _ in large]
        sx = [DeviceMPS(n, 64, 1e-16, 64) for _ in larger]
        zero = DeviceMPS(n, 64, 1e-16, 64)
        copy_batch(ss, [zero] * len(ss))
        apply_batch(ss, small, sort=True, wait=False)
        apply_batch(sl, large, sort=True, wait=False)
        copy_batch(sx, [zero] * len(sx))
        apply_batch(sx, larger, sort=True, wait=False)
        got_small = overlap_zero_batch(ss)
        got_large = overlap_zero_batch(sl)
        got_larger = overlap_zero_batch(sx)
        np.testing.assert_allclose(got_small, want_small, atol=1e-10, rtol=0)
        np.testing.assert_allclose(got_large, want_large, atol=1e-10, rtol=0)
        np.testing.assert_allclose(got_larger, want_larger, atol=1e-10, rtol=0)
