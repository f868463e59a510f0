"""Error flags of queued (async) applies surface through the cost read-backs: a capacity overflow
of an unbounded replay (aer_mps_backend.py:27-42's max_chi None) raises from
aqc_mps_overlap_zero_batch and aqc_mps_zero_hw1_batch without a separate aqc_mps_check_batch, and
the states are usable again afterwards (the flags were reset)."""
import numpy as np
import pytest

from adaptaqc_amd import _lib
from adaptaqc_amd.device import DeviceMPS, apply_batch, copy_batch, overlap_zero_batch, zero_hw1_batch

pytestmark = pytest.mark.gpu


def _entangling_ops(n, layers, seed):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(layers):
        for q in range(layer % 2, n - 1, 2):
            a = rng.standard_normal((4, 4)) + 1j * rng.standard_normal((4, 4))
            u, _ = np.linalg.qr(a)
            ops.append((u, (q, q + 1)))
    return _lib.ops_array(ops)


def test_overflow_raises_from_overlap_readback():
    n = 8
    states = [DeviceMPS(n, 2, 1e-16, None) for _ in range(3)]
    ops = _entangling_ops(n, 6, 1)
    apply_batch(states, [ops] * 3, sort=True, wait=False)
    with pytest.raises(_lib.AqcError, match="capacity"):
        overlap_zero_batch(states)
    # flags were reset: a fresh, harmless replay reads back cleanly
    for s in states:
        s.load_aer(([(np.array([[1.0 + 0j]]), np.array([[0.0 + 0j]]))] * n, [np.ones(1)] * (n - 1)))
    ov = overlap_zero_batch(states)
    np.testing.assert_allclose(np.abs(ov), 1.0, atol=1e-12)


def test_overflow_raises_from_window_readback():
    n = 8
    base = DeviceMPS(n, 2, 1e-16, None)
    cands = [DeviceMPS(n, 2, 1e-16, None) for _ in range(2)]
    copy_batch(cands, [base] * 2)
    ops = _entangling_ops(n, 6, 2)
    apply_batch(cands, [ops] * 2, sort=True, wait=False)
    with pytest.raises(_lib.AqcError, match="capacity"):
        zero_hw1_batch(base, cands)
