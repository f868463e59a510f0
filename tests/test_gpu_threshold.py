"""The truncation threshold of the reference's own MPS example (1e-8,
examples/advanced_mps_example.py:46; mps_sim_with_args, aer_mps_backend.py:27-42) on the device,
against the oracle (oracle/mps.py, reduce_zeros restated: CHOP, max_chi, tail sum below the
threshold): exact bond dimensions and the fidelity between the device and oracle states within
1e-6 (BASELINE.json's truncated-MPS bar), at max_chi = None and at a binding max_chi, through the
fused per-state chain (k_chain, >= 32 states), the lock-step path (one state at a time) and the
multi-workgroup path (2 chi = 256).

The states (bench.graded_vidal_mps) have geometrically decaying Schmidt spectra, so every
two-site update's singular values straddle the tail boundary: the kept count comes from the tail
rule (about 50 of 128 at decay 0.9), or from max_chi with the tail rule acting after it (decay
0.95).  Capacities are chosen so that the unbounded runs never need more than the capacity (the
oracle's kept counts for these seeds and layers stay at or below it)."""
import numpy as np
import pytest

import bench
from oracle import mps as M

pytestmark = pytest.mark.gpu
THR = 1e-8


def _layer(n, a, d, seed):
    rng = np.random.default_rng(seed)
    return bench.thin_layer_oracle_ops(a, a + d, rng.uniform(-np.pi, np.pi, 4))


def _oracle(n, aer, ops, max_chi):
    st = M.run_circuit(n, ops, THR, max_chi, mps=M.MPS.from_aer(aer))
    pre = st.preprocessed()
    return [1] + [x.shape[2] for x in pre], pre


def _check(dev, ref_dims, ref_pre, label):
    np.testing.assert_array_equal(dev.dims(), ref_dims, err_msg=label)
    pre = dev.preprocessed()
    nrm = abs(M.mps_dot(pre, pre))
    fid = abs(M.mps_dot(ref_pre, pre)) ** 2
    assert abs(nrm - 1.0) < 1e-10, (label, nrm)
    assert abs(fid - 1.0) < 1e-6, (label, fid)


def _run_batch(n, cap, max_chi, states, layers, batch):
    """states: Aer tuples; layers: (state index, oracle ops); batch: one apply_batch call (fused
    chain when >= 32 states at 2 chi = 128) or one state at a time (lock-step)."""
    from adaptaqc_amd import _lib
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceMPS, apply_batch
    from conftest import to_circuit

    work = []
    for si, _ in layers:
        d = DeviceMPS(n, cap, THR, max_chi)
        d.load_aer(states[si])
        work.append(d)
    ops = [_lib.ops_array(device_ops(to_circuit(n, o))) for _, o in layers]
    _lib.gram_stats()
    _lib.gram_big_stats()
    if batch:
        apply_batch(work, ops, sort=True)
    else:
        for d, o in zip(work, ops):
            d.apply(o)
            d.sort()
    stats = (_lib.gram_stats(), _lib.gram_big_stats())
    for k, (si, o) in enumerate(layers):
        ref_dims, ref_pre = _oracle(n, states[si], o, max_chi)
        _check(work[k], ref_dims, ref_pre, f"evaluation {k} (state {si})")
    return stats


@pytest.mark.parametrize("max_chi,decay,dists", [(None, 0.9, (1, 2, 3)), (64, 0.9, (1, 2, 3)),
                                                 (64, 0.95, (1, 2, 5, 25))],
                         ids=["unbounded", "maxchi64", "maxchi64-binding"])
def test_threshold_fused_chain_vs_oracle(max_chi, decay, dists):
    """>= 32 states in one batch: k_chain (capacity 64, 2 chi = 128) with the Gram path deciding the
    kept count by the tail rule (gram_keep) or the register Jacobi where it declines."""
    n, cap = 50, 64
    states = [bench.graded_vidal_mps(n, 64, 300 + s, decay) for s in range(4)]
    reps = -(-32 // (len(states) * len(dists)))
    layers = [(si, _layer(n, 20, d, 1000 * r + 10 * si + d)) for r in range(reps) for si in range(len(states))
              for d in dists]
    assert len(layers) >= 32
    gram, _ = _run_batch(n, cap, max_chi, states, layers, batch=True)
    assert gram["calls"] > 0
    # the tail rule keeps ~50 of 128 at decay 0.9: the Gram path must take most of those updates
    if decay == 0.9:
        assert gram["taken"] >= 0.5 * gram["calls"], gram


@pytest.mark.parametrize("max_chi", [None, 64])
def test_threshold_lockstep_single_states_vs_oracle(max_chi):
    """The same truncation one state at a time (the lock-step launches of a single evaluation)."""
    n, cap = 50, 64
    states = [bench.graded_vidal_mps(n, 64, 310 + s, 0.9) for s in range(2)]
    layers = [(si, _layer(n, 18, d, 77 + d)) for si in range(2) for d in (1, 3)]
    _run_batch(n, cap, max_chi, states, layers, batch=False)


@pytest.mark.parametrize("max_chi,decay,dists", [(None, 0.9, (1, 2)), (128, 0.95, (1, 3)), (None, 0.95, (2,))],
                         ids=["unbounded", "maxchi128", "unbounded-wide"])
def test_threshold_multi_workgroup_vs_oracle(max_chi, decay, dists):
    """2 chi = 256 two-site updates (capacity 128, 24 qubits at chi = 128): the multi-workgroup Gram
    path (gram_big.hip) or the block Jacobi where it declines, and the 2 chi = 128 path for the
    smaller thetas of the routed gates."""
    n, cap = 24, 128
    states = [bench.graded_vidal_mps(n, 128, 320 + s, decay) for s in range(2)]
    layers = [(si, _layer(n, 9, d, 55 + 10 * si + d)) for si in range(2) for d in dists]
    _, big = _run_batch(n, cap, max_chi, states, layers, batch=True)
    assert big["calls"] > 0


def _deficient_state(seed, tiny=None):
    """16 qubits with bonds ... 64 128 | 64 | 128 64 ...: the two-site block of sites (7, 8) is 256 x 256
    but has rank <= 2 x 64 after a CNOT -- 128 numerically zero singular values, which the Gram form
    cannot tell from 1e-16 (the CHOP).  tiny: the last 8 Schmidt values of the middle bond scaled
    by tiny (1e-4: sigma^2 from 7e-14 down to 8e-16 -- kept by the reference, inside the Gram form's
    noise band)."""
    rng = np.random.default_rng(seed)
    dims = [1, 2, 4, 8, 16, 32, 64, 128, 64, 128, 64, 32, 16, 8, 4, 2, 1]
    A = [rng.standard_normal((2, dims[i], dims[i + 1])) + 1j * rng.standard_normal((2, dims[i], dims[i + 1]))
         for i in range(16)]
    if tiny is not None:
        A[7][:, :, -8:] *= tiny
    return bench.vidal_from_tensors(A)


@pytest.mark.parametrize("tiny", [None, 1e-4], ids=["exact-zeros", "tiny-values"])
def test_rank_deficient_two_site_block_certificate(tiny):
    """The reference's default truncation (threshold 1e-16, max_chi None) on a 256 x 256 two-site
    block of rank 128: the multi-workgroup Gram path keeps the 128 values clear of the CHOP's band,
    assumes the other 128 chopped, and certifies it with ||X - X V V^H||_F^2 < CHOP / 2 computed from
    X (gram_big.hip k_gb_cert).  With true values of sigma^2 ~ 1e-14 among the dropped ones the
    certificate fails and the block Jacobi decides.  Exact bond dimensions and fidelity 1e-6 against
    the oracle either way."""
    n = 16
    aer = _deficient_state(41, tiny)
    rng = np.random.default_rng(5)
    ops = [("rz", (7,), (rng.uniform(-3, 3),)), ("rz", (8,), (rng.uniform(-3, 3),)), ("cx", (7, 8), ()),
           ("ry", (7,), (rng.uniform(-3, 3),)), ("ry", (8,), (rng.uniform(-3, 3),))]
    _, big = _run_batch_thr(n, 128, None, [aer], [(0, ops)], 1e-16)
    assert big["certificates"] >= 1, big
    if tiny is None:
        assert big["certified"] >= 1 and big["taken"] >= 1, big
    else:
        assert big["declined_certificate"] >= 1, big


def _deficient_state_128(seed, tiny):
    """14 qubits with bonds ... 32 64 | 32 | 64 32 ...: the two-site block of sites (6, 7) is 128 x 128
    (the 1024-thread Gram path) with rank <= 2 x 32 after a CNOT; tiny as in _deficient_state."""
    rng = np.random.default_rng(seed)
    dims = [1, 2, 4, 8, 16, 32, 64, 32, 64, 32, 16, 8, 4, 2, 1]
    A = [rng.standard_normal((2, dims[i], dims[i + 1])) + 1j * rng.standard_normal((2, dims[i], dims[i + 1]))
         for i in range(14)]
    if tiny is not None:
        A[6][:, :, -4:] *= tiny
    return bench.vidal_from_tensors(A)


@pytest.mark.parametrize("tiny", [None, 1e-4], ids=["exact-zeros", "tiny-values"])
def test_rank_deficient_two_site_block_certificate_128(tiny):
    """The same at 2 chi = 128 (gram_svd_body / gram_certified): 64 of the 128 values are exact zeros
    (or, with tiny, four of the kept ones sit inside the Gram form's noise band), the kept count
    assumes the open ones chopped and ||X - X V V^H||_F^2 < CHOP / 2 certifies it -- or fails, and the
    register Jacobi decides.  Exact bond dimensions and fidelity 1e-6 against the oracle."""
    n = 14
    aer = _deficient_state_128(43, tiny)
    rng = np.random.default_rng(6)
    ops = [("rz", (6,), (rng.uniform(-3, 3),)), ("rz", (7,), (rng.uniform(-3, 3),)), ("cx", (6, 7), ()),
           ("ry", (6,), (rng.uniform(-3, 3),)), ("ry", (7,), (rng.uniform(-3, 3),))]
    g, _ = _run_batch_thr(n, 64, None, [aer], [(0, ops)], 1e-16)
    assert g["certificates"] >= 1, g
    if tiny is None:
        assert g["certified"] >= 1 and g["taken"] >= 1, g
    else:
        assert g["certified"] < g["certificates"], g


def _run_batch_thr(n, cap, max_chi, states, layers, thr):
    global THR
    old, THR = THR, thr
    try:
        return _run_batch(n, cap, max_chi, states, layers, batch=False)
    finally:
        THR = old
