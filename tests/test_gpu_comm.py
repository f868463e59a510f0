"""libaqchip's RCCL exchange (aqc_comm_*, include/aqc_hip.h) on the GPU box: a one-rank
communicator (the box has one GPU; RCCL refuses two ranks on one device), the host and device
all-gathers, the max all-reduce, and the sharded candidate sweep's exchange through it against
the unsharded sweep.  Multi-rank behaviour of the same gather / arg-max logic is covered over gloo
(tests/test_distributed.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _hip():
    """The HIP runtime libaqchip itself links (device buffers for the device-pointer all-gather;
    torch is not used here: it would bring its own HIP runtime into the process)."""
    import ctypes

    for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    raise RuntimeError("libamdhip64.so not found")


def test_rccl_one_rank_collectives():
    import ctypes

    from adaptaqc_amd import _lib
    from adaptaqc_amd.comm import RcclComm

    uid = RcclComm.unique_id()
    comm = RcclComm(uid, 0, 1)
    x = np.arange(5, dtype=np.float64) * 1.5
    np.testing.assert_array_equal(comm.allgather(x), x[None, :])
    assert comm.allreduce_max(2.25) == 2.25
    # device buffers on the library's stream
    hip = _hip()
    src_h = np.arange(7, dtype=np.float64) * 0.5
    dst_h = np.zeros(7)
    ds, dd = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(ds), ctypes.c_size_t(56)) == 0
    assert hip.hipMalloc(ctypes.byref(dd), ctypes.c_size_t(56)) == 0
    try:
        assert hip.hipMemcpy(ds, src_h.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(56), 1) == 0  # H2D
        comm.allgather_device(ds.value, dd.value, 7)
        _lib.check(_lib.lib().aqc_stream_join(None))  # the legacy default stream waits for it
        assert hip.hipMemcpy(dst_h.ctypes.data_as(ctypes.c_void_p), dd, ctypes.c_size_t(56), 2) == 0  # D2H
        np.testing.assert_array_equal(dst_h, src_h)
    finally:
        hip.hipFree(ds)
        hip.hipFree(dd)
    comm.close()


def test_sharded_sweep_through_rccl_exchange():
    """The pair-sharded sweep (sharding.PairShard), exchanged through the RCCL communicator with
    the host-array gather, equals the unsharded sweep and picks the same pair."""
    import bench
    from adaptaqc_amd.comm import RcclComm
    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch
    from adaptaqc_amd.sharding import PairShard, gather_scores_host
    from adaptaqc_amd.utils.constants import coupling_map_fully_entangled

    n, chi = 30, 32
    cmap = coupling_map_fully_entangled(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(bench.near_product_mps(n, chi, 77))
    want = pair_grads_batch([d], svec, cmap, u0, gm, deg)
    comm = RcclComm(RcclComm.unique_id(), 0, 1)
    shard = PairShard(cmap, n, 0, 1)
    local = pair_grads_batch([d], svec, shard.local_pairs, u0, gm, deg)
    full = gather_scores_host(local, shard, comm.allgather)
    np.testing.assert_allclose(full, want, rtol=0, atol=1e-14)
    assert int(np.argmax(full[0])) == int(np.argmax(want[0]))
    comm.close()


def _two_rank_compile_worker(rank, world, port, method, out):
    """One rank of a two-rank compile on the box's one GPU: gloo carries the sweep's all-gather,
    the device sweeps (general gradient: aqc_pair_grads; ISL: pair RDMs) run on the GPU."""
    import os
    import sys

    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out[rank] = _compile(method, True)
    dist.destroy_process_group()


def _compile(method, sharded):
    from conftest import to_circuit

    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig
    from adaptaqc_amd.utils.ansatzes import identity_resolvable

    rng = np.random.default_rng(11)
    n, ops = 8, []
    for layer in range(4):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    comp = AdaptCompiler(to_circuit(n, ops), backend=AerMPSBackend(),
                         adapt_config=AdaptConfig(method=method, max_layers=4),
                         custom_layer_2q_gate=identity_resolvable(), comm=True if sharded else None)
    res = comp.compile()
    hist = comp.general_gradient_history if method == "general_gradient" else comp.entanglement_measures_history
    return (list(map(tuple, comp.qubit_pair_history)), [list(map(float, h)) for h in hist], float(res.overlap))


@pytest.mark.parametrize("method", ["general_gradient", "ISL"])
def test_two_ranks_share_each_layers_sweep(method):
    """VERDICT r5 #6 on hardware: two processes on the GPU run the same compile with a
    communicator (TorchComm over gloo); each scores its ranks' pairs on the device, and both end
    with the single-process compile's pair sequence and sweep values (to 1e-12: the device sums
    of a rank's share and of the whole map group the same chains)."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_two_rank_compile_worker, args=(2, port, method, out), nprocs=2, join=True)
    pairs, hist, ov = _compile(method, False)
    assert len(pairs) == 4 and 0.0 < ov <= 1.0
    for r in range(2):
        rp, rh, rov = out[r]
        assert rp == pairs
        assert len(rh) == len(hist)
        for a, b in zip(rh, hist):
            np.testing.assert_allclose(a, b, atol=1e-12)
        assert abs(rov - ov) < 1e-10
