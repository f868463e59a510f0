"""Pair sharding + all-gather + arg-max across ranks (gloo, world size 2 and 3, CPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import adapt_host as H


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scores(nstates, npairs):
    rng = np.random.default_rng(42)
    s = rng.random((nstates, npairs))
    s[:, 7] = s.max(axis=1)  # ties: first index must win
    return s


def _worker(rank, world, port, n, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from adaptaqc_amd.sharding import PairShard, gather_scores, select_pairs

    cmap = H.coupling_map_full(n)
    full = _scores(3, len(cmap))
    sh = PairShard(cmap, n, rank, world)
    local = torch.as_tensor(full[:, sh.local_index], dtype=torch.float64)
    got = gather_scores(local, sh, nstates=3)
    prio = np.ones(len(cmap))
    best = select_pairs(got.numpy(), prio)
    out[rank] = (got.numpy().tobytes(), best.tolist())
    dist.destroy_process_group()


def _state_sweep_worker(rank, world, port, n, G, out):
    """Each rank computes its own block of sweeps (the oracle's environment form on CPU) through
    the product's state sharding, then one all-gather of (best pair, score)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from adaptaqc_amd.sharding import StateShard, best_pairs, gather_best

    sh = StateShard(G, rank, world)
    cmap = H.coupling_map_full(n)
    scores = torch.as_tensor(np.array([_sweep_scores(n, k, cmap) for k in sh.indices()]), dtype=torch.float64)
    best, score = best_pairs(scores, np.ones(len(cmap)))
    b_all, s_all = gather_best(best, score, sh)
    out[rank] = (b_all.numpy().tolist(), s_all.numpy().tobytes(), list(sh.indices()))
    dist.destroy_process_group()


def _sweep_scores(n, k, cmap):
    """1225-pair-style sweep of state k (random small MPS, seeded by k) by the oracle's env form."""
    from oracle import gradients as ogr
    from oracle import mps as M

    rng = np.random.default_rng(500 + k)
    ops = []
    for q in range(n):
        ops.append(("ry", (q,), (float(rng.uniform(0.1, 0.4)),)))
    for q in range(n - 1):
        ops.append(("cx", (q, q + 1), ()))
        ops.append(("rz", (q + 1,), (float(rng.uniform(-np.pi, np.pi)),)))
    psi = M.run_circuit(n, ops, 1e-16, 8).preprocessed()
    layer = [("rz", (0,), (0.3,)), ("ry", (1,), (0.2,)), ("cx", (0, 1), ()), ("rx", (0,), (0.1,)), ("rx", (1,), (0.4,))]
    gens, degs = ogr.get_generators_and_degeneracies(layer, True, True)
    return ogr.general_grad_of_pairs_env(psi, n, ogr.inverse_ops(layer), gens, degs, cmap)


@pytest.mark.parametrize("world", [2, 4])
def test_state_sharded_sweeps_across_ranks(world):
    """Config 4's decomposition: a global batch of 8 sweeps, each rank really computing its block,
    every rank ending with all 8 (pair, score) selections equal to the single-process answer."""
    n, G = 8, 8
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_state_sweep_worker, args=(world, _free_port(), n, G, out), nprocs=world, join=True)
    cmap = H.coupling_map_full(n)
    full = np.array([_sweep_scores(n, k, cmap) for k in range(G)])
    want_b = np.argmax(full, axis=1)
    want_s = full[np.arange(G), want_b]
    assert np.max(full) > 1e-3
    seen = []
    for r in range(world):
        b, s_bytes, idx = out[r]
        assert b == want_b.tolist()
        np.testing.assert_array_equal(np.frombuffer(s_bytes), want_s)
        seen += idx
    assert sorted(seen) == list(range(G))


@pytest.mark.parametrize("world", [2, 3])
def test_gather_and_argmax_across_ranks(world):
    n = 12
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    cmap = H.coupling_map_full(n)
    full = _scores(3, len(cmap))
    for r in range(world):
        got = np.frombuffer(out[r][0]).reshape(3, -1)
        np.testing.assert_array_equal(got, full)
        assert out[r][1] == np.argmax(full, axis=1).tolist()


def test_partition_balanced_and_complete():
    from adaptaqc_amd.sharding import PairShard, partition_first_qubits

    n = 50
    for world in (1, 2, 4, 8):
        parts = partition_first_qubits(n, world)
        assert sorted(a for p in parts for a in p) == list(range(n - 1))
        loads = [sum(n - 1 - a for a in p) for p in parts]
        assert max(loads) - min(loads) <= n
        cmap = H.coupling_map_full(n)
        idx = sorted(i for r in range(world) for i in PairShard(cmap, n, r, world).local_index)
        assert idx == list(range(len(cmap)))


def test_gather_scores_host_matches_global_order():
    """The host-array exchange (used with libaqchip's RCCL communicator, comm.RcclComm) puts every
    rank's shard back in the coupling-map order, for any world size, with the arg-max the
    reference takes (np.argmax, lowest index on ties)."""
    import numpy as np

    from adaptaqc_amd.sharding import PairShard, gather_scores_host
    from adaptaqc_amd.utils.constants import coupling_map_fully_entangled

    n = 11
    cmap = coupling_map_fully_entangled(n)
    rng = np.random.default_rng(3)
    truth = rng.random((2, len(cmap)))
    truth[:, 7] = truth.max() + 1  # a unique maximum
    for world in (1, 2, 3, 4):
        shards = [PairShard(cmap, n, r, world) for r in range(world)]
        locals_ = [truth[:, s.local_index] for s in shards]

        def allgather(x, w=world):  # what every rank receives from RCCL's all-gather
            m = shards[0].max_local
            out = np.zeros((w, len(x)))
            for r in range(w):
                buf = np.zeros((2, m))
                buf[:, : locals_[r].shape[1]] = locals_[r]
                out[r] = buf.reshape(-1)
            return out

        for r in range(world):
            full = gather_scores_host(locals_[r], shards[r], allgather)
            np.testing.assert_array_equal(full, truth)
            assert int(np.argmax(full[0])) == 7


def _product_sweep_setup(n):
    """A circuit (ry layer + CX ladder + rz) and the identity-resolvable layer's generators, in the
    product's types and the oracle's."""
    from adaptaqc_amd.circuit import QuantumCircuit
    from adaptaqc_amd.utils import ansatzes
    from adaptaqc_amd.utils.gradients import get_generators_and_degeneracies
    from oracle import gradients as ogr

    rng = np.random.default_rng(9)
    qc = QuantumCircuit(n)
    for q in range(n):
        qc.ry(float(rng.uniform(0.1, 0.4)), q)
    for q in range(n - 1):
        qc.cx(q, q + 1)
        qc.rz(float(rng.uniform(-np.pi, np.pi)), q + 1)
    layer = ansatzes.identity_resolvable()
    gens, degs = get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in layer.data]
    og, od = ogr.get_generators_and_degeneracies(o_layer, True, True)
    return qc, layer, gens, degs, o_layer, og, od


def _oracle_scorer(calls):
    """Stand-ins for the device replay and the device sweep (no GPU here): the oracle's MPS of the
    circuit and its environment-form gradients of exactly the pairs asked for."""
    from oracle import gradients as ogr
    from oracle import mps as M

    def replay(circuit, sim=None, **_):
        ops = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in circuit.data]
        return M.run_circuit(circuit.num_qubits, ops, 1e-16, 8).preprocessed()

    def grads(psi, n, inverse_zero_ansatz, generators, degeneracies, pairs, starting_circuit=None, backend=None):
        calls.append(list(pairs))
        o_inv = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in inverse_zero_ansatz.data]
        o_gens = [[(i.operation.name, i.qubits, tuple(i.operation.params)) for i in g.data] for g in generators]
        return ogr.general_grad_of_pairs_env(psi, n, o_inv, o_gens, list(degeneracies), list(pairs))

    return replay, grads


def _product_comm_worker(rank, world, port, n, out):
    """The product's general_grad_of_pairs and AdaptCompiler's pair choice with a TorchComm (gloo):
    each rank scores its share (oracle injected for the device), one all-gather, same selection."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from types import SimpleNamespace

    from adaptaqc_amd.compilers.adapt.adapt_compiler import AdaptCompiler
    from adaptaqc_amd.compilers.adapt.adapt_config import AdaptConfig
    from adaptaqc_amd.sharding import TorchComm
    from adaptaqc_amd.utils import gradients as gr

    qc, layer, gens, degs, _, _, _ = _product_sweep_setup(n)
    cmap = H.coupling_map_full(n)
    calls = []
    gr.device_mps_from_circuit, gr.grads_for_state = _oracle_scorer(calls)
    comm = TorchComm()
    got = gr.general_grad_of_pairs(qc, layer.inverse(), gens, degs, cmap, None, SimpleNamespace(simulator=None),
                                   comm=comm)
    # the compiler's own sweep and selection (adapt_compiler.py:832-856) on the same communicator
    ac = object.__new__(AdaptCompiler)
    ac.__dict__.update(starting_circuit=None, full_circuit=qc, inverse_zero_ansatz=layer.inverse(), generators=gens,
                       degeneracies=degs, coupling_map=cmap, backend=SimpleNamespace(simulator=None), comm=comm,
                       qubit_pair_history=[(0, 1), (2, 3)], adapt_config=AdaptConfig(), initial_single_qubit_layer=False)
    g2 = ac._get_all_qubit_pair_gradients()
    pick = ac._find_best_gradient_qubit_pair(g2)
    out[rank] = (np.asarray(got).tobytes(), np.asarray(g2).tobytes(), tuple(pick), calls)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_product_sweep_shares_pairs_across_ranks(world):
    """the product's general_grad_of_pairs / AdaptCompiler with a communicator.  Every
    rank scores only the pairs of its first qubits, and every rank ends with the single-process
    gradient list (bit for bit: the same oracle scores, gathered) and the same selected pair."""
    from types import SimpleNamespace

    from adaptaqc_amd.compilers.adapt.adapt_compiler import AdaptCompiler
    from adaptaqc_amd.compilers.adapt.adapt_config import AdaptConfig
    from adaptaqc_amd.utils import gradients as gr

    n = 9
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_product_comm_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    qc, layer, gens, degs, _, _, _ = _product_sweep_setup(n)
    cmap = H.coupling_map_full(n)
    calls = []
    saved = gr.device_mps_from_circuit, gr.grads_for_state
    try:
        gr.device_mps_from_circuit, gr.grads_for_state = _oracle_scorer(calls)
        want = gr.general_grad_of_pairs(qc, layer.inverse(), gens, degs, cmap, None, SimpleNamespace(simulator=None))
        ac = object.__new__(AdaptCompiler)
        ac.__dict__.update(starting_circuit=None, full_circuit=qc, inverse_zero_ansatz=layer.inverse(), generators=gens,
                           degeneracies=degs, coupling_map=cmap, backend=SimpleNamespace(simulator=None), comm=None,
                           qubit_pair_history=[(0, 1), (2, 3)], adapt_config=AdaptConfig(),
                           initial_single_qubit_layer=False)
        want_pick = ac._find_best_gradient_qubit_pair(ac._get_all_qubit_pair_gradients())
    finally:
        gr.device_mps_from_circuit, gr.grads_for_state = saved
    assert calls[0] == cmap and max(want) > 1e-3
    scored = []
    for r in range(world):
        got, g2, pick, rcalls = out[r]
        np.testing.assert_array_equal(np.frombuffer(got), want)
        np.testing.assert_array_equal(np.frombuffer(g2), want)
        assert pick == tuple(want_pick)
        assert len(rcalls) == 2 and rcalls[0] == rcalls[1] and len(rcalls[0]) < len(cmap)
        scored += rcalls[0]
    assert sorted(scored) == sorted(cmap)  # every pair scored by exactly one rank
