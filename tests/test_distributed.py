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
