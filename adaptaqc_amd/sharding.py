"""Candidate-pair sharding across the GPUs of one node (one process per GPU).

The sweep (gradients.general_grad_of_pairs) produces one score per coupling-map pair; the pair
with the largest ``score * reuse_priority`` wins (adapt_compiler.py:832-837, np.argmax = first
maximum).  Pairs are independent, so each rank computes the pairs whose first qubit
``a = min(c, t)`` it owns -- one device chain per owned ``a`` -- and a single all-gather of the
float64 scores (RCCL over xGMI with backend "nccl"; gloo on CPU for tests) gives every rank the
full vector, after which every rank takes the identical arg-max.  psi itself is replicated by
deterministic recomputation on every rank, so the gather is the only exchange.
"""
from __future__ import annotations

import numpy as np


def chain_work(n, a):
    """Device work of the chain for first qubit a (vector-matrix steps)."""
    return n - 1 - a


def partition_first_qubits(n, world):
    """Greedy longest-first assignment of first qubits to ranks, balancing sum of chain work."""
    load = [0] * world
    owner = [0] * max(n - 1, 0)
    for a in sorted(range(n - 1), key=lambda x: -chain_work(n, x)):
        r = min(range(world), key=lambda k: (load[k], k))
        owner[a] = r
        load[r] += chain_work(n, a)
    return [[a for a in range(n - 1) if owner[a] == r] for r in range(world)]


def local_pair_indices(coupling_map, owned_first):
    owned = set(owned_first)
    return [i for i, (c, t) in enumerate(coupling_map) if min(c, t) in owned]


class PairShard:
    """Static description of one rank's share of a coupling map."""

    def __init__(self, coupling_map, n, rank, world):
        self.coupling_map = list(coupling_map)
        self.rank, self.world = rank, world
        parts = partition_first_qubits(n, world)
        self.index_lists = [local_pair_indices(self.coupling_map, p) for p in parts]
        self.local_index = self.index_lists[rank]
        self.local_pairs = [self.coupling_map[i] for i in self.local_index]
        self.max_local = max((len(x) for x in self.index_lists), default=0)


def gather_scores(local_scores, shard: PairShard, group=None, nstates: int = 1):
    """All-gather per-rank scores ([nstates, n_local] torch tensor) into the global pair order.

    Returns a torch tensor [nstates, n_pairs] identical on every rank.
    """
    import torch
    import torch.distributed as dist

    dev = local_scores.device
    m = shard.max_local
    buf = torch.zeros((nstates, m), dtype=torch.float64, device=dev)
    buf[:, : local_scores.shape[1]] = local_scores
    if shard.world > 1:
        gathered = torch.empty((shard.world * nstates, m), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(gathered, buf.contiguous(), group=group)
        gathered = gathered.view(shard.world, nstates, m)
    else:
        gathered = buf.unsqueeze(0)
    full = torch.empty((nstates, len(shard.coupling_map)), dtype=torch.float64, device=dev)
    for r, idx in enumerate(shard.index_lists):
        if idx:
            full[:, torch.as_tensor(idx, device=dev)] = gathered[r, :, : len(idx)]
    return full


def select_pairs(full_scores, priorities):
    """np.argmax(scores * priorities) per state (first index wins ties)."""
    s = np.asarray(full_scores, dtype=np.float64) * np.asarray(priorities, dtype=np.float64)
    return np.argmax(s, axis=-1)
