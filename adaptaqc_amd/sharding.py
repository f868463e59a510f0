"""Candidate sweep sharding across the GPUs of one node (one process per GPU).

Two decompositions of the sweep (gradients.general_grad_of_pairs) over ranks:

* pairs (one sweep, latency): below.  Every rank rebuilds the environments of psi; the chains
  of the owned first qubits are the only part that divides, so the sweep's critical path (the
  n-step environment chain, bound by one CU's streaming rate) does not shrink with the rank count.
* states (many sweeps, throughput; config 4's strong scaling): a fixed global batch of G states --
  independent sweeps, e.g. the candidate states of a layer search or several targets compiled
  together -- split into contiguous blocks of G / world states per rank (``StateShard``); each rank
  runs its sweeps on its own GPU and one all-gather of the per-state (best pair, best score) gives
  every rank all G selections.  No environment or psi is exchanged.

Pairs:

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
    # the index lists go to the device once per shard and device: a fresh host->device copy here
    # would wait for the scores' producer (the sweep) and stall the host every step
    cache = shard.__dict__.setdefault("_index_dev", {})
    if dev not in cache:
        cache[dev] = [torch.as_tensor(idx, device=dev) if idx else None for idx in shard.index_lists]
    for r, (idx, di) in enumerate(zip(shard.index_lists, cache[dev])):
        if idx:
            full[:, di] = gathered[r, :, : len(idx)]
    return full


def gather_scores_host(local_scores, shard: PairShard, allgather):
    """The same exchange with host arrays and any all-gather callable (``allgather(x)`` returns
    (world, len(x)) in rank order): libaqchip's RCCL communicator (``comm.RcclComm.allgather``)
    for callers without torch.distributed, or a gloo/MPI stand-in in tests.  local_scores:
    [nstates, n_local] numpy.  Returns [nstates, n_pairs], identical on every rank."""
    local = np.asarray(local_scores, dtype=np.float64)
    nstates = local.shape[0]
    m = shard.max_local
    buf = np.zeros((nstates, m))
    buf[:, : local.shape[1]] = local
    gathered = np.asarray(allgather(buf.reshape(-1))).reshape(shard.world, nstates, m)
    full = np.empty((nstates, len(shard.coupling_map)))
    for r, idx in enumerate(shard.index_lists):
        if idx:
            full[:, idx] = gathered[r, :, : len(idx)]
    return full


def select_pairs(full_scores, priorities):
    """np.argmax(scores * priorities) per state (first index wins ties)."""
    s = np.asarray(full_scores, dtype=np.float64) * np.asarray(priorities, dtype=np.float64)
    return np.argmax(s, axis=-1)


class StateShard:
    """Contiguous block of a global batch of G independent states (one sweep each) for one rank."""

    def __init__(self, global_states, rank, world):
        if global_states % world:
            raise ValueError(f"global batch {global_states} does not divide over {world} ranks")
        self.global_states, self.rank, self.world = global_states, rank, world
        self.per_rank = global_states // world
        self.start = rank * self.per_rank
        self.stop = self.start + self.per_rank

    def indices(self):
        return range(self.start, self.stop)


def best_pairs(scores, priorities):
    """Per-state arg-max of scores * priorities (first maximum, as np.argmax) and its score, on the
    scores' device: ([S] int64, [S] float64).  On a GPU: libaqchip's arg-max kernel
    (device.argmax_rows); host tensors (gloo tests) take torch's."""
    import torch

    p = priorities if isinstance(priorities, torch.Tensor) else torch.as_tensor(
        np.asarray(priorities, dtype=np.float64))
    p = p.to(device=scores.device, dtype=torch.float64)
    if scores.is_cuda:
        from .device import argmax_rows

        return argmax_rows(scores.contiguous(), p.contiguous())
    s = scores[:, : p.shape[0]] * p
    best = torch.argmax(s, dim=1)
    return best, s.gather(1, best[:, None])[:, 0]


def gather_best(best, score, shard: StateShard, group=None):
    """All-gather every rank's per-state (best pair index, score) into global state order: one
    collective of 2 x per_rank float64 per rank (RCCL over xGMI with backend "nccl")."""
    import torch
    import torch.distributed as dist

    local = torch.stack([best.to(torch.float64), score.to(torch.float64)])  # [2, per_rank]
    if shard.world == 1:
        return best.to(torch.int64), score
    out = torch.empty((shard.world * 2, shard.per_rank), dtype=torch.float64, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    out = out.view(shard.world, 2, shard.per_rank).permute(1, 0, 2).reshape(2, -1)
    return out[0].to(torch.int64), out[1]


# ---- the product's communicator: one per-layer pair sweep over the ranks of one node -----------
class TorchComm:
    """A torch.distributed process group as the sweep's communicator: ``allgather`` of host float64
    scores in rank order.  Backend "nccl" (RCCL over xGMI on MI355X) gathers through a device
    buffer on this rank's GPU; gloo (CPU, the tests) on host tensors."""

    def __init__(self, group=None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("TorchComm needs torch.distributed.init_process_group first")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._nccl = dist.get_backend(group) == "nccl"

    def allgather(self, local) -> np.ndarray:
        import torch
        import torch.distributed as dist

        x = torch.as_tensor(np.ascontiguousarray(np.asarray(local, dtype=np.float64).reshape(-1)))
        if self._nccl:
            x = x.to(f"cuda:{torch.cuda.current_device()}")
        out = torch.empty((self.world * x.numel(),), dtype=torch.float64, device=x.device)
        dist.all_gather_into_tensor(out, x, group=self.group)
        return out.cpu().numpy().reshape(self.world, -1)

    def __reduce__(self):  # (a compiler pickled at a checkpoint drops the communicator)
        return (_no_comm, ())


def _no_comm():
    return None


def as_comm(comm):
    """None (one process), an object with ``rank``, ``world`` and ``allgather`` (``TorchComm``,
    ``comm.RcclComm``), a torch.distributed ProcessGroup, or True for the default group."""
    if comm is None or comm is False:
        return None
    if comm is True:
        return TorchComm()
    if hasattr(comm, "allgather") and hasattr(comm, "world") and hasattr(comm, "rank"):
        return comm
    return TorchComm(comm)


def sharded_pair_scores(score_pairs, pairs, n, comm):
    """Scores of every pair of ``pairs`` (coupling-map order) with this rank computing only its
    share: ``score_pairs(local_pairs) -> list`` runs on the rank's GPU for the pairs whose first
    qubit min(c, t) the rank owns (PairShard: first qubits balanced by chain length), and one
    all-gather of the float64 scores gives every rank the whole vector -- so every rank's np.argmax
    (adapt_compiler.py:832-837, first maximum on ties) picks the same pair.  One process: the
    plain sweep."""
    comm = as_comm(comm)
    pairs = list(pairs)
    if comm is None or comm.world == 1:
        return [float(x) for x in score_pairs(pairs)]
    shard = PairShard(pairs, n, comm.rank, comm.world)
    local = np.asarray(score_pairs(shard.local_pairs) if shard.local_pairs else [], dtype=np.float64)
    full = gather_scores_host(local[None, :], shard, comm.allgather)[0]
    return [float(x) for x in full]
