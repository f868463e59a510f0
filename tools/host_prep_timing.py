"""Host-side time of each call in bench.py's step (no extra syncs: the calls return as soon as their
work is queued, so each figure is the host's own cost -- plan building, staging, launches -- except
overlap_zero_batch, whose read-back waits for the chain).  Lab tool, 1 GPU.

    python3 tools/host_prep_timing.py [steps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import (DeviceMPS, apply_batch, check_batch, copy_batch,  # noqa: E402
                                 overlap_zero_batch, pair_grads_batch)
from adaptaqc_amd.sharding import PairShard, gather_scores  # noqa: E402
from adaptaqc_amd.utils.constants import coupling_map_fully_entangled  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
n, B = bench.N_QUBITS, 256
cmap = coupling_map_fully_entangled(n)
shard = PairShard(cmap, n, 0, 1)
layer, gens, deg, u0, gm = bench.layer_inputs()
svec = np.zeros((n, 2), complex)
svec[:, 0] = 1.0
distinct = bench.bench_states(n, bench.CHI, 8, "near-product")
states = []
for s in range(B):
    d = DeviceMPS(n, bench.CHI, 1e-16, bench.CHI)
    d.load_aer(distinct[s % len(distinct)])
    states.append(d)
work = [DeviceMPS(n, bench.CHI, 1e-16, bench.CHI) for _ in range(4 * B)]
src = [states[k // 4] for k in range(4 * B)]
rng = np.random.default_rng(7)
ops = [_lib.ops_array(bench.thin_layer_ops(bench.LAYER_A, bench.LAYER_A + d, rng.uniform(-np.pi, np.pi, 4)))
       for s in range(B) for d in bench.DISTANCES]
scores = torch.zeros((B, len(cmap)), dtype=torch.float64, device="cuda")
prio = torch.ones(len(cmap), dtype=torch.float64, device="cuda")
T = {}
for it in range(K + 1):
    if it == 1:
        T.clear()
    marks = [("start", time.perf_counter())]
    pair_grads_batch(states, svec, shard.local_pairs, u0, gm, deg, out=scores.data_ptr())
    marks.append(("sweep", time.perf_counter()))
    full = gather_scores(scores, shard, nstates=B)
    best = torch.argmax(full * prio, dim=1)
    marks.append(("gather+argmax", time.perf_counter()))
    copy_batch(work, src)
    marks.append(("copy_batch", time.perf_counter()))
    apply_batch(work, ops, sort=True, wait=False)
    marks.append(("apply_batch", time.perf_counter()))
    costs = 1.0 - np.abs(overlap_zero_batch(work)) ** 2
    marks.append(("overlap0 (waits)", time.perf_counter()))
    check_batch(work)
    marks.append(("check_batch", time.perf_counter()))
    for (_, a), (name, b) in zip(marks, marks[1:]):
        T[name] = T.get(name, 0.0) + (b - a)
    T["step"] = T.get("step", 0.0) + (marks[-1][1] - marks[0][1])
for k, v in T.items():
    print(f"{k:18s} {1e3 * v / K:9.3f} ms/step (host)")
