"""Wall-clock split of one bench step into phases (syncs between phases; lab tool, 1 GPU)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, apply_batch, copy_batch, overlap_zero_batch, pair_grads_batch  # noqa: E402
from adaptaqc_amd.sharding import PairShard, gather_scores  # noqa: E402
from adaptaqc_amd.utils.constants import coupling_map_fully_entangled  # noqa: E402

n, B = 50, int(sys.argv[1]) if len(sys.argv) > 1 else 256
cmap = coupling_map_fully_entangled(n)
shard = PairShard(cmap, n, 0, 1)
layer, gens, deg, u0, gm = bench.layer_inputs()
svec = np.zeros((n, 2), complex)
svec[:, 0] = 1.0
distinct = [bench.random_vidal_mps(n, 64, 1000 + k) for k in range(8)]
states = []
for s in range(B):
    d = DeviceMPS(n, 64, 1e-16, 64)
    d.load_aer(distinct[s % 8])
    states.append(d)
work = [DeviceMPS(n, 64, 1e-16, 64) for _ in range(4 * B)]
src = [states[k // 4] for k in range(4 * B)]
rng = np.random.default_rng(7)
ops = [_lib.ops_array(bench.thin_layer_ops(12, 12 + d, rng.uniform(-np.pi, np.pi, 4))) for s in range(B) for d in bench.DISTANCES]
scores = torch.zeros((B, len(cmap)), dtype=torch.float64, device="cuda")
T = {}


def tick(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0)
    return t


for it in range(4):
    if it == 1:
        T.clear()
    t = time.perf_counter()
    pair_grads_batch(states, svec, shard.local_pairs, u0, gm, deg, out=scores.data_ptr())
    t = tick("sweep", t)
    full = gather_scores(scores, shard, nstates=B)
    best = torch.argmax(full, dim=1)
    t = tick("gather+argmax", t)
    copy_batch(work, src)
    t = tick("copy", t)
    apply_batch(work, ops)
    t = tick("apply_batch", t)
    ov = overlap_zero_batch(work)
    t = tick("overlap0", t)
for k, v in T.items():
    print(f"{k:15s} {1e3 * v / 3:9.2f} ms/step")
