"""Candidate sweep on the headline batch (256 states, 50 q, chi = 64, 1225 pairs): time of
pair_grads_batch per chain mode (aqc_sweep_set_chain_mode 1 = one chain per workgroup, 2 = first
qubits grouped 8 to a workgroup on the matrix cores), and the max difference between the modes."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, pair_grads_batch  # noqa: E402
from adaptaqc_amd.utils.constants import coupling_map_fully_entangled  # noqa: E402

n, chi = bench.N_QUBITS, bench.CHI
S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cmap = coupling_map_fully_entangled(n)
layer, gens, deg, u0, gm = bench.layer_inputs()
svec = np.zeros((n, 2), complex)
svec[:, 0] = 1.0
distinct = bench.bench_states(n, chi, 4, "near-product")
states = []
for s in range(S):
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(distinct[s % 4])
    states.append(d)
out = torch.zeros((S, len(cmap)), dtype=torch.float64, device="cuda")
res = {}
ref = None
for mode in (1, 2):
    _lib.check(_lib.lib().aqc_sweep_set_chain_mode(ctypes.c_int(mode)))
    pair_grads_batch(states, svec, cmap, u0, gm, deg, out=out.data_ptr())
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pair_grads_batch(states, svec, cmap, u0, gm, deg, out=out.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    got = out.cpu().numpy().copy()
    if ref is None:
        ref = got
    res[f"mode{mode}_ms"] = 1e3 * float(np.median(ts))
    res[f"mode{mode}_maxdiff_vs_mode1"] = float(np.max(np.abs(got - ref)))
_lib.check(_lib.lib().aqc_sweep_set_chain_mode(ctypes.c_int(0)))
res["grad_max"] = float(np.max(ref))
print(json.dumps(res))
