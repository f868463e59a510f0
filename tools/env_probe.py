"""Where the four-workgroup environment chains spend a step (aqc_env_ticks): z_all_batch on B
50-qubit chi = 64 states, wall time per call and shader-clock ticks per step of one workgroup
(T product, its columns of the new environment, the hand-off).

    python3 tools/env_probe.py [B]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.device import DeviceMPS, z_all_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 7
n, chi = 50, 64
states = []
for k in range(B):
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(bench.near_product_mps(n, chi, 300 + k))
    states.append(d)
L = _lib.lib()
z_all_batch(states)  # warm-up
t = np.zeros(4)
_lib.check(L.aqc_env_ticks(_lib.ptr(t)))
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    z_all_batch(states)
wall = (time.perf_counter() - t0) / reps
_lib.check(L.aqc_env_ticks(_lib.ptr(t)))
steps = max(t[3], 1)
print(json.dumps({"states": B, "n": n, "chi": chi, "ms_per_call": 1e3 * wall,
                  "ticks_per_step": {"T": t[0] / steps, "new_env_columns": t[1] / steps, "handoff": t[2] / steps},
                  "steps": int(steps)}))
