"""Compile wall time: cached Rotoselect/Rotosolve candidates vs the reference's per-candidate
simulations (lab tool, 1 GPU)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend  # noqa: E402
from adaptaqc_amd.backends.aer_mps_backend import mps_sim_with_args  # noqa: E402
from adaptaqc_amd.circuit import QuantumCircuit  # noqa: E402
from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig  # noqa: E402


def target(n, depth, seed):
    rng = np.random.default_rng(seed)
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            getattr(qc, ["rx", "ry", "rz"][rng.integers(3)])(rng.uniform(-np.pi, np.pi), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    return qc


for label, n, backend_fn, method in (("SV 12q", 12, AerSVBackend, "ISL"),
                                     ("SV 16q", 16, AerSVBackend, "ISL"),
                                     ("MPS 20q chi32", 20, lambda: AerMPSBackend(mps_sim_with_args(max_chi=32)), "ISL")):
    for cached in (False, True):
        comp = AdaptCompiler(target(n, 3, 1), backend=backend_fn(),
                             adapt_config=AdaptConfig(method=method, max_layers=8))
        comp.use_cached_rotations = cached
        t0 = time.perf_counter()
        res = comp.compile()
        dt = time.perf_counter() - t0
        print(f"{label:14s} cached={cached!s:5s} {dt:8.2f} s  layers={len(comp.qubit_pair_history)} "
              f"evals={comp.cost_evaluation_counter} overlap={res.overlap:.6f}", flush=True)
