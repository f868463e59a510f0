"""cProfile of one Rotoselect layer pass through this package's cached evaluator (the binding
test's own_run: 50-qubit chi = 64 near-product MPS + one thinly-dressed layer on (20, 21)), to see
where a gate's ~1.4 ms goes beside the batched GPU work.  Usage: python3 tools/roto_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
from adaptaqc_amd.backends import AerMPSBackend, mps_sim_with_args  # noqa: E402
from adaptaqc_amd.circuit import QuantumCircuit  # noqa: E402
from adaptaqc_amd.utils.cached_rotations import make_evaluator  # noqa: E402
from adaptaqc_amd.utils.cost_minimiser import CostMinimiser  # noqa: E402
from conftest import FakeCompiler  # noqa: E402
from test_gpu_binding import _thin_layer_ir  # noqa: E402


def main():
    n, chi = 50, 64
    rng = np.random.default_rng(77)
    full = QuantumCircuit(n)
    full.set_matrix_product_state(bench.near_product_mps(n, chi, 12))
    _thin_layer_ir(full, [(20, 21)], rng)
    be = AerMPSBackend(mps_sim_with_args(max_chi=chi))
    n_rot = sum(1 for ins in full.data[1:] if ins.operation.name in ("rx", "ry", "rz"))

    def run():
        fc = FakeCompiler(full.copy())
        fc.backend = be
        fc.cost_evaluation_counter = 0
        fc.optimise_local_cost = False

        def cost():
            fc.cost_evaluation_counter += 1
            return be.evaluate_global_cost(fc)

        cm = CostMinimiser(cost, lambda: (1, len(fc.full_circuit.data)), fc.full_circuit,
                           evaluator_factory=lambda: make_evaluator(fc))
        cost()
        t0 = time.perf_counter()
        cm._reduce_cost(True, None)
        return time.perf_counter() - t0

    run()
    ts = [run() for _ in range(5)]
    print(f"rotations {n_rot}, per gate ms: {[round(1e3 * t / n_rot, 3) for t in ts]}", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        run()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
