"""Config 2 through the compiler's own path: ``AerSVBackend.evaluate_global_cost`` on QuantumCircuit
objects (the circuit -> aqc_op_t conversion included), with one gate's angle rewritten in place
before every evaluation as Rotosolve does.  Two modes: the memoised conversion the backend uses
(``circuit.device_ops_array``) and a fresh conversion every time (``ops_array(device_ops(...))``).
One JSON line per mode.  Usage: python3 tools/sv_compiler_path.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd.circuit import QuantumCircuit, device_ops, device_ops_array  # noqa: E402
from adaptaqc_amd.device import DeviceSV  # noqa: E402


def brickwork_qc(n, depth, seed):
    rng = np.random.default_rng(seed)
    qc = QuantumCircuit(n)
    for layer in range(depth):
        for q in range(n):
            getattr(qc, ("rx", "ry", "rz")[rng.integers(3)])(rng.uniform(-np.pi, np.pi), q)
        for q in range(layer % 2, n - 1, 2):
            qc.cx(q, q + 1)
    return qc


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = 20
    circuits = [brickwork_qc(n, 20, seed) for seed in range(10)]
    sv = DeviceSV(n)
    rng = np.random.default_rng(1)
    for mode in ("memo", "fresh"):
        conv = (lambda qc: device_ops_array(qc)) if mode == "memo" else (lambda qc: _lib.ops_array(device_ops(qc)))
        for qc in circuits:  # warm-up (first conversions, plans)
            sv.reset()
            sv.apply(conv(qc))
            sv.amp0()
        n_ev, t_conv = 0, 0.0
        t0 = time.perf_counter()
        for _ in range(reps):
            for qc in circuits:
                for _k in range(3):  # Rotosolve: three angles of one gate, evaluated in turn
                    ins = qc.data[int(rng.integers(len(qc.data)))]
                    if ins.operation.params:
                        ins.operation.params[0] = float(rng.uniform(-np.pi, np.pi))
                    t1 = time.perf_counter()
                    ops = conv(qc)
                    t_conv += time.perf_counter() - t1
                    sv.reset()
                    sv.apply(ops)
                    _ = 1.0 - abs(sv.amp0()) ** 2
                    n_ev += 1
        el = time.perf_counter() - t0
        print(json.dumps({"metric": "SV evaluate_global_cost evals/sec through the backend path (config 2 circuits)",
                          "mode": mode, "value": n_ev / el, "unit": "evals/s", "ms_per_eval": 1e3 * el / n_ev,
                          "conversion_ms_per_eval": 1e3 * t_conv / n_ev, "gates": len(circuits[0].data),
                          "note": "brickwork depth 20 seeds 0-9 as QuantumCircuit objects; one angle rewritten "
                                  "in place before each evaluation"}), flush=True)


if __name__ == "__main__":
    main()
