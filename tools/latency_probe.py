"""Single-state latency (bench.py's latency block: one overlap evaluation per distance, one
Rotoselect gate's 7 evaluations as a batch) under the lock-step launches (fused chain from 32
states, the default) and under the fused chain for any batch size (aqc_mps_set_fused_chain(2)).
One JSON line per mode.  Usage: python3 tools/latency_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402


def main():
    q0 = bench.bench_states(bench.N_QUBITS, bench.CHI, 1)[0]
    L = _lib.lib()
    for mode in (1, 2, 1):
        _lib.check(L.aqc_mps_set_fused_chain(mode))
        out = bench.latency_block(q0, None)
        out = {k: v for k, v in out.items() if k.startswith(("overlap_eval_ms", "rotoselect_gate_7"))}
        print(json.dumps({"fused_chain_mode": mode, **out}), flush=True)
    _lib.check(L.aqc_mps_set_fused_chain(1))


if __name__ == "__main__":
    main()
