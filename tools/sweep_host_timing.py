"""Where the time of bench.py's sweep-only rate goes (by_kind.gradient_evals_per_s): 256 states,
chi = 64, 1225 pairs.  Wall time per call of (a) pair_grads_batch with a host result, (b) with a
device result (stream-ordered, no host wait) plus torch.cuda.synchronize, (c) bench.py's sweep():
(b) + gather_scores + arg-max, and (d) k back-to-back calls of (c) with one sync at the end.

    python3 tools/sweep_host_timing.py [reps]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch

    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch
    from adaptaqc_amd.sharding import PairShard, gather_scores
    from adaptaqc_amd.utils.constants import coupling_map_fully_entangled

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n, chi, S = bench.N_QUBITS, bench.CHI, 256
    cmap = coupling_map_fully_entangled(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    distinct = [bench.near_product_mps(n, chi, 1000 + k) for k in range(8)]
    states = []
    for s in range(S):
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.load_aer(distinct[s % 8])
        states.append(d)
    shard = PairShard(cmap, n, 0, 1)
    out = torch.zeros((S, len(cmap)), dtype=torch.float64, device="cuda")
    prio_t = torch.ones(len(cmap), dtype=torch.float64, device="cuda")

    def a():
        pair_grads_batch(states, svec, cmap, u0, gm, deg)

    def b():
        pair_grads_batch(states, svec, cmap, u0, gm, deg, out=out.data_ptr())
        torch.cuda.synchronize()

    def c():
        pair_grads_batch(states, svec, shard.local_pairs, u0, gm, deg, out=out.data_ptr())
        full = gather_scores(out, shard, nstates=S)
        best = torch.argmax(full * prio_t, dim=1)
        torch.cuda.synchronize()
        return best

    def c_nosync():
        pair_grads_batch(states, svec, shard.local_pairs, u0, gm, deg, out=out.data_ptr())
        full = gather_scores(out, shard, nstates=S)
        return torch.argmax(full * prio_t, dim=1)

    res = {}
    for name, fn in (("a_host_out", a), ("b_device_out_sync", b), ("c_bench_sweep_sync", c)):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name + "_ms"] = 1e3 * float(np.median(ts))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c_nosync()
    torch.cuda.synchronize()
    res["d_bench_sweep_pipelined_ms"] = 1e3 * (time.perf_counter() - t0) / reps
    # host-side cost of one call alone (launch path, no GPU wait): time to return
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pair_grads_batch(states, svec, cmap, u0, gm, deg, out=out.data_ptr())
    res["e_call_return_ms"] = 1e3 * (time.perf_counter() - t0)
    torch.cuda.synchronize()
    res["gradient_evals_per_s_pipelined"] = S * len(cmap) / (res["d_bench_sweep_pipelined_ms"] * 1e-3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
