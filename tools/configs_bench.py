"""Measurement of BASELINE.json configs 2, 4 and 5 on one MI355X (config 3 is bench.py).

    python tools/configs_bench.py [--configs 2,4,5] [--reps N]

One JSON line per config, each with the dominant kernel's roofline (HIP events on the launch
stream, libaqchip's KernelTimer) -- the unit of work and its algorithmic bytes / flops are the
SURVEY.md 8(d) figures of record:
  * config 2: 20-qubit random brickwork circuit (depth 20, seeds 0..9; per layer rx/ry/rz on every
    qubit with U(-pi, pi) angle and axis, then cx on (2i, 2i+1) or (2i+1, 2i+2) alternately) plus
    a tail of 0 / 10 / 50 thinly-dressed layers; one evaluate_global_cost = reset + full
    re-simulation + amp0 (the reference's structure, aer_sv_backend.py:23-47).  Kernel unit: one
    fused segment = one pass over the 16 MiB state, 32 * 2^n bytes.
  * config 4: 50-qubit chi = 128 candidate sweep (1225 pairs, identity_resolvable generators,
    |s> = |0..0>) on B states; the gradient-chain kernel's flops (16 chi^2 per (pair, bond) step).
  * config 5: 100-qubit chi = 256 MPS: a brickwork layer of (rz ry rz) x (rz ry rz) . CX two-site
    gates on 24 disjoint neighbouring pairs in the middle of a random chi = 256 Vidal MPS
    (max_chi = 256, threshold 1e-16; the disjoint updates run as one lock-step wave); unit = one
    two-site gate at full chi: contraction 32 chi^3 + SVD nominal 84 (2 chi)^3 flops (SURVEY 8d:
    0.54 + 11.3 GFLOP).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd import gates as G  # noqa: E402

FP64_PEAK = bench.FP64_PEAK_TFLOPS
HBM_PEAK = bench.HBM_PEAK_GBS


def roof_hbm(fam):
    q = _lib.timing_query(fam)
    avg = q["ms"] / max(q["launches"], 1)
    ach = q["bytes"] / max(q["launches"], 1) / (avg * 1e-3) / 1e9
    return {"kernel": fam, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK, "unit": "GB/s", "frac": ach / HBM_PEAK,
            "traffic": None, "avg_launch_ms": avg, "launches": q["launches"]}


def roof_flops(fam, flops_per_launch=None):
    q = _lib.timing_query(fam)
    n = max(q["launches"], 1)
    avg = q["ms"] / n
    f = q["flops"] / n if flops_per_launch is None else flops_per_launch
    ach = f / (avg * 1e-3) / 1e12
    return {"kernel": fam, "bound": "mfma", "achieved": ach, "peak": FP64_PEAK, "unit": "TFLOP/s",
            "frac": ach / FP64_PEAK, "traffic": None, "avg_launch_ms": avg, "launches": q["launches"]}


def brickwork_sv_ops(n, depth, seed, tail_layers):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(depth):
        for q in range(n):
            ax = ("rx", "ry", "rz")[rng.integers(3)]
            ops.append((G.one_qubit(ax, [rng.uniform(-np.pi, np.pi)]), (q,)))
        for q in range(layer % 2, n - 1, 2):
            ops.append((G.TWO_QUBIT["cx"], (q, q + 1)))
    for t in range(tail_layers):
        a = int(rng.integers(n))
        b = int((a + 1 + rng.integers(n - 1)) % n)
        ops += bench.thin_layer_ops(a, b, rng.uniform(-np.pi, np.pi, 4))
    return _lib.ops_array(ops)


def config2(reps):
    from adaptaqc_amd.device import DeviceSV

    n = 20
    circuits = [brickwork_sv_ops(n, 20, seed, tail) for seed in range(10) for tail in (0, 10, 50)]
    sv = DeviceSV(n)
    for ops in circuits[:3]:  # warm-up
        sv.reset()
        sv.apply(ops)
        sv.amp0()
    def run():
        n_ev = 0
        t0 = time.perf_counter()
        for _ in range(reps):
            for ops in circuits:
                sv.reset()
                sv.apply(ops)
                _ = 1.0 - abs(sv.amp0()) ** 2
                n_ev += 1
        return n_ev, time.perf_counter() - t0

    evals, el = run()  # wall rate without per-launch timing events
    _lib.timing_reset()
    _lib.timing_enable(True)
    run()  # kernel durations for the roofline
    _lib.timing_enable(False)
    roof = roof_hbm("sv_segment")
    # the register-tile kernel also carries the fused gates' arithmetic: report the FP64 side too
    fl = roof_flops("sv_segment")
    roof["fp64"] = {"achieved": fl["achieved"], "peak": fl["peak"], "unit": "TFLOP/s", "frac": fl["frac"]}
    if fl["frac"] > roof["frac"]:
        roof["bound_note"] = "FP64 arithmetic of the fused gates exceeds the HBM fraction (MALL-resident state)"
    gates = float(np.mean([len(c) for c in circuits]))
    # Independent evaluations side by side (Rotoselect candidates, several compiles): B state
    # vectors, each on its own stream, the B circuits' passes in flight together (two tile
    # workgroups per CU: two waves per SIMD) -- reported beside the one-at-a-time rate, checked
    # against it value for value.
    conc = {}
    seq_costs = []
    for ops in circuits:
        sv.reset()
        sv.apply(ops)
        seq_costs.append(1.0 - abs(sv.amp0()) ** 2)
    for B in (2, 4):
        svs = [DeviceSV(n) for _ in range(B)]

        def run_b():
            n_ev, costs = 0, []
            t0 = time.perf_counter()
            for _ in range(reps):
                for g in range(0, len(circuits), B):
                    grp = circuits[g:g + B]
                    for st, ops in zip(svs, grp):
                        st.reset()
                        st.apply(ops)
                    for st, _ in zip(svs, grp):
                        costs.append(1.0 - abs(st.amp0()) ** 2)
                        n_ev += 1
            return n_ev, time.perf_counter() - t0, costs

        run_b()
        nb, elb, costs = run_b()
        same = float(np.max(np.abs(np.array(costs[:len(circuits)]) - np.array(seq_costs))))
        conc[f"streams_{B}"] = {"evals_per_s": nb / elb, "max_abs_diff_vs_one_at_a_time": same}
        del svs
    return {"metric": "SV evaluate_global_cost evals/sec, 20 qubits (config 2)", "value": evals / el,
            "concurrent": conc,
            "unit": "evals/s", "ms_per_eval": 1e3 * el / evals, "dtype": "c128", "data": "synthetic",
            "config": {"workload": "config2: 20-qubit brickwork depth 20 (seeds 0-9) + 0/10/50 thin layers; "
                                   "full re-simulation from |0> + amp0 per eval", "n_qubits": n,
                       "mean_gates": gates, "segments_per_eval": roof["launches"] / evals},
            "roofline": roof}


def config4(states, reps):
    from adaptaqc_amd.device import DeviceMPS, pair_grads_batch
    from adaptaqc_amd.utils.constants import coupling_map_fully_entangled

    n, chi = 50, 128
    cmap = coupling_map_fully_entangled(n)
    layer, gens, deg, u0, gm = bench.layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0
    # near-product states: gradients well above rounding (random Vidal states give ~1e-16)
    distinct = [bench.near_product_mps(n, chi, 2000 + k) for k in range(min(states, 4))]
    st = []
    for s in range(states):
        d = DeviceMPS(n, chi, 1e-16, chi)
        d.load_aer(distinct[s % len(distinct)])
        st.append(d)
    out = pair_grads_batch(st, svec, cmap, u0, gm, deg)
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        out = pair_grads_batch(st, svec, cmap, u0, gm, deg)
    el = time.perf_counter() - t0
    _lib.timing_enable(False)
    roof = roof_flops("grad_chain")
    return {"metric": "candidate-sweep gradient evals/sec, 50-qubit MPS chi=128 (config 4, 1 GPU)",
            "value": states * len(cmap) * reps / el, "unit": "evals/s", "ms_per_sweep": 1e3 * el / (reps * states),
            "dtype": "c128", "data": "synthetic near-product Vidal MPS (bench.near_product_mps)",
            "config": {"workload": "config4: 1225-pair identity_resolvable sweep, |s>=|0..0>", "n_qubits": n,
                       "chi": chi, "states": states, "mean_grad": float(np.mean(out))},
            "roofline": roof}


def config5(gates, reps):
    from adaptaqc_amd.device import DeviceMPS

    n, chi = 100, 256
    rng = np.random.default_rng(0)
    aer = bench.random_vidal_mps(n, chi, 5)
    base = DeviceMPS(n, chi, 1e-16, chi)
    base.load_aer(aer)
    work = DeviceMPS(n, chi, 1e-16, chi)

    def brick(a):
        u = [G.one_qubit(g, [rng.uniform(-np.pi, np.pi)]) for g in ("rz", "ry", "rz", "rz", "ry", "rz")]
        ua = u[2] @ u[1] @ u[0]
        ub = u[5] @ u[4] @ u[3]
        return [(ua, (a,)), (ub, (a + 1,)), (G.TWO_QUBIT["cx"], (a, a + 1))]

    mid = n // 2 - gates  # disjoint neighbouring pairs in the middle (all bonds at chi)
    ops = _lib.ops_array([o for k in range(gates) for o in brick(mid + 2 * k)])
    work.copy_from(base)
    work.apply(ops)
    work.dims()
    _lib.gram_big_stats()  # reset
    gbt = np.zeros(9)
    _lib.check(_lib.lib().aqc_svd_gram_big_ticks(_lib.ptr(gbt)))  # reset
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        work.copy_from(base)
        work.apply(ops)
        work.dims()  # synchronises
    el = time.perf_counter() - t0
    _lib.timing_enable(False)
    gbs = _lib.gram_big_stats()
    _lib.check(_lib.lib().aqc_svd_gram_big_ticks(_lib.ptr(gbt)))
    if gbs["taken"]:
        ncol = reps * (2 * chi - 1)  # job 0's columns over the timed calls
        gbs["ticks_per_column"] = {k: gbt[i] / ncol for i, k in enumerate(
            ("pass", "publish", "wait", "reads_pv", "w_row_norms"))}
        gbs["ticks_per_column"]["zlarfg"] = gbt[8] / ncol
        gbs["ticks_per_call"] = {"eigenvalues": gbt[5] / reps, "back": gbt[6] / reps, "inverse_iteration": gbt[7] / reps}
    import ctypes
    sw = ctypes.c_int()
    _lib.check(_lib.lib().aqc_mps_jacobi_stats(work.h, ctypes.byref(sw)))
    nom = 32.0 * chi ** 3 + bench.svd_nominal_flops(2 * chi, 2 * chi)
    svd = _lib.timing_query("mps_svd")
    th = _lib.timing_query("mps_theta")
    sp = _lib.timing_query("mps_split")
    per_gate_ms = 1e3 * el / (reps * gates)
    # one lock-step wave holds all `gates` disjoint updates: nominal flops per launch = gates x
    roof = roof_flops("mps_svd", gates * bench.svd_nominal_flops(2 * chi, 2 * chi))
    bj = np.zeros(4)
    _lib.check(_lib.lib().aqc_bj_ticks(_lib.ptr(bj)))  # block-pair visit phases (pair mode)
    if bj[3] > 0:
        roof["pair_visit_ticks"] = {"gram": bj[0] / bj[3], "jacobi": bj[1] / bj[3], "apply": bj[2] / bj[3],
                                    "visits": bj[3]}
    return {"metric": "two-site gate applications/sec at full chi, 100-qubit MPS chi=256 (config 5)",
            "value": reps * gates / el, "unit": "gates/s", "ms_per_gate": per_gate_ms,
            "nominal_tflops": nom / (per_gate_ms * 1e-3) / 1e12, "dtype": "c128", "data": "synthetic random Vidal MPS",
            "config": {"workload": "config5: (rz ry rz)x(rz ry rz).CX on disjoint middle pairs, max_chi=256",
                       "n_qubits": n, "chi": chi, "gates": gates, "max_jacobi_sweeps": sw.value,
                       "svd_path": "gram_big" if gbs["taken"] else "block_jacobi", "gram_big_stats": gbs,
                       "dims_after": [int(x) for x in work.dims()[mid:mid + 2 * gates + 1]]},
            "breakdown_ms_per_gate": {"svd": svd["ms"] / (reps * gates), "theta": th["ms"] / (reps * gates),
                                      "split": sp["ms"] / (reps * gates)},
            "roofline": roof}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,4,5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--states4", type=int, default=128)
    ap.add_argument("--gates5", type=int, default=24)
    ap.add_argument("--chain-mode", type=int, default=0, help="aqc_sweep_set_chain_mode (0 auto, 1, 2)")
    args = ap.parse_args()
    import ctypes
    _lib.check(_lib.lib().aqc_sweep_set_chain_mode(ctypes.c_int(args.chain_mode)))
    os.environ.setdefault("AQC_DEVICE", "0")
    for c in args.configs.split(","):
        if c == "2":
            r = config2(args.reps)
        elif c == "4":
            r = config4(args.states4, args.reps)
        elif c == "5":
            r = config5(args.gates5, args.reps)
        else:
            raise SystemExit(f"unknown config {c}")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
