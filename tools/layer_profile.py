"""One ADAPT-AQC compile layer as a reference user runs it: the paper setting
of examples/advanced_mps_example.py:40-58 -- general_gradient pair selection, the identity_resolvable
layer, rotosolve_frequency = 10, starting_circuit = "tenpy_product_state", the AerMPSBackend with the
example's truncation threshold 1e-8 (max_chi None, the reference default) -- on a 50-qubit chi = 64
target MPS, through this package's AdaptCompiler (adapt_compiler.py:585-706: the candidate sweep,
Rotoselect on the new layer, Rotosolve over the layers every 10th, absorption into the cached MPS).
Per layer: wall time and its stages (pair selection = the gradient sweep; Rotoselect; Rotosolve;
absorption; the rest), cost evaluations, the cost.  Then the oracle port (oracle/, the reference's
algorithm structure: per-pair / per-generator MPS builds and dots for the sweep, one full replay per
Rotoselect / Rotosolve candidate) on one host core for the same layer-10 circuit: a bounded sample
of its stages, scaled (stated in the output).

Per layer also the largest bond of the full circuit's MPS after the layer (one extra evaluation,
outside the stage timers) and the layer's two-site SVD paths (Gram path taken / declined).

    python3 tools/layer_profile.py [--target near-product|graded] [--layers 11] [--max-chi 0] > out.json
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


class Stages:
    def __init__(self):
        self.t = {}
        self.layer = None

    def wrap(self, obj, name, stage_of):
        fn = getattr(obj, name)

        def wrapped(*a, **k):
            t0 = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                st = stage_of(*a, **k)
                self.t[st] = self.t.get(st, 0.0) + time.perf_counter() - t0

        setattr(obj, name, wrapped)


def gpu_layers(args, record=False):
    from adaptaqc_amd.backends import AerMPSBackend, mps_sim_with_args
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig
    from adaptaqc_amd.utils.ansatzes import identity_resolvable
    from adaptaqc_amd.utils.constants import ALG_ROTOSELECT

    from adaptaqc_amd import _lib
    from adaptaqc_amd.mps_operations import device_mps_from_circuit

    if args.target == "graded":  # decaying Schmidt spectra, as a ground state's (bench.graded_vidal_mps)
        target = bench.graded_vidal_mps(bench.N_QUBITS, bench.CHI, args.seed, 0.9)
    else:
        target = bench.near_product_mps(bench.N_QUBITS, bench.CHI, args.seed)
    sim = mps_sim_with_args(mps_truncation_threshold=args.threshold, max_chi=args.max_chi or None)
    config = AdaptConfig(method="general_gradient", cost_improvement_num_layers=1e3, rotosolve_frequency=10,
                         max_layers=args.layers)
    t0 = time.perf_counter()
    comp = AdaptCompiler(target=target, backend=AerMPSBackend(simulator=sim), adapt_config=config,
                         starting_circuit="tenpy_product_state", custom_layer_2q_gate=identity_resolvable())
    setup_s = time.perf_counter() - t0
    st = Stages()
    st.wrap(comp, "_find_appropriate_qubit_pair", lambda *a, **k: "pair_selection_sweep")
    st.wrap(comp.minimizer, "minimize_cost",
            lambda *a, **k: "rotoselect" if k.get("algorithm_kind") == ALG_ROTOSELECT else "rotosolve")
    st.wrap(comp, "_absorb_n_gates_into_mps", lambda *a, **k: "absorption")
    layers = []
    add = comp._add_layer

    def add_layer(index):
        st.t = {}
        c0 = comp.cost_evaluation_counter
        _lib.gram_stats(), _lib.gram_big_stats()
        t1 = time.perf_counter()
        cost = add(index)
        wall = time.perf_counter() - t1
        g, gb = _lib.gram_stats(), _lib.gram_big_stats()
        bond = int(max(device_mps_from_circuit(comp.full_circuit, sim).dims()))
        row = {"layer": index, "wall_ms": 1e3 * wall,
               "stages_ms": {k: round(1e3 * v, 3) for k, v in st.t.items()},
               "other_ms": round(1e3 * (wall - sum(st.t.values())), 3),
               "cost_evaluations": comp.cost_evaluation_counter - c0, "cost": float(cost), "max_bond_after": bond,
               "svd": {"gram128_taken": g["taken"], "gram128_declined": g["declined_shape"] + g["declined_floor"],
                       "gram_big_taken": gb["taken"], "gram_big_declined": gb["declined"] + gb["declined_floor"]
                       + gb["timeouts"] + gb["declined_certificate"]},
               "pair": [int(x) for x in comp.qubit_pair_history[-1]]}
        layers.append(row)
        print(json.dumps(row), flush=True)
        return cost

    snap = {}

    def add_layer_snap(index):
        cost = add_layer(index)
        snap["circuit"] = comp.full_circuit.copy()  # the last layer's circuit (for the CPU port)
        snap["evals"] = layers[-1]["cost_evaluations"]
        return cost

    comp._add_layer = add_layer_snap
    # the cached Rotoselect / Rotosolve evaluator's calls of every layer (the like-for-like CPU
    # column replays them: the same prefix caching and candidate batching, on the oracle); recorded
    # in a second, untimed compile (recording snapshots the circuit per call: ~0.2 ms each)
    from adaptaqc_amd.utils import cached_rotations as cr

    calls = snap.setdefault("calls", {})
    orig_goto, orig_costs = cr.MPSPrefixBatch._goto, cr.MPSPrefixBatch._costs
    if not record:
        orig_goto = orig_costs = None

    def rec(kind, obj, index, mats=None):
        layer = len(layers)
        circ = obj.compiler.full_circuit
        calls.setdefault(layer, []).append((kind, int(index), (circ.num_qubits, _oracle_ops(circ)),
                                            None if mats is None else [np.array(m, dtype=complex) for m in mats]))

    def goto(obj, index):
        rec("goto", obj, index)
        return orig_goto(obj, index)

    def costs(obj, index, mats):
        rec("costs", obj, index, mats)
        return orig_costs(obj, index, mats)

    if record:
        cr.MPSPrefixBatch._goto, cr.MPSPrefixBatch._costs = goto, costs
    t1 = time.perf_counter()
    res = comp.compile()
    if record:
        cr.MPSPrefixBatch._goto, cr.MPSPrefixBatch._costs = orig_goto, orig_costs
    total = time.perf_counter() - t1
    comp._profile_snapshot = snap
    return comp, layers, {"setup_s": setup_s, "compile_s": total, "overlap": float(res.overlap),
                          "layers": len(layers), "cost_evaluations": int(res.cost_evaluations)}


def _oracle_ops(circ):
    from adaptaqc_amd.circuit import qubit_indices

    ops = []
    for ins in circ.data:
        name = ins.operation.name
        if name == "set_matrix_product_state":
            ops.append(("set_mps", (), (ins.operation.params[0],)))
        else:
            ops.append((name, tuple(qubit_indices(circ, ins)), tuple(float(p) for p in ins.operation.params)))
    return ops


def _apply(st, ops, thr, max_chi):
    """oracle/mps.py run_circuit's gate loop on `st` in place (no sort)."""
    from oracle import gates as OG

    for name, qubits, params in ops:
        if name in ("barrier", "measure", "id", "set_mps"):
            continue
        m = OG.matrix(name, params)
        if len(qubits) == 1:
            st.apply_1q(qubits[0], m)
        else:
            st.apply_2q(qubits[0], qubits[1], m, thr, max_chi)


def cpu_cached_replay(log, threshold, max_chi, budget_s):
    """Like for like: the device's cached evaluator (cached_rotations.MPSPrefixBatch) replayed on the
    oracle on one core -- the prefix MPS kept across candidates and gates (rebuilt from the cached
    target only when the varied gate moves left or the payload changes), each candidate's gate plus
    the suffix from a copy of it, the sort, <0|psi>.  The calls run in order until budget_s; the rest
    is scaled by candidate count (stated)."""
    from threadpoolctl import threadpool_limits

    from oracle import mps as M

    phi, pos, key = None, None, None
    t_goto = t_cand = 0.0
    n_cand_done = 0
    n_cand_all = sum(len(c[3]) for c in log if c[0] == "costs")  # (kind, index, (n, ops), mats)
    n_goto_all = sum(1 for c in log if c[0] == "goto")
    n_goto_done = 0
    t_start = time.perf_counter()
    with threadpool_limits(limits=1):
        for kind, index, (nq, ops), mats in log:
            if time.perf_counter() - t_start > budget_s and n_cand_done:
                break
            t0 = time.perf_counter()
            if kind == "goto":
                start = 1 if ops and ops[0][0] == "set_mps" else 0
                k = id(ops[0][2][0]) if start else None
                if phi is None or pos is None or index < pos or k != key:
                    phi = M.MPS.from_aer(ops[0][2][0]) if start else M.MPS(nq)
                    _apply(phi, ops[start:index], threshold, max_chi)
                else:
                    _apply(phi, ops[pos:index], threshold, max_chi)
                pos, key = index, k
                t_goto += time.perf_counter() - t0
                n_goto_done += 1
            else:
                q = ops[index][1][0]
                n = phi.n
                for m in mats:
                    st = phi.copy()
                    st.apply_1q(q, m)
                    _apply(st, ops[index + 1:], threshold, max_chi)
                    st.sort_qubits(threshold, max_chi)
                    _ = 1 - abs(M.mps_dot(st.preprocessed(), M.zero_mps(n))) ** 2
                t_cand += time.perf_counter() - t0
                n_cand_done += len(mats)
    per_cand = t_cand / max(n_cand_done, 1)
    per_goto = t_goto / max(n_goto_done, 1)
    est = t_goto + t_cand + per_cand * (n_cand_all - n_cand_done) + per_goto * (n_goto_all - n_goto_done)
    return {"cores": 1, "candidates": n_cand_all, "candidates_timed": n_cand_done, "prefix_moves": n_goto_all,
            "prefix_moves_timed": n_goto_done, "s_per_candidate": per_cand, "s_estimate": est}


def cpu_port_layer(comp, typical_evals, threshold, max_chi, pairs_sample):
    """The oracle port on one core for one layer of the same compile: one full replay of the last
    layer's circuit (cached target MPS + the layers' gates + starting^-1; the cost of one Rotoselect /
    Rotosolve candidate in the reference) and a sample of the reference-structure sweep
    (gradients.py:23-124: per pair, per generator an MPS build and a dot) on the target with the
    starting circuit's product state, scaled to the 1225 pairs."""
    from threadpoolctl import threadpool_limits

    from adaptaqc_amd.circuit import qubit_indices
    from oracle import adapt_host, gradients as ogr, mps as M

    circ = comp._profile_snapshot["circuit"]
    n = circ.num_qubits
    ops = []
    for ins in circ.data:
        name = ins.operation.name
        if name == "set_matrix_product_state":
            ops.append(("set_mps", (), (ins.operation.params[0],)))
        else:
            ops.append((name, tuple(qubit_indices(circ, ins)), tuple(float(p) for p in ins.operation.params)))
    start_ops = [(i.operation.name, tuple(qubit_indices(comp.starting_circuit, i)),
                  tuple(float(p) for p in i.operation.params)) for i in comp.starting_circuit.data]
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        st = M.run_circuit(n, ops, threshold, max_chi)
        _ = 1 - abs(M.mps_dot(st.preprocessed(), M.zero_mps(n))) ** 2
        t_eval = time.perf_counter() - t0
        psi = M.MPS.from_aer(bench.near_product_mps(bench.N_QUBITS, bench.CHI, 21)).preprocessed()
        _, og, od, inv0 = bench.oracle_layer()
        cmap = adapt_host.coupling_map_full(n)
        idx = np.random.default_rng(3).choice(len(cmap), pairs_sample, replace=False)
        t0 = time.perf_counter()
        ogr.general_grad_of_pairs_ref(psi, n, inv0, og, od, [cmap[i] for i in idx], start_ops, threshold, max_chi)
        t_pairs = time.perf_counter() - t0
    sweep_s = t_pairs / pairs_sample * len(cmap)
    return {"cores": 1, "one_evaluation_s": t_eval, "sweep_pairs_timed": pairs_sample, "sweep_pairs_s": t_pairs,
            "sweep_s_scaled": sweep_s, "evaluations_per_layer": typical_evals,
            "layer_s_estimate": sweep_s + typical_evals * t_eval,
            "note": "one core; the sweep scaled from the timed pairs to 1225, the Rotoselect / Rotosolve part as "
                    "the GPU layer's evaluation count x one full replay"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=11)
    ap.add_argument("--target", choices=["near-product", "graded"], default="near-product")
    ap.add_argument("--threshold", type=float, default=1e-8)
    ap.add_argument("--max-chi", type=int, default=0)
    ap.add_argument("--seed", type=int, default=21)
    ap.add_argument("--cpu-pairs", type=int, default=6)
    ap.add_argument("--cpu-budget", type=float, default=60.0, help="s per like-for-like replay before scaling")
    args = ap.parse_args()
    comp, layers, summary = gpu_layers(args)
    typical = [r for r in layers if r["layer"] > 0 and "rotosolve" not in r["stages_ms"]]
    with_rs = [r for r in layers if "rotosolve" in r["stages_ms"]]
    out = {"workload": "paper setting (examples/advanced_mps_example.py:40-58) on a 50-qubit chi=64 target "
                       f"({'bench.graded_vidal_mps, decay 0.9' if args.target == 'graded' else 'bench.near_product_mps'})",
           "threshold": args.threshold, "max_chi": args.max_chi or None,
           **summary,
           "median_layer_ms": float(np.median([r["wall_ms"] for r in typical])) if typical else None,
           "median_stages_ms": {k: float(np.median([r["stages_ms"].get(k, 0.0) for r in typical]))
                                for k in ("pair_selection_sweep", "rotoselect", "absorption")} if typical else None,
           "rotosolve_layer_ms": [r["wall_ms"] for r in with_rs]}
    if args.cpu_pairs > 0 and typical:
        evals = int(np.median([r["cost_evaluations"] for r in typical]))
        out["cpu_port"] = cpu_port_layer(comp, evals, args.threshold, args.max_chi or None, args.cpu_pairs)
        out["speedup_vs_cpu_1core"] = out["cpu_port"]["layer_s_estimate"] / (1e-3 * out["median_layer_ms"])
        # like for like: the device's algorithms on one CPU core -- the environment-form sweep
        # (oracle/gradients.py, the device's factorisation through T_ab) and the cached evaluator's
        # calls of the median typical layer replayed on the oracle (same prefix caching / batching)
        from threadpoolctl import threadpool_limits

        from oracle import adapt_host, gradients as ogr, mps as M

        psi = M.MPS.from_aer(bench.near_product_mps(bench.N_QUBITS, bench.CHI, 21)).preprocessed()
        _, og, od, inv0 = bench.oracle_layer()
        cmap = adapt_host.coupling_map_full(bench.N_QUBITS)
        with threadpool_limits(limits=1):
            t0 = time.perf_counter()
            ogr.general_grad_of_pairs_env(psi, bench.N_QUBITS, inv0, og, od, cmap)
            sweep_env_s = time.perf_counter() - t0
        print(json.dumps({"note": "second compile, recording the cached evaluator's calls (untimed)"}), flush=True)
        comp_rec, _, _ = gpu_layers(args, record=True)
        calls = comp_rec._profile_snapshot.get("calls", {})
        med = sorted(typical, key=lambda r: r["wall_ms"])[len(typical) // 2]
        roto = cpu_cached_replay(calls.get(med["layer"], []), args.threshold, args.max_chi or None, args.cpu_budget)
        layer_s = sweep_env_s + roto["s_estimate"]
        out["cpu_like_for_like"] = {
            "cores": 1, "layer": med["layer"], "gpu_layer_ms": med["wall_ms"], "sweep_env_s": sweep_env_s,
            "rotoselect_cached": roto, "layer_s_estimate": layer_s,
            "speedup_vs_cpu_1core_like_for_like": layer_s / (1e-3 * med["wall_ms"]),
            "note": "the device's algorithms on the oracle, one core: environment-form sweep (timed) + the "
                    "cached evaluator's recorded calls of this layer replayed with the same prefix caching "
                    "and candidate batching (timed up to the budget, the rest scaled by candidate count)"}
        if with_rs:
            rs = with_rs[0]
            rr = cpu_cached_replay(calls.get(rs["layer"], []), args.threshold, args.max_chi or None, args.cpu_budget)
            out["cpu_like_for_like"]["rotosolve_layer"] = {
                "layer": rs["layer"], "gpu_layer_ms": rs["wall_ms"], "cached": rr,
                "speedup_vs_cpu_1core_like_for_like": (sweep_env_s + rr["s_estimate"]) / (1e-3 * rs["wall_ms"])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
