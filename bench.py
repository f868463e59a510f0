"""Benchmark: overlap + gradient evaluations / s, 50-qubit MPS chi = 64 (BASELINE.json config 3).

One step, per rank, on a global batch of S = world * states_per_rank synthetic random 50-qubit
MPS (Vidal form, bonds min(2^k, 2^(50-k), 64)), all resident in HBM:
  (i)  candidate sweep: gradient norm of the identity_resolvable layer (rotoselect generators,
       12 distinct, |s> = |0..0>) for all 1225 pairs of the full coupling map, pairs sharded
       across ranks by first qubit (each rank covers its shard for all S states), one RCCL
       all-gather of the float64 scores, and the per-state arg-max pair selection;
  (ii) overlap evaluations on this rank's own states_per_rank states: apply a thinly-dressed
       layer (4 rotations + CX) at pair distances 1, 2, 5, 25 (Aer swap routing, two-site SVD
       with max_chi = 64 truncation, sort back at save) and take 1 - |<0|psi>|^2.
value = (S * 1225 + S * 4) evaluations / step time (max over ranks): weak scaling.

Also reported: the dominant kernel's roofline (HIP events on the MPS stream around every launch
of the timed region) and a CPU baseline: the oracle's port of the reference algorithm
(per-pair, per-generator MPS build + whole-psi dot; numpy LAPACK SVDs) timed on a bounded
sample on rank 0 at N = 1.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_QUBITS = 50
CHI = 64
DISTANCES = (1, 2, 5, 25)
LAYER_A = 12
FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (vector = matrix), MI355X_MICROARCH.md / SURVEY 8(d)
HBM_PEAK_GBS = 8000.0
TRAFFIC_JSON = "r1_traffic.json"


def vidal_from_tensors(A):
    """Vidal canonical form (Aer tuple) of the MPS with site tensors A[i] of shape (2, l, r):
    left-canonicalise by QR, then right-to-left SVDs give the lambdas; normalised."""
    A = [np.asarray(a, dtype=complex).copy() for a in A]
    n = len(A)
    for i in range(n - 1):  # left-canonicalise
        s, l, r = A[i].shape
        q, rr = np.linalg.qr(A[i].transpose(1, 0, 2).reshape(l * s, r))
        A[i] = q.reshape(l, s, -1).transpose(1, 0, 2)
        A[i + 1] = np.einsum("ab,sbc->sac", rr, A[i + 1])
    A[n - 1] /= np.linalg.norm(A[n - 1])
    lam = [None] * (n + 1)
    for i in range(n - 1, 0, -1):  # right sweep with SVDs -> lambdas
        s, l, r = A[i].shape
        u, sv, vh = np.linalg.svd(A[i].transpose(1, 0, 2).reshape(l, s * r), full_matrices=False)
        sv = sv / np.linalg.norm(sv)
        lam[i] = sv
        A[i] = vh.reshape(-1, s, r).transpose(1, 0, 2)
        A[i - 1] = np.einsum("sab,bc->sac", A[i - 1], u * sv[None, :])
    gam = []
    for i in range(n):
        g = A[i]
        if i == 0:
            g = g / lam[1][None, None, :]
        elif i < n - 1:
            g = g / lam[i + 1][None, None, :]
        gam.append((g[0].copy(), g[1].copy()))
    return gam, [lam[i] for i in range(1, n)]


def random_vidal_mps(n, chi, seed):
    """Random normalised MPS in exact Vidal canonical form (Aer tuple): bonds min(2^k, 2^(n-k), chi),
    complex-normal tensors."""
    rng = np.random.default_rng(seed)
    dims = [min(2 ** k, 2 ** (n - k), chi) for k in range(n + 1)]
    A = [(rng.standard_normal((2, dims[i], dims[i + 1])) + 1j * rng.standard_normal((2, dims[i], dims[i + 1])))
         for i in range(n)]
    return vidal_from_tensors(A)


def thin_layer_ops(a, b, angles):
    """Thinly-dressed CNOT layer with rotoselect-style angles: rx, rx, cx, rx, rx."""
    from adaptaqc_amd import gates as G

    rx = lambda t: G.one_qubit("rx", [t])
    return [(rx(angles[0]), (a,)), (rx(angles[1]), (b,)), (G.TWO_QUBIT["cx"], (a, b)),
            (rx(angles[2]), (a,)), (rx(angles[3]), (b,))]


def layer_inputs():
    from adaptaqc_amd.utils import ansatzes
    from adaptaqc_amd.utils.gradients import get_generators_and_degeneracies, layer_operators

    layer = ansatzes.identity_resolvable()
    gens, deg = get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
    u0, gm = layer_operators(layer.inverse(), gens)
    return layer, gens, deg, u0, np.stack(gm)


def svd_nominal_flops(m, n):
    """LAPACK-style complex SVD with both singular-vector sets: 4 x (4m^2n + 8mn^2 + 9n^3), m >= n."""
    m, n = max(m, n), min(m, n)
    return 4.0 * (4 * m * m * n + 8 * m * n * n + 9 * n ** 3)


def cpu_baseline(seed_states, layer, u0, gm, deg, budget_s=20.0):
    """Oracle port of the reference path on a bounded sample (rank 0, N = 1)."""
    from oracle import adapt_host, gradients as ogr, mps as M

    qmps = seed_states[0]
    n = N_QUBITS
    st = M.MPS.from_aer(qmps)
    psi = st.preprocessed()
    o_layer = [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in layer.data]
    og, od = ogr.get_generators_and_degeneracies(o_layer, True, True)
    inv0 = ogr.inverse_ops(o_layer)
    cmap = adapt_host.coupling_map_full(n)
    rng = np.random.default_rng(0)
    # (ii) overlap evals: replay the layer on the cached MPS + <0|psi> (reference: Aer replay)
    t0 = time.perf_counter()
    n_ov = 0
    for d in DISTANCES:
        ops = [("rx", (LAYER_A,), (0.3,)), ("rx", (LAYER_A + d,), (0.7,)), ("cx", (LAYER_A, LAYER_A + d), ()),
               ("rx", (LAYER_A,), (-0.2,)), ("rx", (LAYER_A + d,), (1.1,))]
        out = M.run_circuit(n, ops, 1e-16, CHI, mps=st)
        _ = 1 - abs(M.mps_dot(out.preprocessed(), M.zero_mps(n))) ** 2
        n_ov += 1
    t_ov = (time.perf_counter() - t0) / n_ov
    # (i) gradient evals: reference structure on a sample of pairs
    t0 = time.perf_counter()
    n_gr = 0
    order = rng.permutation(len(cmap))
    while time.perf_counter() - t0 < budget_s and n_gr < len(cmap):
        pair = cmap[order[n_gr]]
        ogr.general_grad_of_pairs_ref(psi, n, inv0, og, od, [pair], (), 1e-16, CHI)
        n_gr += 1
    t_gr = (time.perf_counter() - t0) / max(n_gr, 1)
    per_state = len(DISTANCES) * t_ov + len(cmap) * t_gr
    return {
        "value": (len(DISTANCES) + len(cmap)) / per_state,
        "unit": "evals/s",
        "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
        "kind": "port",
        "sample": (f"1 state: {len(DISTANCES)} overlap evals ({t_ov * 1e3:.1f} ms each) + {n_gr} of 1225 pair "
                   f"gradients ({t_gr * 1e3:.1f} ms each, 12 generators) extrapolated to the step mix"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--states", type=int, default=256, help="states per rank")
    ap.add_argument("--distinct", type=int, default=8, help="distinct random states generated")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="projection only (1 process): rank 0's share of an N-GPU run -- pair shard of N, "
                         "sweep over N x states -- with the all-gather replaced by a local scatter")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ["AQC_DEVICE"] = str(local)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceMPS, apply_batch, copy_batch, overlap_zero_batch, pair_grads_batch
    from adaptaqc_amd.sharding import PairShard, gather_scores
    from adaptaqc_amd.utils.constants import coupling_map_fully_entangled

    n, B = N_QUBITS, args.states
    sim = args.simulate_world if (args.simulate_world > 1 and world == 1) else 0
    shard_world = sim or world
    S = shard_world * B
    cmap = coupling_map_fully_entangled(n)
    shard = PairShard(cmap, n, rank, shard_world)
    layer, gens, deg, u0, gm = layer_inputs()
    svec = np.zeros((n, 2), complex)
    svec[:, 0] = 1.0

    distinct = [random_vidal_mps(n, CHI, 1000 + k) for k in range(min(args.distinct, S))]
    states = []
    for s in range(S):
        d = DeviceMPS(n, CHI, 1e-16, CHI)
        d.load_aer(distinct[s % len(distinct)])
        states.append(d)
    own = states[rank * B:(rank + 1) * B]
    work = [DeviceMPS(n, CHI, 1e-16, CHI) for _ in range(B * len(DISTANCES))]
    reload_src = [own[k // len(DISTANCES)] for k in range(len(work))]
    rng = np.random.default_rng(7)
    layer_ops = []
    for s in range(B):
        for d in DISTANCES:
            layer_ops.append(_lib.ops_array(thin_layer_ops(LAYER_A, LAYER_A + d, rng.uniform(-np.pi, np.pi, 4))))
    prio = np.ones(len(cmap))
    local_scores = torch.zeros((S, max(len(shard.local_pairs), 1)), dtype=torch.float64, device="cuda")

    def step():
        # (i) sharded candidate sweep + all-gather + arg-max
        if shard.local_pairs:
            pair_grads_batch(states, svec, shard.local_pairs, u0, gm, deg, out=local_scores.data_ptr())
        if sim:  # projection: rank 0's scores scattered locally, no collective
            full = torch.zeros((S, len(cmap)), dtype=torch.float64, device="cuda")
            full[:, torch.as_tensor(shard.local_index, device="cuda")] = local_scores[:, : len(shard.local_pairs)]
        else:
            full = gather_scores(local_scores[:, : len(shard.local_pairs)], shard, nstates=S)
        best = torch.argmax(full * torch.as_tensor(prio, device=full.device), dim=1)
        # (ii) overlap evals on own states
        copy_batch(work, reload_src)
        apply_batch(work, layer_ops, sort=True)  # replay + save (sorted), as mps_from_circuit
        ov = overlap_zero_batch(work)
        costs = 1.0 - np.abs(ov) ** 2
        return best, costs

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    _lib.timing_reset()
    _lib.timing_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        best, costs = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    _lib.timing_enable(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        chk = best.to(torch.int64).clone()
        ref = chk.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(chk, ref), "arg-max pair differs across ranks"
    ms_step = 1e3 * elapsed / args.steps
    evals_per_step = S * (len(cmap) + len(DISTANCES))
    value = evals_per_step * args.steps / elapsed

    fams = {f: _lib.timing_query(f)
            for f in ("mps_chain", "mps_svd", "mps_theta", "mps_split", "grad_chain", "mps_overlap0", "mps_copy")}
    dom = max(fams, key=lambda f: fams[f]["ms"])
    fd = fams[dom]
    launches = max(fd["launches"], 1)
    avg_ms = fd["ms"] / launches
    if dom == "mps_chain":
        # fused per-state chain (k_chain): per two-site update the nominal SVD flops of the
        # 128 x 128 theta (84 n^3) + theta (32 chi^3) + split GEMM (32 chi^3), from the launch's
        # KernelTimer record; one launch serves every state of the step
        roof = {"kernel": "k_chain (fused two-site updates: theta, Jacobi SVD, split)", "bound": "mfma",
                "achieved": fd["flops"] / launches / (avg_ms * 1e-3) / 1e12, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "updates_per_launch": fd["flops"] / launches / ((84.0 * 8 + 64.0) * CHI ** 3),
                "svd_share_of_flops": 84.0 * 8 / (84.0 * 8 + 64.0)}
    elif dom == "mps_svd":
        # jobs per launch: the 4B two-site updates of one lock-step wave (all 128 x 128 at chi = 64)
        jobs = fd["bytes"] / (2.0 * 4 * CHI * CHI * 16)
        achieved_flop = jobs / launches * svd_nominal_flops(2 * CHI, 2 * CHI)
        roof = {"kernel": "k_jacobi (two-site SVD)", "bound": "mfma", "achieved": achieved_flop / (avg_ms * 1e-3) / 1e12,
                "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s"}
    else:
        roof = {"kernel": dom, "bound": "hbm", "achieved": fd["bytes"] / launches / (avg_ms * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof["frac"] = roof["achieved"] / roof["peak"]
    roof["traffic"] = None
    # HBM bytes per launch of the same kernel and launch mix from the committed PMC passes
    # (tools/pmc_bench.sh: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md corrections)
    tj = os.path.join(ROOT, "profiles", TRAFFIC_JSON)
    want = {"mps_chain": "k_chain", "mps_svd": "k_jacobi_reg"}.get(dom)
    if want and os.path.exists(tj):
        with open(tj) as fh:
            tr = json.load(fh)
        if tr["kernel"] == want:
            roof["traffic"] = tr["traffic_bytes_per_launch"]
            roof["traffic_source"] = f"profiles/{TRAFFIC_JSON} ({tr['kernel']}, rocprofv3 PMC)"
    if want:
        roof["algorithmic_bytes_per_launch"] = fd["bytes"] / launches
    roof["avg_launch_ms"] = avg_ms
    roof["launches"] = fd["launches"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(distinct, layer, u0, gm, deg, args.cpu_budget)

    if rank == 0 and sim:
        print(json.dumps({"projection": f"rank 0 of a {sim}-GPU run on one GPU (no collective)",
                          "ms_per_step": ms_step, "per_gpu_evals_per_s": evals_per_step / sim * args.steps / elapsed,
                          "projected_value": evals_per_step * args.steps / elapsed,
                          "breakdown_ms": {f: round(v["ms"] / args.steps, 3) for f, v in fams.items()}}))
    elif rank == 0:
        line = {
            "metric": "overlap+gradient evals/sec, 50-qubit MPS chi=64, 1/2/4/8 MI355X",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "c128",
            "data": "synthetic random Vidal MPS (seeded), random layer angles",
            "config": {
                "workload": "config3: 50-qubit chi=64 MPS; per state 1225-pair identity_resolvable gradient sweep "
                            "(sharded, RCCL all-gather, arg-max) + 4 thinly-dressed-layer overlap evals (d=1,2,5,25)",
                "n_qubits": n, "chi": CHI, "states_per_rank": B, "global_states": S,
                "pairs": len(cmap), "generators": int(len(deg)), "parallelism": f"pairs sharded x{world}",
            },
            "breakdown_ms": {f: round(v["ms"] / args.steps, 3) for f, v in fams.items()},
            "gradient_evals_per_s": S * len(cmap) * args.steps / elapsed,
            "overlap_evals_per_s": S * len(DISTANCES) * args.steps / elapsed,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
