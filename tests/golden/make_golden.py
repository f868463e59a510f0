"""Generate the committed golden fixtures under tests/golden/ (run in the build container).

1. ``random_mps.npz``: the reference's ``paper/random_mps/target_seed_*.pkl`` (54 x 50-qubit
   Aer-format MPS, chi = 2), read with a numpy-only unpickler (oracle/fixtures.py).  The
   reference does not exist on the GPU box, so the tests read this npz instead.
2. ``oracle_goldens.npz``: oracle outputs on those fixtures and on seeded random circuits:
   <psi|0> overlaps, <Z_i>, Hamming-weight-1 amplitudes, all-pairs gradient norms (identity-
   resolvable layer with rotoselect generators, and the thinly-dressed default layer), each
   gradient set cross-checked on a subset of pairs against the reference-structured oracle.

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""
import argparse
import glob
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import adapt_host, fixtures, gradients as gr, mps as M, sv  # noqa: E402


def layer_ops(kind):
    if kind == "identity_resolvable":
        spec = [("rx", (0,)), ("rx", (1,)), ("cx", (0, 1)), ("rx", (0,)), ("rx", (1,)), ("cx", (0, 1)),
                ("rx", (0,)), ("rx", (1,))]
    else:  # thinly dressed (ansatzes.py:41-48)
        spec = [("rx", (0,)), ("rx", (1,)), ("cx", (0, 1)), ("rx", (0,)), ("rx", (1,))]
    return [(nm, q, () if nm == "cx" else (0.0,)) for nm, q in spec]


def grad_inputs(kind):
    layer = layer_ops(kind)
    gens, deg = gr.get_generators_and_degeneracies(layer, rotoselect=True, inverse=True)
    return gr.inverse_ops(layer), gens, deg


def random_circuit_ops(n, depth, rng):
    ops = []
    for layer in range(depth):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    return ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--pairs-check", type=int, default=24)
    args = ap.parse_args()

    files = glob.glob(os.path.join(args.reference, "paper", "random_mps", "target_seed_*.pkl"))
    files.sort(key=lambda f: int(re.findall(r"seed_(\d+)", f)[0]))
    d = {"seeds": np.array([int(re.findall(r"seed_(\d+)", f)[0]) for f in files])}
    mpss = []
    for f, seed in zip(files, d["seeds"]):
        q = fixtures.load_aer_mps_pickle(f)
        mpss.append(q)
        d.update(fixtures.pack_npz_dict(q, f"s{seed}_"))
    np.savez_compressed(os.path.join(HERE, "random_mps.npz"), **d)
    print(f"random_mps.npz: {len(files)} fixtures")

    g = {}
    n = 50
    cmap = adapt_host.coupling_map_full(n)
    g["cmap"] = np.array(cmap, dtype=np.int32)
    rng = np.random.default_rng(1234)
    for kind in ("identity_resolvable", "thinly_dressed"):
        inv0, gens, deg = grad_inputs(kind)
        g[f"{kind}_ndeg"] = np.array(deg)
    pick = [0, 1, 17, 53]
    for idx in pick:
        seed = int(d["seeds"][idx])
        st = M.MPS.from_aer(mpss[idx])
        pre = st.preprocessed()
        g[f"s{seed}_ov0"] = np.array(M.mps_dot(pre, M.zero_mps(n)))
        g[f"s{seed}_z"] = np.array([M.mps_expectation_z(pre, q) for q in range(n)])
        g[f"s{seed}_hw1"] = np.array([M.extract_amplitude(pre, 1 << q) for q in range(n)])
        for kind in ("identity_resolvable", "thinly_dressed"):
            inv0, gens, deg = grad_inputs(kind)
            full = gr.general_grad_of_pairs_env(pre, n, inv0, gens, deg, cmap)
            sub = sorted(rng.choice(len(cmap), size=args.pairs_check, replace=False).tolist())
            ref = gr.general_grad_of_pairs_ref(pre, n, inv0, gens, deg, [cmap[i] for i in sub])
            err = np.max(np.abs(np.array(full)[sub] - np.array(ref)))
            assert err < 1e-12, (seed, kind, err)
            g[f"s{seed}_grad_{kind}"] = np.array(full)
            print(f"seed {seed} {kind}: max|env - ref| over {len(sub)} pairs = {err:.2e}")
    # seeded small circuits: SV amplitudes / costs and MPS with / without truncation
    for seed in range(3):
        r = np.random.default_rng(seed)
        nq = 8
        ops = random_circuit_ops(nq, 6, r)
        ops += [("cx", (0, 5), ()), ("cz", (6, 1), ()), ("swap", (2, 7), ()), ("cx", (7, 3), ())]
        psi = sv.simulate(nq, ops)
        g[f"circ{seed}_sv"] = psi
        g[f"circ{seed}_ops_names"] = np.array([o[0] for o in ops])
        g[f"circ{seed}_ops_q"] = np.array([list(o[1]) + [-1] * (2 - len(o[1])) for o in ops], dtype=np.int32)
        g[f"circ{seed}_ops_p"] = np.array([o[2][0] if o[2] else 0.0 for o in ops])
        for chi in (0, 4):
            st = M.run_circuit(nq, ops, 1e-16, chi or None)
            g[f"circ{seed}_chi{chi}_ov0"] = np.array(M.mps_dot(st.preprocessed(), M.zero_mps(nq)))
            g[f"circ{seed}_chi{chi}_z"] = np.array([M.mps_expectation_z(st.preprocessed(), q) for q in range(nq)])
            g[f"circ{seed}_chi{chi}_dims"] = np.array([1] + [x.shape[2] for x in st.preprocessed()])
    np.savez_compressed(os.path.join(HERE, "oracle_goldens.npz"), **g)
    print("oracle_goldens.npz written")


if __name__ == "__main__":
    main()
