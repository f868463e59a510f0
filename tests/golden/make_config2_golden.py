"""Golden values of BASELINE config 2: the exact 30-circuit workload that
tools/configs_bench.py times -- 20 qubits, brickwork depth 20 (per layer a random rx / ry / rz on
every qubit, then cx on (2i, 2i+1) / (2i+1, 2i+2) alternately), seeds 0..9, with 0 / 10 / 50
thinly-dressed layers on random pairs appended -- simulated by the oracle (oracle/sv.py, the
restatement of the reference's Aer statevector path).  Per circuit: amplitude 0 (the global cost
1 - |a0|^2), the 20 <Z_i> (the local cost), and four projections <r_k|psi> onto seeded random unit
vectors (a check of the whole state).  The three tails of a seed share their prefix, so each seed
is one simulation with snapshots.

    python tests/golden/make_config2_golden.py      # writes tests/golden/config2_sv.npz (~2 min)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import sv as osv  # noqa: E402

N, DEPTH, SEEDS, TAILS = 20, 20, range(10), (0, 10, 50)
THIN_AXES = ("rx", "rx", "rx", "rx")  # bench.THIN_AXES (bench.thin_layer_ops default)


def config2_named_ops(seed, tail_layers):
    """tools/configs_bench.py brickwork_sv_ops as (name, qubits, params): the same RNG draws."""
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(DEPTH):
        for q in range(N):
            ax = ("rx", "ry", "rz")[rng.integers(3)]
            ops.append((ax, (q,), (float(rng.uniform(-np.pi, np.pi)),)))
        for q in range(layer % 2, N - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    for t in range(tail_layers):
        a = int(rng.integers(N))
        b = int((a + 1 + rng.integers(N - 1)) % N)
        ang = rng.uniform(-np.pi, np.pi, 4)
        ops += [(THIN_AXES[0], (a,), (float(ang[0]),)), (THIN_AXES[1], (b,), (float(ang[1]),)), ("cx", (a, b), ()),
                (THIN_AXES[2], (a,), (float(ang[2]),)), (THIN_AXES[3], (b,), (float(ang[3]),))]
    return ops


def probes():
    rng = np.random.default_rng(2024)
    r = rng.standard_normal((4, 2 ** N)) + 1j * rng.standard_normal((4, 2 ** N))
    return r / np.linalg.norm(r, axis=1, keepdims=True)


def main():
    R = probes()
    amp0, z, proj = [], [], []
    for seed in SEEDS:
        full = config2_named_ops(seed, max(TAILS))
        base = len(config2_named_ops(seed, 0))
        psi, done = None, 0
        for tail in TAILS:
            upto = base + 5 * tail
            psi = osv.simulate(N, full[done:upto], psi)
            done = upto
            assert full[:upto] == config2_named_ops(seed, tail)
            amp0.append(psi[0])
            z.append(osv.z_expectations(psi, N))
            proj.append(R.conj() @ psi)
            print(f"seed {seed} tail {tail}: cost {1 - abs(psi[0]) ** 2:.15f}", flush=True)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "config2_sv.npz"),
                        amp0=np.array(amp0), z=np.array(z), proj=np.array(proj),
                        seeds=np.repeat(np.array(list(SEEDS)), len(TAILS)), tails=np.tile(np.array(TAILS), len(SEEDS)))


if __name__ == "__main__":
    main()
