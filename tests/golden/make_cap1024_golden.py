"""Golden values for the bond-capacity-1024 tests (tests/test_gpu_bigchi.py), from the oracle
(oracle/mps.py, the restatement of Aer's MPS simulator as the reference drives it):

* "brick": 21 qubits, brickwork depth 24 (ry, rz on every qubit, then cx on alternating pairs; seed 5),
  threshold 1e-8 (examples/advanced_mps_example.py:46), max_chi None -- the middle bonds reach 800
  and 704.  Stored: bond dimensions, the Schmidt values of bonds 9, 10, 11, <0..0|psi>, <Z_q> at five
  qubits, <phi_k|psi> for four seeded random product states phi_k, and the fidelity
  |<psi_exact|psi_mps>|^2 against the exact statevector (oracle/sv.py).
* "bj": 22 qubits, bench.random_vidal_mps(22, 520, 8) and one dressed CX on sites (10, 11) (seed 8):
  a 1040 x 1040 two-site block, above the Gram path's side 1024, truncated by max_chi 1024.
  Stored: bond dimensions, the Schmidt values of the new bond, <phi_k|psi> for four product states.

    python tests/golden/make_cap1024_golden.py      # writes tests/golden/cap1024.npz (~1 min, 8 cores)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import mps as M  # noqa: E402
from oracle import sv as osv  # noqa: E402


def brick_ops(n=21, depth=24, seed=5):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(depth):
        for q in range(n):
            a, b = float(rng.uniform(-np.pi, np.pi)), float(rng.uniform(-np.pi, np.pi))
            ops += [("ry", (q,), (a,)), ("rz", (q,), (b,))]
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    return ops


def bj_ops(seed=8, pair=(10, 11)):
    rng = np.random.default_rng(seed)
    ops = []
    for q in pair:
        ops.append(("ry", (q,), (rng.uniform(-np.pi, np.pi),)))
        ops.append(("rz", (q,), (rng.uniform(-np.pi, np.pi),)))
    ops.append(("cx", pair, ()))
    return ops


def product_states(n, k, seed):
    """k random product states: per qubit a unit 2-vector (phi[k][q] = (a, b))."""
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((k, n, 2)) + 1j * rng.standard_normal((k, n, 2))
    return v / np.linalg.norm(v, axis=2, keepdims=True)


def product_mps(phi):
    """Preprocessed MPS of a product state: site q = (2, 1, 1) with entries phi[q]."""
    return [np.asarray(p, dtype=complex).reshape(2, 1, 1) for p in phi]


def mps_sv_overlap(pre, psi):
    """<psi | mps> for a preprocessed MPS and a dense little-endian statevector."""
    n = len(pre)
    t = np.asarray(psi).conj().reshape(-1, 1)  # [rest x (open bond = 1)]
    for q in range(n):
        a = pre[q]  # (2, l, r)
        rest = t.shape[0] // 2
        t = t.reshape(rest, 2, t.shape[1])  # qubit q is the lowest remaining bit
        t = np.einsum("xsl,slr->xr", t, a, optimize=True)
    return complex(t.reshape(-1)[0])


def main():
    out = {}
    ops = brick_ops()
    ref = M.run_circuit(21, ops, 1e-8, None)
    pre = ref.preprocessed()
    out["brick_dims"] = np.array([1] + [x.shape[2] for x in pre])
    for b in (9, 10, 11):
        out[f"brick_lam{b}"] = ref.l[b]
    out["brick_ov0"] = np.array(M.mps_dot(pre, M.zero_mps(21)))
    out["brick_zq"] = np.array([0, 9, 10, 11, 20])
    out["brick_z"] = np.array([M.mps_expectation_z(pre, q) for q in out["brick_zq"]])
    phi = product_states(21, 4, 101)
    out["brick_phi"] = phi
    out["brick_phi_ov"] = np.array([M.mps_dot(product_mps(p), pre) for p in phi])
    psi = osv.simulate(21, ops)
    out["brick_fid_exact"] = np.array(abs(mps_sv_overlap(pre, psi)) ** 2)
    print("brick dims", out["brick_dims"].tolist(), "fidelity vs exact", float(out["brick_fid_exact"]), flush=True)

    import bench

    aer = bench.random_vidal_mps(22, 520, 8)
    ref = M.run_circuit(22, bj_ops(), 1e-16, 1024, mps=M.MPS.from_aer(aer))
    pre = ref.preprocessed()
    out["bj_dims"] = np.array([1] + [x.shape[2] for x in pre])
    out["bj_lam10"] = ref.l[10]
    phi = product_states(22, 4, 202)
    out["bj_phi"] = phi
    out["bj_phi_ov"] = np.array([M.mps_dot(product_mps(p), pre) for p in phi])
    print("bj dims", out["bj_dims"].tolist(), flush=True)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "cap1024.npz"), **out)


if __name__ == "__main__":
    main()
