"""One two-site update (CX 24,25 on a random chi=64 MPS): Jacobi variants vs the oracle (lab tool)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from adaptaqc_amd import _lib  # noqa: E402
from adaptaqc_amd import gates as G  # noqa: E402
from adaptaqc_amd.device import DeviceMPS  # noqa: E402
from oracle import mps as M  # noqa: E402

l = _lib.lib()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
chi = int(sys.argv[2]) if len(sys.argv) > 2 else 64
a = n // 2 - 1
q = bench.random_vidal_mps(n, chi, 1000)
ref = M.MPS.from_aer(q)
ref.apply_2q(a, a + 1, G.TWO_QUBIT["cx"], 1e-16, chi)
rg, rl = ref.to_aer()


def theta2(g, lam, p):
    ll = lam[p - 1] if p > 0 else np.ones(1)
    lr = lam[p + 1] if p + 1 < len(g) - 1 else np.ones(1)
    A = np.stack(g[p]) * ll[None, :, None] * lam[p][None, None, :]
    B = np.stack(g[p + 1]) * lr[None, None, :]
    return np.einsum("aim,bmj->aibj", A, B)


tref = theta2(rg, rl, a)
for v in (3, 2):
    _lib.check(l.aqc_mps_set_jacobi_variant(v))
    d = DeviceMPS(n, chi, 1e-16, chi)
    d.load_aer(q)
    d.apply(_lib.ops_array([(G.TWO_QUBIT["cx"], (a, a + 1))]))
    g, lam = d.to_aer()
    lerr = np.max(np.abs(lam[a] - rl[a])) if len(lam[a]) == len(rl[a]) else f"len {len(lam[a])} vs {len(rl[a])}"
    t = theta2(g, lam, a)
    terr = np.max(np.abs(t - tref)) if t.shape == tref.shape else f"shape {t.shape} vs {tref.shape}"
    # isometry checks: left-canonical A = Gp * ll must have orthonormal columns
    ll = lam[a - 1]
    A = (np.stack(g[a]) * ll[None, :, None]).reshape(-1, len(lam[a]))
    lr = lam[a + 1] if a + 1 < n - 1 else np.ones(1)
    B = (np.stack(g[a + 1]) * lr[None, None, :]).transpose(1, 0, 2).reshape(len(lam[a]), -1)
    print(f"variant {v}: lambda err {lerr}, theta' err {terr}, "
          f"|A^H A - I| {np.max(np.abs(A.conj().T @ A - np.eye(A.shape[1]))):.2e}, "
          f"|B B^H - I| {np.max(np.abs(B @ B.conj().T - np.eye(B.shape[0]))):.2e}, ov {d.overlap_zero()}", flush=True)
print("oracle ov", M.mps_dot(ref.preprocessed(), M.zero_mps(n)))
