"""Which singular values the register Jacobi variants get wrong on degenerate spectra (aqc_svd_debug
variants 2 = 16-lane groups, 5 = 8-lane groups, 3 = no QR), at 2 chi = 128, 64 and 32."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_svd import _run, _spectrum_theta  # noqa: E402

for n in (128, 64, 32):
    for name, s in [("2x1 + graded", np.concatenate([np.ones(2), 0.5 * 0.9 ** np.arange(n - 2)])),
                    ("8x1 + 1e-3", np.concatenate([np.ones(8), 1e-3 * np.ones(n - 8)])),
                    ("4x1 + 4x0.5 + graded", np.concatenate([np.ones(4), 0.5 * np.ones(4), 0.2 * 0.9 ** np.arange(n - 8)]))]:
        th = _spectrum_theta(n, n, s, 5)
        ref = np.linalg.svd(th, compute_uv=False)
        for v in ((2, 5, 8, 9) if n == 128 else (2, 3)):
            w, sig, _, sw = _run(th, v)
            d = np.sort(sig)[::-1] - ref
            idx = np.argsort(-np.abs(d))[:4]
            print(f"n={n:3d} {name:22s} v{v} sweeps {sw:2d}: worst idx {idx.tolist()} d {[float('%.2e' % x) for x in d[idx]]}", flush=True)
