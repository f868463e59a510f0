"""Lab: the Gram SVD's lower-triangle S3 at 1024 threads (aqc_svd_debug variant 9) against numpy on
shapes whose C selects one stage (C <= 65) or both (C > 65); variant 8 (256 threads) beside it."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_svd import _run, _spectrum_theta  # noqa: E402

for m, n in ((128, 40), (128, 64), (128, 66), (128, 80), (128, 96), (128, 128)):
    c = min(m, n)
    theta = _spectrum_theta(m, n, 0.93 ** np.arange(c), 11 + m + n)
    s_ref = np.linalg.svd(theta, compute_uv=False)
    K = min(64, c)
    out = [f"{m}x{n}"]
    for v in (8, 9):
        w, sig, _, sw = _run(theta, v)
        got = np.sort(sig)[::-1]
        out.append(f"v{v} sw={sw} err={np.max(np.abs(got[:K] - s_ref[:K])):.2e}")
    print("  ".join(out), flush=True)
