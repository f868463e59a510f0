"""Host-side wall time of each call in bench.py's step (AQC_HT=1 also prints the library's own
host phases): which host work leaves the GPU idle between kernels."""
import os
import sys
import time

sys.argv = ["bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-parity", "--no-latency"]
os.environ["AQC_HT"] = "1"
sys.path.insert(0, os.getcwd())
from adaptaqc_amd import device  # noqa: E402


def wrap(name):
    f = getattr(device, name)

    def g(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        print(f"py {name} {1e3 * (time.perf_counter() - t):.3f} ms", file=sys.stderr)
        return r
    setattr(device, name, g)


for n in ("apply_batch", "copy_batch", "overlap_zero_batch", "pair_grads_batch"):
    wrap(n)
import runpy  # noqa: E402

runpy.run_path("bench.py", run_name="__main__")
