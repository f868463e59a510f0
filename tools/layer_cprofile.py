"""Host-side profile (cProfile) of a short paper-setting compile (tools/layer_profile.py's graded
target, 4 layers, no CPU port): where the host spends the Rotoselect visits' time between device
calls.  Prints the top functions by cumulative and by own time."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import layer_profile as lp

    class A:
        target, threshold, max_chi, seed, layers = "graded", 1e-8, 0, 21, 2

    lp.gpu_layers(A)  # warm-up compile (library load, first allocations)
    A.layers = 4
    pr = cProfile.Profile()
    pr.enable()
    lp.gpu_layers(A)
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
