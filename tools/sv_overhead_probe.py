"""Fixed per-evaluation cost of the SV path: reset + a one-gate apply + amp0 in a loop (wall) against
the kernel time (HIP events), n = 14 and 20.  Usage: python3 tools/sv_overhead_probe.py"""
import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
from adaptaqc_amd import _lib
from adaptaqc_amd.device import DeviceSV
from adaptaqc_amd import gates as G
for n in (14, 20):
    sv = DeviceSV(n)
    ops = _lib.ops_array([(G.one_qubit("rx", [0.3]), (0,))])
    for _ in range(50): sv.reset(); sv.apply(ops); sv.amp0()
    t = time.perf_counter(); N = 2000
    for _ in range(N): sv.reset(); sv.apply(ops); sv.amp0()
    el = (time.perf_counter() - t) / N
    _lib.timing_reset(); _lib.timing_enable(True)
    for _ in range(200): sv.reset(); sv.apply(ops); sv.amp0()
    _lib.timing_enable(False)
    k = _lib.timing_query("sv_segment")
    print(f"n={n}: one-gate eval {el*1e6:.1f} us wall, kernel {k['ms']/k['launches']*1e3:.1f} us")
    t = time.perf_counter()
    for _ in range(N): sv.amp0()
    print(f"  amp0 again (handed off, stream idle) {(time.perf_counter()-t)/N*1e6:.1f} us")
