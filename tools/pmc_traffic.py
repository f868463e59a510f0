"""HBM traffic per launch of the bench's dominant kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write k_jacobi_reg > profiles/<round>_traffic.json

FETCH_SIZE and WRITE_SIZE are kilobytes per dispatch (TCC_EA0_RDREQ / _WRREQ based).  Per
MI355X_MICROARCH.md (HBM section) gfx950's FETCH_SIZE reports half the bytes of wide coalesced
reads (16 B per lane), which is this kernel's load shape (one complex128 per lane), so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Scratch (register spill) traffic is
included: it is real memory traffic.  bench.py reads the JSON for roofline.traffic.
"""
import glob
import json
import os
import sqlite3
import sys


def per_dispatch(path, counter, kernel):
    vals = {}
    for db in glob.glob(os.path.join(path, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        for d, k, v in c.execute("select dispatch_id, kernel_name, value from counters_collection "
                                 "where counter_name = ?", (counter,)):
            if kernel in k:
                vals[(db, d)] = vals.get((db, d), 0.0) + v
    return vals


def main(fetch_dir, write_dir, kernel):
    f = per_dispatch(fetch_dir, "FETCH_SIZE", kernel)
    w = per_dispatch(write_dir, "WRITE_SIZE", kernel)
    fetch = 2.0 * 1024.0 * sum(f.values()) / max(len(f), 1)
    write = 1024.0 * sum(w.values()) / max(len(w), 1)
    print(json.dumps({"kernel": kernel, "dispatches": [len(f), len(w)],
                      "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                      "traffic_bytes_per_launch": fetch + write,
                      "note": "FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE exact; KB -> bytes"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
