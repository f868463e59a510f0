"""GPU idle time inside bench.py's steps from a rocprofv3 kernel trace (rocpd database).

    python tools/step_gaps.py gpurun_out/<dir>/run_results.db [anchor-kernel-substring]

A step runs from one launch of the anchor kernel (default k_chain) to the next.  For each step:
wall time, union of kernel busy time, idle time, and the largest gaps with the kernels on either
side -- where the host leaves the GPU waiting.
"""
import sqlite3
import sys


def main(db, anchor="k_chain"):
    c = sqlite3.connect(db)
    try:
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
    except sqlite3.OperationalError:
        cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
        print("kernels columns:", cols)
        raise
    idx = [i for i, r in enumerate(rows) if anchor in r[0]]
    for s in range(len(idx) - 1):
        seg = rows[idx[s]:idx[s + 1]]
        t0, t1 = seg[0][1], rows[idx[s + 1]][1]
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        prev_end, prev_name = None, None
        for name, st, en in seg:
            if prev_end is not None and st > prev_end:
                gaps.append((st - prev_end, prev_name, name))
            if cur_e is None or st > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
            if prev_end is None or en > prev_end:
                prev_end, prev_name = en, name
        busy += cur_e - cur_s
        gaps.sort(reverse=True)
        print(f"step {s}: wall {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms, "
              f"kernels {len(seg)}")
        for g, a, b in gaps[:6]:
            print(f"   gap {g / 1e3:8.1f} us  after {a[:60]}  before {b[:60]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
