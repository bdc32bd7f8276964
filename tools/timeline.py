#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 --kernel-trace database: the window between the ends of two
consecutive steps (one training step), per HW queue: busy time, idle gaps, and the kernels in
order. Shows which branch stream is the critical path. A step ends with its last RMSprop launch
before the next step's loss kernel (the fused backward + RMSprop issues one launch per layer, the
last after the join).

    python tools/timeline.py gpurun_out/prof/run_results.db [--step -2] [--list]
"""
import argparse
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--step", type=int, default=-2, help="which step window (python index over rmsprop ends)")
    p.add_argument("--list", action="store_true")
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id, grid_x, grid_y, grid_z from kernels order by start").fetchall()
    ends, last = [], None
    for r in rows:
        if "rmsprop" in r[0]:
            last = r[2] if last is None else max(last, r[2])
        elif "::ce_kernel" in r[0] and last is not None:
            ends.append(last)
            last = None
    if last is not None:
        ends.append(last)
    t0, t1 = ends[a.step - 1], ends[a.step]
    win = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    print(f"step window {(t1 - t0) / 1e3:.1f} us, {len(win)} kernels")
    by_q = {}
    for r in win:
        by_q.setdefault(r[3], []).append(r)
    for q, ks in sorted(by_q.items(), key=lambda kv: kv[1][0][1]):
        busy = sum(k[2] - k[1] for k in ks)
        span = ks[-1][2] - ks[0][1]
        print(f"queue {q}: {len(ks)} kernels, busy {busy / 1e3:.1f} us, span {(ks[0][1] - t0) / 1e3:.1f}.."
              f"{(ks[-1][2] - t0) / 1e3:.1f} us ({span / 1e3:.1f})")
        if a.list:
            prev = None
            for k in ks:
                gap = (k[1] - prev) / 1e3 if prev else 0.0
                print(f"   {(k[1] - t0) / 1e3:8.1f} +{(k[2] - k[1]) / 1e3:7.1f} (gap {gap:5.1f})  "
                      f"[{k[4]},{k[5]},{k[6]}] {k[0][:80]}")
                prev = k[2]


if __name__ == "__main__":
    main()
