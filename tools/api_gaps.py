#!/usr/bin/env python3
"""Long host API calls in a rocprofv3 --hip-trace --kernel-trace database: which HIP call
blocks the launching thread (and so starves the queues) during the step.

    python tools/api_gaps.py gpurun_out/hiptr/run_results.db [--min-us 100]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--min-us", type=float, default=100.0)
    p.add_argument("--steps", type=int, default=2)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    ks = c.execute("select name, start, end, queue_id, corr_id from kernels order by start").fetchall()
    kname = {k[4]: k for k in ks}
    ends = [k[2] for k in ks if "rmsprop" in k[0]]
    t0, t1 = ends[-1 - a.steps], ends[-1]
    regs = c.execute("select name, start, end, corr_id, tid from regions where start >= ? and start <= ? order by start",
                     (t0 - 20_000_000, t1)).fetchall()
    tot = defaultdict(lambda: [0, 0.0])
    for n, s, e, corr, tid in regs:
        tot[n][0] += 1
        tot[n][1] += (e - s) / 1e3
    print(f"window {(t1 - t0) / 1e3:.1f} us over {a.steps} steps; API totals (us):")
    for n, (cnt, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {n:40s} {cnt:6d} {us:10.1f}")
    print(f"calls >= {a.min_us} us (start offset from window start):")
    for n, s, e, corr, tid in regs:
        d = (e - s) / 1e3
        if d >= a.min_us and s >= t0:
            k = kname.get(corr)
            extra = f" -> {k[0][:60]} (q{k[3]})" if k else ""
            # what was running on the queues when the call returned
            print(f"  {(s - t0) / 1e3:9.1f} +{d:8.1f} {n}{extra}")


if __name__ == "__main__":
    main()
