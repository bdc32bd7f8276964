#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 SQLite (rocpd) database: name, calls, total / average
microseconds and share, the same columns as rocprofv3 --stats' kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top N] [--match SUBSTR]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    if name is None:
        raise SystemExit(f"no kernel name column in {cols}")
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        if a.match and a.match not in n:
            continue
        short = re.sub(r"\(.*$", "", n) if n.count("(") else n
        t = agg.setdefault(short, [0, 0.0])
        t[0] += 1
        t[1] += (e - s) / 1e3
    total = sum(v[1] for v in agg.values())
    print(f"{'kernel':<90} {'calls':>6} {'total_us':>12} {'avg_us':>10} {'pct':>6}")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{k[:90]:<90} {n:>6} {us:>12.1f} {us / n:>10.2f} {100 * us / total:>6.2f}")
    print(f"{'TOTAL':<90} {sum(v[0] for v in agg.values()):>6} {total:>12.1f}")


if __name__ == "__main__":
    main()
