#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace database (rocpd SQLite, the default output format)
into per-kernel stats, the same columns as rocprofv3's kernel_stats.csv.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--csv out.csv] [--top 40]
        [--per-step STEPS]   # also print each kernel's time per step (total / STEPS)
"""
import argparse
import csv
import sqlite3
import statistics
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels").fetchall()
    by = {}
    for name, dur, gx, gy, gz, wx in rows:
        by.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in by.values())
    out = []
    for name, d in by.items():
        out.append({"Name": name, "Calls": len(d), "TotalDurationNs": sum(d), "AverageNs": sum(d) / len(d),
                    "Percentage": 100.0 * sum(d) / total, "MinNs": min(d), "MaxNs": max(d),
                    "StdDev": statistics.pstdev(d) if len(d) > 1 else 0.0})
    out.sort(key=lambda r: -r["TotalDurationNs"])
    return out, total


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--csv")
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--per-step", type=int, default=0)
    a = p.parse_args()
    out, total = stats(a.db)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()), quoting=csv.QUOTE_NONNUMERIC)
            w.writeheader()
            w.writerows(out)
    print(f"total kernel time {total / 1e6:.3f} ms over {sum(r['Calls'] for r in out)} dispatches")
    for r in out[: a.top]:
        extra = f"  {r['TotalDurationNs'] / a.per_step / 1e3:9.1f} us/step" if a.per_step else ""
        print(f"{r['Percentage']:6.2f}% {r['Calls']:6d} x {r['AverageNs'] / 1e3:9.2f} us{extra}  {r['Name'][:110]}")


if __name__ == "__main__":
    sys.exit(main())
