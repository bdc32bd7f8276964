#!/usr/bin/env python3
"""Dump the API calls and kernels of a rocprofv3 --hip-trace --kernel-trace database into
two small CSV files (the database itself is too large to bring back from the box).

    python tools/trace_dump.py DB OUTDIR [--last-ms 40]
"""
import csv
import os
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    last = float(sys.argv[4]) if len(sys.argv) > 4 else 40.0
    os.makedirs(out, exist_ok=True)
    c = sqlite3.connect(db)
    t_end = c.execute("select max(end) from kernels").fetchone()[0]
    t0 = t_end - int(last * 1e6)
    with open(os.path.join(out, "kernels.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "start", "end", "queue", "stream", "corr"])
        for r in c.execute("select name, start, end, queue_id, stream_id, corr_id from kernels where start >= ? order by start", (t0,)):
            w.writerow(r)
    with open(os.path.join(out, "api.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "start", "end", "corr", "tid"])
        for r in c.execute("select name, start, end, corr_id, tid from regions where start >= ? order by start", (t0,)):
            w.writerow(r)


if __name__ == "__main__":
    main()
