#!/usr/bin/env python3
"""Per-kernel HBM traffic from the two PMC passes of tools/gpu_pmc.sh.

    python tools/pmc_summary.py gpurun_out [--fetch-scale 2.0] [--csv out.csv]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reports 1/2 of the
bytes of wide (16 B/lane) streaming reads (MI355X_MICROARCH.md, HBM section); the default
--fetch-scale 2 applies that correction (calibrated in DESIGN.md against kernels of known
traffic). The achieved rate uses the durations recorded in the same PMC runs.
"""
import argparse
import csv
import os
import sqlite3


def load(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, value, duration from counters_collection where counter_name = ?",
                     (counter,)).fetchall()
    by = {}
    for name, v, dur in rows:
        e = by.setdefault(name, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += v * 1024.0
        e[2] += dur
    return by


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--fetch-scale", type=float, default=2.0)
    p.add_argument("--csv")
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    f = load(os.path.join(a.dir, "pmc_FETCH_SIZE", "run_results.db"), "FETCH_SIZE")
    w = load(os.path.join(a.dir, "pmc_WRITE_SIZE", "run_results.db"), "WRITE_SIZE")
    out = []
    for name, (n, fb, fd) in f.items():
        wn, wb, wd = w.get(name, (n, 0.0, fd))
        fetch = fb / n * a.fetch_scale
        write = wb / max(wn, 1)
        dur = (fd / n + wd / max(wn, 1)) / 2.0
        out.append({"kernel": name, "calls": n, "fetch_MB": fetch / 1e6, "write_MB": write / 1e6,
                    "dur_us": dur / 1e3, "GBps": (fetch + write) / max(dur, 1.0),
                    "total_MB": (fetch + write) * n / 1e6})
    out.sort(key=lambda r: -r["total_MB"])
    print(f"{'total MB':>9s} {'calls':>5s} {'fetch MB':>9s} {'write MB':>9s} {'us':>8s} {'GB/s':>7s}  kernel")
    for r in out[: a.top]:
        print(f"{r['total_MB']:9.1f} {r['calls']:5d} {r['fetch_MB']:9.2f} {r['write_MB']:9.2f} {r['dur_us']:8.1f} "
              f"{r['GBps']:7.0f}  {r['kernel'][:90]}")
    if a.csv:
        with open(a.csv, "w", newline="") as fh:
            wr = csv.DictWriter(fh, fieldnames=list(out[0].keys()))
            wr.writeheader()
            wr.writerows(out)


if __name__ == "__main__":
    main()
