#!/usr/bin/env python3
"""HBM traffic per launch of the RGB branch kernels (bench.py's rgb_branch leg), from the two PMC
passes of tools/gpu_session.sh rgb_pmc (FETCH_SIZE x2 for the gfx950 wide-read correction +
WRITE_SIZE, mean over the launches):
    python tools/rgb_pmc.py gpurun_out > profiles/r04_rgb_pmc.json
"fwd" = rgb_fwd_kernel (+ its feat memset, a fill kernel, not counted: 64 KB); "bwd" =
rgb_bwd_kernel + rgb_colsum_kernel (the backward's two launches)."""
import json
import os
import sqlite3
import sys

PARTS = {"fwd": ["rgb_fwd_kernel"], "bwd": ["rgb_bwd_kernel", "rgb_colsum_kernel"]}


def mean_bytes(db, counter, pat):
    c = sqlite3.connect(db)
    vals = [v * 1024.0 for name, v in c.execute(
        "select kernel_name, value from counters_collection where counter_name = ?", (counter,)) if pat in name]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main(d):
    out = {}
    for key, pats in PARTS.items():
        fetch = write = 0.0
        ok = True
        for p in pats:
            f, nf = mean_bytes(os.path.join(d, "pmc_FETCH_SIZE", "run_results.db"), "FETCH_SIZE", p)
            w, nw = mean_bytes(os.path.join(d, "pmc_WRITE_SIZE", "run_results.db"), "WRITE_SIZE", p)
            if f is None or w is None:
                ok = False
                break
            fetch += 2.0 * f
            write += w
        if ok:
            out[key] = {"kernels": pats, "fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": round(fetch + write),
                        "note": "FETCH_SIZE x2 + WRITE_SIZE per launch (mean), tools/rgb_bench.py under rocprofv3 --pmc"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
