#!/usr/bin/env python3
"""HBM traffic per launch of bench.py's roofline kernels, from rocprofv3 PMC counters.

    run:        python tools/roofline_pmc.py run          (the kernels bench.py times, 20 launches each)
    on the box: timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/rpmc_FETCH_SIZE -o run -- python tools/roofline_pmc.py run
                timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/rpmc_WRITE_SIZE -o run -- python tools/roofline_pmc.py run
    summarize:  python tools/roofline_pmc.py summarize gpurun_out > profiles/r01_roofline_pmc.json

FETCH_SIZE on gfx950 counts 1/2 of the bytes of wide streaming reads (MI355X_MICROARCH.md,
HBM section; calibrated here on rmsprop_kernel: 51.6 MB read = 2 x FETCH_SIZE), so fetch is
doubled; WRITE_SIZE is exact for 16-B stores and for float atomics. Separate passes: the
two counters do not fit one TCC pass.
"""
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

_WG = "wgrad_big<4, 2, 4, 4, 64>" if os.environ.get("F3_WGRAD_BIG", "1") != "0" else "wgrad_glds_bf16<128, 128>"
KERNELS = {"wgrad": _WG, "tcn_fwd": "igemm_big<1, 1, 8>"}


def run():
    import torch
    import bench
    r = bench.roofline_kernels(torch.device("cuda"), 256, 18, "bf16")
    print(json.dumps({k: [v["kernel"], v["ms_per_launch"], v["frac"]] for k, v in r.items()}))


def per_launch(db, counter, pattern):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, value from counters_collection where counter_name = ?", (counter,)).fetchall()
    vals = [v * 1024.0 for name, v in rows if pattern in name]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def summarize(d):
    import torch  # noqa: F401  (bench imports torch)
    import bench
    names = {"wgrad": KERNELS["wgrad"].replace(", ", ",") + " (tcn 9x1 weight gradient, C=256, T=8, N=256, V=18)",
             "tcn_fwd": "igemm_big<1,1,8> (tcn 9x1 fwd, C=256, T=8, N=256, V=18)"}
    out = {}
    for key, pat in KERNELS.items():
        f, nf = per_launch(os.path.join(d, "rpmc_FETCH_SIZE", "run_results.db"), "FETCH_SIZE", pat)
        w, nw = per_launch(os.path.join(d, "rpmc_WRITE_SIZE", "run_results.db"), "WRITE_SIZE", pat)
        if f is None or w is None:
            continue
        out[key] = {"kernel": names[key], "fetch_bytes": 2.0 * f, "write_bytes": w,
                    "bytes_per_launch": round(2.0 * f + w), "launches": [nf, nw],
                    "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, mean over launches"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])
